"""Native reverse mode of strict_nan stacks (cnf_desc.strict_nan, the
reference's inf * 0 = NaN at masked positions, flows/flows.py:101-112): the
layer-at-a-time kernels of cnf_wvjp.hip follow torch autograd's rules for the
reference's op sequence over every feature.  Gradients must match CPU autograd
of the reference's own ops, NaN / inf positions included, through the
cnf::flow operator (C++ autograd), through ctypes (cnf_vjp) and through the
fused loss (cnf_loss_vjp)."""
import numpy as np
import pytest
import torch

from _golden import load
from _model import build_flow
from cnf_hip import _lib, engine
from cnf_hip import vjp as V

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _same(got, ref, name):
    got, ref = got.detach().cpu().double(), ref.detach().cpu().double()
    assert got.shape == ref.shape, name
    assert torch.equal(torch.isnan(got), torch.isnan(ref)), (name, torch.isnan(got).sum().item(),
                                                             torch.isnan(ref).sum().item())
    assert torch.equal(torch.isinf(got), torch.isinf(ref)), name
    fin = torch.isfinite(ref)
    if fin.any():
        scale = ref[fin].abs().max().item() + 1e-30
        assert (got[fin] - ref[fin]).abs().max().item() <= 1e-4 * scale + 1e-7, name


def _case(kind):
    """(flow state, x, y): the g6_d4_nan fixture (masked exp(s) = inf in every
    row) or a variant where only some rows overflow."""
    meta, state, d = load("g6_d4_nan")
    x = torch.from_numpy(d["x"])
    y = torch.from_numpy(d["y"])
    if kind == "some_rows":
        # s at the masked feature = 200 (w . h) + 88: exp(s) overflows in the rows
        # where w . h > 0.0036 (37 of the 64 at x * 8), the others stay finite
        state = dict(state)
        b = np.array(state["layers.0.s.layers.1.bias"], copy=True)
        w = np.array(state["layers.0.s.layers.1.weight"], copy=True)
        b[-1] = 88.0
        w[-1] *= 200.0
        state["layers.0.s.layers.1.bias"] = b
        state["layers.0.s.layers.1.weight"] = w
        x = x * 8.0
    return meta, state, x, y


def _cpu_grads(meta, state, x, y, objective):
    f = build_flow(meta, state, "cpu", strict_nan=True)
    xx = x.clone().requires_grad_(True)
    out = objective(f, xx, y)
    ps = [p for p in f.parameters() if p.requires_grad]
    gs = torch.autograd.grad(out, ps + [xx], allow_unused=True)
    return out.detach(), [torch.zeros_like(p) if g is None else g for g, p in zip(gs, ps + [xx])]


def _loss(f, x, y):
    z, ld = f.transform(x)
    p = torch.softmax(z, 1).gather(1, y.view(-1, 1)).squeeze(1)
    return -torch.mean(torch.log(p + 1e-7) + ld)


def _zs_objective(f, x, y):
    # gradient through every layer output (the zs list) and the log-det
    zs, ld = f(x)
    w = torch.arange(1, x.shape[1] + 1, dtype=x.dtype, device=x.device)
    return sum(((z * w).sum() for z in zs), torch.zeros((), device=x.device)) + 0.5 * ld.sum()


@pytest.mark.parametrize("kind", ["fixture", "some_rows"])
@pytest.mark.parametrize("objective", ["loss", "zs"])
@pytest.mark.parametrize("via_ops", [True, False])
def test_strict_vjp_matches_cpu_autograd(kind, objective, via_ops, monkeypatch):
    monkeypatch.setattr(engine, "USE_TORCH_OPS", via_ops)
    meta, state, x, y = _case(kind)
    obj = _loss if objective == "loss" else _zs_objective
    ref_out, ref = _cpu_grads(meta, state, x, y, obj)
    f = build_flow(meta, state, DEV, strict_nan=True)
    assert f._native_stack().has_native_vjp(), "strict stacks must have a native reverse mode"
    xx = x.to(DEV).requires_grad_(True)
    n0 = engine.stats["vjp"]
    out = obj(f, xx, y.to(DEV))
    ps = [p for p in f.parameters() if p.requires_grad]
    got = torch.autograd.grad(out, ps + [xx], allow_unused=True)
    torch.cuda.synchronize()
    if not via_ops:
        assert engine.stats["vjp"] > n0, "native cnf_vjp did not run"
    if kind == "some_rows":  # the case must really mix NaN and finite rows
        assert torch.isnan(ref[-1]).any(1).any() and not torch.isnan(ref[-1]).any(1).all()
    _same(out, ref_out, "objective")
    for i, (g, r) in enumerate(zip(got, ref)):
        _same(torch.zeros_like(r) if g is None else g, r, "grad %d" % i)


@pytest.mark.parametrize("kind", ["fixture", "some_rows"])
def test_strict_fused_loss_vjp_matches_cpu_autograd(kind):
    meta, state, x, y = _case(kind)
    ref_out, ref = _cpu_grads(meta, state, x, y, _loss)
    f = build_flow(meta, state, DEV, strict_nan=True)
    stack = f._native_stack()
    B = x.shape[0]
    terms, grads, dx = V.loss_and_grads(stack, x.to(DEV), y.to(DEV), grad_scale=1.0 / B,
                                        need_dx=True)
    flat = torch.cat([g.reshape(-1) for g in ref[:-1]])
    _same(grads, flat, "grads")
    _same(dx, ref[-1], "dx")
    _same(terms[0] / B, ref_out, "loss")


def _inv_case(kind):
    """(flow state, z) for the strict INVERSE: the g6_d4_nan stack on a
    random logit batch, or a variant where exp(-s) overflows at a masked
    feature in some rows only (s = -200 (w . h) - 88 there), so that
    b_1 (z - t) e^{-s} = 0 * inf = NaN in those rows (flows/flows.py:123)."""
    meta, state, d = load("g6_d4_nan")
    z = torch.from_numpy(d["x"])
    if kind == "neg_rows":
        state = dict(state)
        b = np.array(state["layers.0.s.layers.1.bias"], copy=True)
        w = np.array(state["layers.0.s.layers.1.weight"], copy=True)
        b[-1] = -88.0
        w[-1] *= -200.0
        state["layers.0.s.layers.1.bias"] = b
        state["layers.0.s.layers.1.weight"] = w
        z = z * 8.0
    return meta, state, z


def _inv_xs_objective(f, z):
    # gradient through every step's output (the xs list) and the log-det
    xs, ld = f.backward(z)
    w = torch.arange(1, z.shape[1] + 1, dtype=z.dtype, device=z.device)
    return sum(((x * w).sum() for x in xs), torch.zeros((), device=z.device)) + 0.5 * ld.sum()


def _inv_final_objective(f, z):
    x, ld = f.inverse_transform(z)
    w = torch.arange(1, z.shape[1] + 1, dtype=z.dtype, device=z.device)
    return (x * w).sum() - 0.25 * ld.sum()


@pytest.mark.parametrize("kind", ["fixture", "neg_rows"])
@pytest.mark.parametrize("objective", ["xs", "final"])
@pytest.mark.parametrize("via_ops", [True, False])
def test_strict_inverse_vjp_matches_cpu_autograd(kind, objective, via_ops, monkeypatch):
    """Autograd through the strict INVERSE (Flow.backward, flows/flows.py:
    114-126) runs cnf_vjp_inverse natively -- through cnf::inverse_flow and
    through ctypes -- and matches CPU autograd of the reference's own ops,
    NaN / inf positions included."""
    monkeypatch.setattr(engine, "USE_TORCH_OPS", via_ops)
    meta, state, z = _inv_case(kind)
    obj = _inv_xs_objective if objective == "xs" else _inv_final_objective
    f_cpu = build_flow(meta, state, "cpu", strict_nan=True)
    zc = z.clone().requires_grad_(True)
    ref_out = obj(f_cpu, zc)
    ps_cpu = [p for p in f_cpu.parameters() if p.requires_grad]
    ref = torch.autograd.grad(ref_out, ps_cpu + [zc], allow_unused=True)
    ref = [torch.zeros_like(p) if g is None else g for g, p in zip(ref, ps_cpu + [zc])]
    f = build_flow(meta, state, DEV, strict_nan=True)
    assert f._native_stack().has_native_vjp_inverse(), "strict stacks: native inverse reverse mode"
    zz = z.to(DEV).requires_grad_(True)
    n0, i0 = engine.stats["vjp"], engine.stats["inverse"]
    out = obj(f, zz)
    ps = [p for p in f.parameters() if p.requires_grad]
    got = torch.autograd.grad(out, ps + [zz], allow_unused=True)
    torch.cuda.synchronize()
    assert engine.stats["inverse"] > i0, "native cnf_inverse did not run"
    if not via_ops:
        assert engine.stats["vjp"] > n0, "native cnf_vjp_inverse did not run"
    if kind == "neg_rows":  # the case must really mix NaN and finite rows
        assert torch.isnan(ref[-1]).any(1).any() and not torch.isnan(ref[-1]).any(1).all()
    _same(out, ref_out.detach(), "objective")
    for k, (g, r) in enumerate(zip(got, ref)):
        _same(torch.zeros_like(r) if g is None else g, r, "grad %d" % k)


def test_strict_inverse_workspace_is_reported():
    """The ABI serves the strict inverse's reverse mode (it reported
    CNF_ERR_UNSUPPORTED before round 5)."""
    meta, state, _ = _inv_case("fixture")
    f = build_flow(meta, state, DEV, strict_nan=True)
    import ctypes
    n = ctypes.c_size_t()
    st = _lib.lib().cnf_vjp_inverse_workspace_bytes(ctypes.byref(f._native_stack().desc),
                                                    ctypes.c_int64(4), ctypes.byref(n))
    assert st == 0 and n.value > 0


# Strict stacks off the D=4 fixture's narrow path: the MFMA-tile
# family's strict geometry (Op = r8(D), Cp = r8(D+1), the zero columns of the
# coupling epilogues) serves wide D, odd D, shift-only (NICE) and random_flip
# stacks.  Synthetic weights N(0, 0.3) (0.05 at D=40); where the stack has an s-net, layer
# 0's s-net is pushed to overflow exp(s) at its last output in about half of
# the rows (inputs x 8), so NaN / inf and finite rows mix.
_SYN = {
    "wide_d40": dict(D=40, hidden=[64], L=3, scale=True, shift=True, random_flip=False),
    "odd_d7": dict(D=7, hidden=[5, 5], L=3, scale=True, shift=True, random_flip=False),
    "nice_d10": dict(D=10, hidden=[5, 5], L=3, scale=False, shift=True, random_flip=False),
    "flip_d10": dict(D=10, hidden=[5, 5], L=3, scale=True, shift=True, random_flip=True),
}


def _syn_case(name, B=96):
    meta = dict(_SYN[name], seed=11)
    np.random.seed(meta["seed"])
    torch.manual_seed(0)
    from flows.flows import Flow, NvpCouplingLayer
    f = Flow([NvpCouplingLayer(meta["D"], list(meta["hidden"]), scale=meta["scale"],
                               shift=meta["shift"], random_flip=meta["random_flip"])
              for _ in range(meta["L"])])
    g = torch.Generator().manual_seed(5)
    state = {}
    for k, v in f.state_dict().items():
        v = v.clone()
        if v.dtype.is_floating_point and ("weight" in k or "bias" in k):
            v = torch.randn(v.shape, generator=g) * (0.3 if meta["D"] <= 16 else 0.05)
        state[k] = v.numpy()
    x = torch.randn(B, meta["D"], generator=g) * 8.0
    y = torch.randint(0, meta["D"], (B,), generator=g)
    if meta["scale"]:
        # the last s output's pre-activation u = w . h + b over the batch (h: the
        # input of layer 0's last s Linear), rescaled so that u > 89 (fp32 exp
        # overflows above 88.72) in about half of the rows
        wk = [k for k in state if k.startswith("layers.0.s.") and k.endswith("weight")][-1]
        bk = wk[:-len("weight")] + "bias"
        ff = build_flow(meta, state, "cpu")
        last = [m for m in ff.layers[0].s.modules() if isinstance(m, torch.nn.Linear)][-1]
        got = {}
        def keep_input(m, i, o):
            got.setdefault("h", i[0].detach())  # (returns None: the output stays)
        hk = last.register_forward_hook(keep_input)
        with torch.no_grad():
            ff(x)
        hk.remove()
        u = got["h"] @ torch.from_numpy(state[wk][-1]).float()
        a = 40.0 / (float(u.std()) + 1e-6)
        state[wk] = state[wk].copy()
        state[bk] = state[bk].copy()
        state[wk][-1] *= a
        state[bk][-1] = 89.0 - a * float(u.median())
    return meta, state, x, y


@pytest.mark.parametrize("name", sorted(_SYN))
@pytest.mark.parametrize("objective", ["loss", "zs"])
def test_strict_vjp_off_the_narrow_path(name, objective):
    meta, state, x, y = _syn_case(name)
    obj = _loss if objective == "loss" else _zs_objective
    ref_out, ref = _cpu_grads(meta, state, x, y, obj)
    f = build_flow(meta, state, DEV, strict_nan=True)
    assert f._native_stack().has_native_vjp(), "strict stacks must have a native reverse mode"
    xx = x.to(DEV).requires_grad_(True)
    n0 = engine.stats["vjp"]
    out = obj(f, xx, y.to(DEV))
    ps = [p for p in f.parameters() if p.requires_grad]
    got = torch.autograd.grad(out, ps + [xx], allow_unused=True)
    torch.cuda.synchronize()
    if not engine.USE_TORCH_OPS:
        assert engine.stats["vjp"] > n0, "native cnf_vjp did not run"
    if meta["scale"] and objective == "zs":  # the case must mix NaN / inf and finite rows
        bad = ~torch.isfinite(ref[-1]).all(1)
        assert bad.any() and not bad.all(), (name, int(bad.sum()))
    _same(out, ref_out, "objective")
    for i, (gg, r) in enumerate(zip(got, ref)):
        _same(torch.zeros_like(r) if gg is None else gg, r, "grad %d" % i)


def _syn_inv_case(name, B=96):
    """_syn_case for the INVERSE: the inverse runs the last layer
    first, so that layer's s-net is pushed instead -- its last output below
    -89 in about half of the rows, where exp(-s) overflows and the masked
    features read 0 * inf = NaN (flows/flows.py:123), the other rows finite."""
    meta, state, x, _ = _syn_case(name, B)
    z = x / 8.0
    if meta["scale"]:
        L = meta["L"]
        pre = "layers.%d.s." % (L - 1)
        wk = [k for k in state if k.startswith(pre) and k.endswith("weight")][-1]
        bk = wk[:-len("weight")] + "bias"
        ff = build_flow(meta, state, "cpu")
        last = [m for m in ff.layers[L - 1].s.modules() if isinstance(m, torch.nn.Linear)][-1]
        got = {}
        def keep_input(m, i, o):
            got.setdefault("h", i[0].detach())
        hk = last.register_forward_hook(keep_input)
        with torch.no_grad():
            ff.layers[L - 1].backward(z)  # the inverse's first step (flows/flows.py:114-126)
        hk.remove()
        u = got["h"] @ torch.from_numpy(state[wk][-1]).float()
        a = 40.0 / (float(u.std()) + 1e-6)
        state[wk] = state[wk].copy()
        state[bk] = state[bk].copy()
        state[wk][-1] *= a
        state[bk][-1] = -89.0 - a * float(u.median())
    return meta, state, z


@pytest.mark.parametrize("name", sorted(_SYN))
def test_strict_inverse_vjp_off_the_narrow_path(name):
    meta, state, z = _syn_inv_case(name)
    f_cpu = build_flow(meta, state, "cpu", strict_nan=True)
    zc = z.clone().requires_grad_(True)
    ref_out = _inv_xs_objective(f_cpu, zc)
    ps_cpu = [p for p in f_cpu.parameters() if p.requires_grad]
    ref = torch.autograd.grad(ref_out, ps_cpu + [zc], allow_unused=True)
    ref = [torch.zeros_like(p) if g is None else g for g, p in zip(ref, ps_cpu + [zc])]
    f = build_flow(meta, state, DEV, strict_nan=True)
    assert f._native_stack().has_native_vjp_inverse()
    zz = z.to(DEV).requires_grad_(True)
    out = _inv_xs_objective(f, zz)
    ps = [p for p in f.parameters() if p.requires_grad]
    got = torch.autograd.grad(out, ps + [zz], allow_unused=True)
    torch.cuda.synchronize()
    if meta["scale"]:  # the case must mix NaN / inf and finite rows
        bad = ~torch.isfinite(ref[-1]).all(1)
        assert bad.any() and not bad.all(), (name, int(bad.sum()))
    _same(out, ref_out.detach(), "objective")
    for k, (g, r) in enumerate(zip(got, ref)):
        _same(torch.zeros_like(r) if g is None else g, r, "grad %d" % k)
