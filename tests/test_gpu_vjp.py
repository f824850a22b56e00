"""Reverse mode (cnf_vjp / cnf_loss_vjp) against the reference's own autograd
gradients (golden g5 fixtures) and the numpy oracle's hand-written backward."""
import numpy as np
import pytest
import torch

from _golden import load, names
from _model import build_flow
from cnf_hip import _lib, engine
from cnf_hip import vjp as V
from oracle import cnf_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _grad_err(got, ref):
    sc = float(np.max(np.abs(ref))) + 1e-3
    return float(np.max(np.abs(got - ref))) / sc


@pytest.mark.parametrize("name", names("g5"))
@pytest.mark.parametrize("kind", ["cal", "ce"])
@pytest.mark.parametrize("via_ops", [False, True])
def test_fused_loss_grads_match_reference_autograd(name, kind, via_ops):
    """cnf_loss_vjp through ctypes and through torch.ops.cnf.loss_and_grads.
    g5_grads_d100_l12 is cfg4's full depth (D=100, L=12, [100,100]): the fused
    wide sweeps (k_wtrain16_fwd / k_wtrain16_bwd + k_wdw16g) held to the
    reference's autograd over every layer, no row exemptions."""
    meta, state, d = load(name)
    flow = build_flow(meta, state, DEV)
    stack = flow._native_stack()
    x = torch.from_numpy(d["x"]).to(DEV)
    y = torch.from_numpy(d["y"]).to(DEV)
    B = x.shape[0]
    k = 0 if kind == "cal" else 1
    if via_ops:
        ops = _lib.torch_ops()
        if ops is None:
            pytest.skip("libcnf_torch.so not built")
        terms, grads = ops.loss_and_grads(x, y, stack.prepared(x.device), stack.desc_ints,
                                          stack._perms, k, 1.0, 1.0 / B)
    else:
        terms, grads, _ = V.loss_and_grads(stack, x, y, kind=k, det=1.0, grad_scale=1.0 / B)
    terms = terms.cpu().numpy()
    ref_loss = float(d["loss_" + kind])
    assert abs(terms[0] / B - ref_loss) / (abs(ref_loss) + 1) <= 1e-5
    worst = 0.0
    for (k, p), g in zip([(k, p) for k, p in flow.named_parameters() if p.requires_grad],
                         V._split(stack, grads)):
        worst = max(worst, _grad_err(g.cpu().numpy(), d["g%s:%s" % (kind, k)]))
    assert worst <= 1e-4, worst


@pytest.mark.parametrize("via_ops", [True, False])
def test_autograd_backward_matches_reference(via_ops, monkeypatch):
    monkeypatch.setattr(engine, "USE_TORCH_OPS", via_ops)
    meta, state, d = load("g5_grads_d10")
    flow = build_flow(meta, state, DEV)
    x = torch.from_numpy(d["x"]).to(DEV)
    y = torch.from_numpy(d["y"]).to(DEV)
    n0, t0 = engine.stats["vjp"], engine.stats["torch_ops"]
    zs, ld = flow(x)
    probs = torch.softmax(zs[-1], dim=1)
    ce = torch.log(probs.gather(1, y.view(-1, 1)) + 1e-7)
    loss = -torch.mean(ce.squeeze() + ld)          # calibrators.py:288-291
    flow.zero_grad()
    loss.backward()
    # the backward is cnf_vjp, from Python (ctypes) or from cnf::flow's C++ autograd
    assert engine.stats["vjp"] == n0 + 1 or engine.stats["torch_ops"] == t0 + 1, \
        "native cnf_vjp did not run"
    assert abs(loss.item() - float(d["loss_cal"])) <= 1e-5 * (abs(float(d["loss_cal"])) + 1)
    worst = 0.0
    for k, p in flow.named_parameters():
        if p.requires_grad:
            worst = max(worst, _grad_err(p.grad.cpu().numpy(), d["gcal:" + k]))
    assert worst <= 1e-4, worst


def _flow(D, L, hidden, sigma, seed, scale=True, shift=True, flip=False):
    from flows.flows import Flow, NvpCouplingLayer
    torch.manual_seed(seed)
    np.random.seed(seed)
    f = Flow([NvpCouplingLayer(D, hidden, scale=scale, shift=shift, random_flip=flip)
              for _ in range(L)])
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for p in f.parameters():
            if p.requires_grad:
                p.copy_(torch.randn(p.shape, generator=g) * sigma)
    return f


@pytest.mark.parametrize("D,L,hidden,scale,shift,flip", [
    (10, 6, [5, 5], True, True, False),
    (10, 5, [5, 5], True, True, True),     # odd L, random_flip
    (3, 2, [5, 5], False, True, False),    # NICE
    (10, 3, [5, 5], True, False, False),   # shift=False
    (10, 3, [], True, True, False),
    (10, 3, [7], True, True, False),
    (10, 12, [5, 5], True, True, True),   # L > 8: the layerwise reverse mode (cnf_wvjp.hip)
    # the MFMA family's layer-at-a-time reverse mode (cnf_wvjp.hip)
    (10, 3, [4, 6, 3], True, True, False),
    (20, 3, [24, 16], True, True, True),
    (17, 2, [], True, True, False),        # odd D, no hidden layer
    (24, 2, [30], False, True, False),     # NICE
    (24, 2, [30], True, False, False),     # shift=False
    (100, 2, [100, 100], True, True, False),
    (64, 3, [130], True, True, True),      # > 128 hidden units: two column tiles
    # the fused training sweeps (cnf_wide16.hip: k_wtrain16_fwd / k_wtrain16_bwd)
    (100, 3, [100], True, True, True),     # one hidden layer
    (100, 2, [], True, True, False),       # no hidden layer
    (100, 2, [100, 100], False, True, True),  # NICE
    (32, 3, [64, 64], True, True, True),   # 16-multiple widths: extra ones-column tiles
    (32, 2, [64, 64], False, True, False),
])
def test_vjp_all_outputs_and_dx_against_cpu_autograd(D, L, hidden, scale, shift, flip):
    # wide conditioners at sigma 0.2 overflow exp(s) (the reference's own
    # gradients are NaN there); 0.05 keeps them finite
    f = _flow(D, L, hidden, 0.2 if D <= 24 else 0.05, 3, scale, shift, flip)
    x = torch.randn(777, D, generator=torch.Generator().manual_seed(1))
    w = torch.randn(L, 777, D, generator=torch.Generator().manual_seed(2))
    wl = torch.randn(777, generator=torch.Generator().manual_seed(3))

    def objective(flow, xx):
        zs, ld = flow(xx)
        return sum((z * w[i].to(z.device)).sum() for i, z in enumerate(zs)) + \
            (ld * wl.to(ld.device)).sum()

    xc = x.clone().requires_grad_(True)
    objective(f, xc).backward()
    ref = {k: p.grad.clone() for k, p in f.named_parameters() if p.requires_grad}
    fg = f.to(DEV)
    fg.zero_grad()
    xg = x.to(DEV).requires_grad_(True)
    n0, t0 = engine.stats["vjp"], engine.stats["torch_ops"]
    objective(fg, xg).backward()
    assert engine.stats["vjp"] == n0 + 1 or engine.stats["torch_ops"] == t0 + 1
    for k, p in fg.named_parameters():
        if p.requires_grad:
            assert _grad_err(p.grad.cpu().numpy(), ref[k].numpy()) <= 1e-4, k
    assert _grad_err(xg.grad.cpu().numpy(), xc.grad.numpy()) <= 1e-4


def test_vjp_is_deterministic_and_matches_oracle_at_scale():
    f = _flow(10, 6, [5, 5], 0.1, 4).to(DEV)
    stack = f._native_stack()
    B = 1 << 20
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(B, 10, device=DEV, generator=g)
    y = torch.randint(0, 10, (B,), device=DEV, generator=g)
    t1, g1, _ = V.loss_and_grads(stack, x, y, grad_scale=1.0 / B)
    t2, g2, _ = V.loss_and_grads(stack, x, y, grad_scale=1.0 / B)
    assert torch.equal(g1, g2) and torch.equal(t1, t2), "non-deterministic reduction"
    # the mean over 1M rows equals the mean of per-shard means (linearity), and a
    # 4096-row slice agrees with the numpy oracle
    st = {k: v.cpu().numpy() for k, v in f.state_dict().items()}
    ol = O.layers_from_state(st, 6, 10, 3)
    xs, ys = x[:4096], y[:4096]
    tl, gl, _ = V.loss_and_grads(stack, xs, ys, grad_scale=1.0 / 4096)
    loss, og = O.loss_and_grads(ol, xs.cpu().numpy(), ys.cpu().numpy(), "cal")
    assert abs(tl[0].item() / 4096 - loss) / (abs(loss) + 1) <= 1e-5
    flat = np.concatenate([np.concatenate([np.concatenate([gw.ravel(), gb.ravel()])
                                           for gw, gb in og[l][n]])
                           for l in range(6) for n in ("s", "t")])
    assert _grad_err(gl.cpu().numpy(), flat) <= 1e-4


def test_wide_vjp_is_deterministic_and_matches_oracle():
    """cfg4-shaped stack (D=100, [100,100]) on the MFMA reverse mode: two runs
    bitwise equal over 2^16 rows; a 1024-row slice against the numpy oracle."""
    f = _flow(100, 2, [100, 100], 0.05, 5, flip=True).to(DEV)
    stack = f._native_stack()
    B = 1 << 16
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(B, 100, device=DEV, generator=g) * 3
    y = torch.randint(0, 100, (B,), device=DEV, generator=g)
    t1, g1, _ = V.loss_and_grads(stack, x, y, grad_scale=1.0 / B)
    t2, g2, _ = V.loss_and_grads(stack, x, y, grad_scale=1.0 / B)
    assert torch.equal(g1, g2) and torch.equal(t1, t2), "non-deterministic reduction"
    st = {k: v.cpu().numpy() for k, v in f.state_dict().items()}
    ol = O.layers_from_state(st, 2, 100, 3)
    xs, ys = x[:1024], y[:1024]
    for kind, k in (("cal", 0), ("ce", 1)):
        tl, gl, _ = V.loss_and_grads(stack, xs, ys, kind=k, grad_scale=1.0 / 1024)
        loss, og = O.loss_and_grads(ol, xs.cpu().numpy().astype(np.float64),
                                    ys.cpu().numpy(), kind)
        assert abs(tl[0].item() / 1024 - loss) / (abs(loss) + 1) <= 1e-5
        flat = np.concatenate([np.concatenate([np.concatenate([gw.ravel(), gb.ravel()])
                                               for gw, gb in og[l][n]])
                               for l in range(2) for n in ("s", "t")])
        assert _grad_err(gl.cpu().numpy(), flat) <= 1e-4


@pytest.mark.parametrize("kind", ["cal", "ce"])
@pytest.mark.parametrize("path", ["fused", "layerwise"])
def test_cfg4_depth_grads_and_dx_match_reference(kind, path):
    """g5_grads_d100_l12 (the reference's autograd at cfg4's full depth):
    every parameter gradient AND the input gradient of every row, through the
    fused sweeps (k_wtrain16_fwd / k_wtrain16_bwd + k_wdw16g) and through the
    layer-at-a-time reverse mode (OPT_NO_WIDE) -- no row exemptions."""
    meta, state, d = load("g5_grads_d100_l12")
    flow = build_flow(meta, state, DEV)
    if path == "layerwise":
        flow.native_options = _lib.OPT_NO_WIDE
    stack = flow._native_stack()
    assert stack.kernel_name() == ("mfma-wide" if path == "fused" else "mfma-tile")
    x = torch.from_numpy(d["x"]).to(DEV)
    y = torch.from_numpy(d["y"]).to(DEV)
    B = x.shape[0]
    terms, grads, dx = V.loss_and_grads(stack, x, y, kind=0 if kind == "cal" else 1, det=1.0,
                                        grad_scale=1.0 / B, need_dx=True)
    ref_loss = float(d["loss_" + kind])
    assert abs(terms[0].item() / B - ref_loss) / (abs(ref_loss) + 1) <= 1e-5
    worst = 0.0
    for (k, p), g in zip([(k, p) for k, p in flow.named_parameters() if p.requires_grad],
                         V._split(stack, grads)):
        worst = max(worst, _grad_err(g.cpu().numpy(), d["g%s:%s" % (kind, k)]))
    assert worst <= 1e-4, worst
    assert _grad_err(dx.cpu().numpy(), d["dx" + kind]) <= 1e-4


def _vjp_ws_bytes(stack, B):
    import ctypes
    from cnf_hip import _lib
    n = ctypes.c_size_t()
    assert _lib.lib().cnf_vjp_workspace_bytes(ctypes.byref(stack.desc), ctypes.c_int64(B),
                                              ctypes.byref(n)) == 0
    return n.value


@pytest.mark.parametrize("flip", [False, True])
def test_fused_wide_training_matches_layerwise_path(flip):
    """cfg4's shape (D=100, L=12, [100,100]) at a ragged batch: the fused
    training sweeps (k_wtrain16_*) against the layer-at-a-time reverse mode
    (OPT_NO_WIDE: k_wgemm / k_wfwd_update / k_wbwd_update), both native, on the
    same inputs -- loss terms, every parameter gradient and dx."""
    from cnf_hip import _lib
    f = _flow(100, 12, [100, 100], 0.03, 6, flip=flip).to(DEV)
    B = (1 << 14) + 37
    g = torch.Generator(device=DEV).manual_seed(2)
    x = torch.randn(B, 100, device=DEV, generator=g) * 2
    y = torch.randint(0, 100, (B,), device=DEV, generator=g)
    assert f._native_stack().kernel_name() == "mfma-wide"
    # the fused path's workspace holds the per-row tape of every layer (640
    # floats per row and layer at this shape)
    assert _vjp_ws_bytes(f._native_stack(), B) > 12 * B * 640 * 4
    t1, g1, d1 = V.loss_and_grads(f._native_stack(), x, y, grad_scale=1.0 / B, need_dx=True)
    f.native_options = _lib.OPT_NO_WIDE
    assert f._native_stack().kernel_name() == "mfma-tile"
    t2, g2, d2 = V.loss_and_grads(f._native_stack(), x, y, grad_scale=1.0 / B, need_dx=True)
    assert ((t1 - t2).abs() / (t2.abs() + 1)).max().item() <= 1e-5
    assert _grad_err(g1.cpu().numpy(), g2.cpu().numpy()) <= 1e-4
    # dx row by row: a row whose hidden pre-activation sits within rounding of
    # 0 takes relu' = 0 in one fp32 evaluation order and 1 in the other (both
    # legitimate -- the reference's own fp32 order is a third); such rows are
    # rare (2 in 2^14 here), every other row agrees to 1e-5 of its own scale
    d1, d2 = d1.double(), d2.double()
    rel = (d1 - d2).abs().amax(1) / (d2.abs().amax(1) + 1e-30)
    assert int((rel > 1e-5).sum()) <= max(2, B // 4000), rel.topk(5)
    assert not torch.equal(g1, g2), "both runs took the same path"


@pytest.mark.parametrize("act_scale", [1e-9, 1e-12])
def test_fused_loss_grads_tiny_activations_small_grad_scale(act_scale):
    """k_vjp2 accumulates the hidden columns' weight gradients against
    h' = 2^-64 h and applies the 2^64 once per wave (cnf_vjp2.h): a product
    g * h' falls into the fp32 denormal range when |g h| < 2^-62.  Held to the
    reference's own fp32 autograd where that happens -- grad_scale 2^-23 (a
    2^23-row batch) and hidden activations of ~1e-9 / 1e-12 (products ~1e-16 /
    1e-19 per row) -- at the same 1e-4 bar as every other gradient."""
    from flows.flows import Flow, NvpCouplingLayer
    torch.manual_seed(11)
    f = Flow([NvpCouplingLayer(10, [5, 5]) for _ in range(3)])
    g = torch.Generator().manual_seed(12)
    with torch.no_grad():
        for k, p in f.named_parameters():
            if not p.requires_grad:
                continue
            v = torch.randn(p.shape, generator=g) * 0.3
            if k.endswith("layers.0.weight") or k.endswith("layers.0.bias"):
                v = v.abs() * act_scale if k.endswith("bias") else v * act_scale
            p.copy_(v)
    B = 4096
    x = torch.randn(B, 10, generator=torch.Generator().manual_seed(13))
    y = torch.randint(0, 10, (B,), generator=torch.Generator().manual_seed(14))
    gs = 2.0 ** -23
    xc = x.clone()
    zs, ld = f(xc)
    p_y = torch.softmax(zs[-1], 1).gather(1, y[:, None]).squeeze(1)
    loss = (-(torch.log(p_y + 1e-7) + ld)).sum() * gs   # calibrators.py:288-291, scaled
    loss.backward()
    ref = {k: p.grad.clone() for k, p in f.named_parameters() if p.requires_grad}
    fg = f.to(DEV)
    stack = fg._native_stack()
    terms, grads, _ = V.loss_and_grads(stack, x.to(DEV), y.to(DEV), kind=0, det=1.0,
                                       grad_scale=gs)
    worst, where = 0.0, None
    for (k, p), gg in zip([(k, p) for k, p in fg.named_parameters() if p.requires_grad],
                          V._split(stack, grads)):
        a, b = gg.cpu().numpy(), ref[k].numpy()
        # relative to the tensor's own scale (no absolute floor: these
        # gradients are ~1e-16 and smaller)
        e = float(np.max(np.abs(a - b))) / max(float(np.max(np.abs(b))), 1e-37)
        if e > worst:
            worst, where = e, k
    assert worst <= 1e-4, (worst, where)
