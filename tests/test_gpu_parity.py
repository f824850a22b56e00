"""Parity of the HIP path (through the C ABI) with the reference.

Small cases: against the golden fixtures (outputs of the reference's own
flows/flows.py).  Full BASELINE sizes: against the numpy oracle on sampled rows
plus size-independent properties (round trip, log-det antisymmetry,
determinism, final-only == all-layers).  Tolerance: the north_star's 1e-5 under
SURVEY 8(c)'s metric max|a-b|/(|ref|+1).
"""
import numpy as np
import pytest
import torch

from _golden import load, names, rel_err
from _model import build_flow
from cnf_hip import engine
from flows.flows import Flow, NvpCouplingLayer
from oracle import cnf_oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-5
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    yield


def _oracle_layers(flow):
    l0 = flow.layers[0]
    st = {k: v.detach().cpu().numpy() for k, v in flow.state_dict().items()}
    return O.layers_from_state(st, len(flow.layers), l0.dim, len(l0.hidden_size) + 1,
                               l0.scale, l0.shift)


CASES = [n for n in names() if not n.startswith("g5")]


@pytest.mark.parametrize("name", CASES)
def test_forward_matches_reference_fixture(name):
    meta, state, d = load(name)
    strict = name == "g6_d4_nan"
    flow = build_flow(meta, state, DEV, strict_nan=strict)
    x = torch.from_numpy(d["x"]).to(DEV)
    n0 = engine.stats["forward"]
    with torch.no_grad():
        zs, ld = flow(x)
    torch.cuda.synchronize()
    assert engine.stats["forward"] == n0 + 1, "native cnf_forward did not run"
    assert len(zs) == meta["L"]
    assert rel_err(torch.stack(zs).cpu().numpy(), d["zs"]) <= TOL
    assert tuple(ld.shape) == d["ld"].shape
    assert rel_err(ld.cpu().numpy(), d["ld"]) <= TOL
    with torch.no_grad():
        z, ld2 = flow.transform(x)
    # final-only launches may run a different kernel (cnf_sgpr.hip: log2(e)
    # folded into the s-net) than the every-layer launch: same result to fp32
    # rounding, and both are held to the fixture above
    assert rel_err(z.cpu().numpy(), d["zs"][-1]) <= TOL
    assert rel_err(ld2.cpu().numpy(), d["ld"]) <= TOL
    assert rel_err(z.cpu().numpy(), zs[-1].cpu().numpy()) <= TOL
    assert rel_err(ld2.cpu().numpy(), ld.cpu().numpy()) <= TOL


@pytest.mark.parametrize("name", [n for n in CASES if n != "g6_d4_nan"])
def test_inverse_matches_reference_fixture(name):
    meta, state, d = load(name)
    if "inv_xs" not in d:
        pytest.skip("no inverse recorded")
    flow = build_flow(meta, state, DEV)
    z = torch.from_numpy(d["zs"][-1]).to(DEV)
    n0 = engine.stats["inverse"]
    with torch.no_grad():
        xs, ld = flow.backward(z)
    assert engine.stats["inverse"] == n0 + 1, "native cnf_inverse did not run"
    got = torch.stack(xs).cpu().numpy()
    if d["inv_xs"].shape[0] == 1:
        got = got[-1:]
    _check_inverse(name, "every-layer", got, d["inv_xs"], ld.cpu().numpy(), d["inv_ld"],
                   meta, state, d)


def _inverse64(meta, state, d):
    """The exact (fp64 numpy oracle) inverse of the fixture's z: every step's x."""
    ly = O.cast_layers(O.layers_from_state(state, meta["L"], meta["D"],
                                           len(meta["hidden"]) + 1, meta["scale"],
                                           meta["shift"]), np.float64)
    xs64, _ = O.flow_inverse(ly, d["zs"][-1].astype(np.float64))
    return xs64


def _fp32_floor(meta, state, d):
    """The reference's own fp32-vs-fp64 error on this inverse."""
    return rel_err(d["inv_xs"][-1], _inverse64(meta, state, d)[-1])


def _oracle32_err(meta, state, d):
    """The numpy oracle's own fp32 inverse against the fixture (the CPU
    restatement's error on the same case)."""
    ly = O.layers_from_state(state, meta["L"], meta["D"], len(meta["hidden"]) + 1,
                             meta["scale"], meta["shift"])
    xs32, _ = O.flow_inverse(ly, d["zs"][-1].astype(np.float32))
    return rel_err(np.asarray(xs32[-1], dtype=np.float32), d["inv_xs"][-1])


# Fixtures whose inverse is ill-conditioned in fp32 (exp(-s) up to e^7): the
# reference's own fp32 result sits this far from its fp64 value, so the GPU is
# held to twice that instead of the flat 1e-5 (DESIGN.md section 5 lists the
# measured numbers).  Every other fixture is held to 1e-5.
RELAXED_INVERSE = {"g6_d10_h0"}


def _check_inverse(name, path, got_x, ref_x, got_ld, ref_ld, meta, state, d):
    """Record the GPU inverse error beside the reference's fp32-vs-fp64 error
    and the oracle's fp32 error (conftest RECORDS -> inverse_errors.jsonl),
    then hold it to 1e-5, or to 2x the reference's own error for the fixtures
    in RELAXED_INVERSE."""
    import conftest
    e_x, e_ld = rel_err(got_x, ref_x), rel_err(got_ld, ref_ld)
    x64 = _inverse64(meta, state, d)[-1]
    floor = rel_err(d["inv_xs"][-1], x64)
    final = np.asarray(got_x)[-1] if np.asarray(got_x).ndim == 3 else np.asarray(got_x)
    gpu64 = rel_err(final, x64)
    conftest.RECORDS.setdefault("inverse_errors", []).append(
        {"fixture": name, "path": path, "gpu_err_x": e_x, "gpu_err_ld": e_ld,
         "ref_fp32_vs_fp64": floor, "gpu_vs_fp64": gpu64,
         "oracle_fp32_err": _oracle32_err(meta, state, d)})
    if name in RELAXED_INVERSE:
        # held to twice the reference's own error, against the fixture AND
        # against the exact answer
        assert e_x <= max(TOL, 2 * floor) and gpu64 <= max(TOL, 2 * floor), (name, path, e_x,
                                                                             gpu64, floor)
    else:
        assert e_x <= TOL, (name, path, e_x, floor)
    assert e_ld <= TOL if name not in RELAXED_INVERSE else e_ld <= max(TOL, 2 * floor)


def test_fast_mode_on_overflow_case_differs_only_at_reference_nans():
    meta, state, d = load("g6_d4_nan")
    flow = build_flow(meta, state, DEV, strict_nan=False)
    with torch.no_grad():
        zs, ld = flow(torch.from_numpy(d["x"]).to(DEV))
    got = torch.stack(zs).cpu().numpy()
    ok = ~np.isnan(d["zs"])
    assert np.isnan(d["zs"]).any()
    assert rel_err(got[ok], d["zs"][ok]) <= TOL


def test_single_layer_calls_are_native():
    meta, state, d = load("g2_nvp_d10_n01")
    flow = build_flow(meta, state, DEV)
    x = torch.from_numpy(d["x"]).to(DEV)
    n0 = engine.stats["forward"]
    with torch.no_grad():
        z1, ld1 = flow.layers[0](x)
        xb, ldb = flow.layers[0].backward(z1)
    assert engine.stats["forward"] == n0 + 1
    assert rel_err(z1.cpu().numpy(), d["zs"][0]) <= TOL
    assert rel_err(xb.cpu().numpy(), d["x"]) <= TOL
    assert torch.allclose(ldb, -ld1, atol=1e-6)


def _make_flow(D, L, hidden, sigma, seed, random_flip=False, scale=True):
    torch.manual_seed(seed)
    np.random.seed(seed)
    f = Flow([NvpCouplingLayer(D, hidden, scale=scale, random_flip=random_flip)
              for _ in range(L)])
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for p in f.parameters():
            if p.requires_grad:
                p.copy_(torch.randn(p.shape, generator=g) * sigma)
    return f.to(DEV)


def _logits(B, D, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.randn(B, D, device=DEV, generator=g)
    y = torch.randint(0, D, (B,), device=DEV, generator=g)
    x[torch.arange(B, device=DEV), y] += 2.0
    return x - x.mean(dim=1, keepdim=True)


@pytest.mark.parametrize("D,L,hidden,B,sigma,flip", [
    (10, 6, [5, 5], 1 << 20, 0.1, False),        # cfg2 / cfg5 at full size
    (10, 6, [5, 5], 1 << 23, 0.1, False),        # 8M rows: many tiles per persistent block
    (10, 6, [5, 5], 1000003, 0.2, True),         # ragged batch, random_flip
    (3, 2, [5, 5], 1 << 20, 0.2, False),         # cfg1 shape, RealNVP
    (100, 12, [100, 100], 1 << 16, 0.03, False), # cfg4
])
def test_full_size_properties(D, L, hidden, B, sigma, flip):
    flow = _make_flow(D, L, hidden, sigma, 5, random_flip=flip)
    x = _logits(B, D, 7)
    with torch.no_grad():
        z, ld = flow.transform(x)
        z2, ld2 = flow.transform(x)
        xr, ild = flow.inverse_transform(z)
    assert torch.equal(z, z2) and torch.equal(ld, ld2), "non-deterministic"
    err = ((xr - x).abs() / (x.abs() + 1)).max().item()
    assert err <= TOL, err
    assert ((ild + ld).abs() / (ld.abs() + 1)).max().item() <= TOL
    # sampled rows against the numpy oracle
    idx = torch.randperm(B, generator=torch.Generator().manual_seed(1))[:2048].to(DEV)
    xs = x[idx].cpu().numpy()
    ol = _oracle_layers(flow)
    if flip:
        for l, ly in enumerate(flow.layers):
            ol[l] = O.OracleLayer(D, ol[l].s_net, ol[l].t_net, ly.perm.reshape(-1).cpu().numpy())
    ozs, old = O.flow_forward(ol, xs)
    assert rel_err(z[idx].cpu().numpy(), ozs[-1]) <= TOL
    assert rel_err(ld[idx].cpu().numpy(), old) <= TOL


def test_edge_batches():
    flow = _make_flow(10, 6, [5, 5], 0.2, 3)
    for B in (0, 1, 2, 63, 255, 257):
        x = _logits(max(B, 1), 10, B)[:B]
        with torch.no_grad():
            zs, ld = flow(x)
        ol = _oracle_layers(flow)
        ozs, old = O.flow_forward(ol, x.cpu().numpy())
        assert rel_err(torch.stack(zs).cpu().numpy(), np.stack(ozs)) <= TOL
        assert ld.shape == (torch.Size([]) if B == 1 else torch.Size([B]))


def test_nonaligned_input_view():
    flow = _make_flow(10, 6, [5, 5], 0.2, 4)
    big = _logits(4097, 10, 2)
    x = big.view(-1)[3:3 + 4096 * 10].view(4096, 10)   # 12-byte offset: scalar I/O path
    with torch.no_grad():
        z, ld = flow.transform(x)
    ozs, old = O.flow_forward(_oracle_layers(flow), x.cpu().numpy())
    assert rel_err(z.cpu().numpy(), ozs[-1]) <= TOL


@pytest.mark.parametrize("kind", [0, 1])
def test_fused_forward_loss_matches_oracle(kind):
    flow = _make_flow(10, 6, [5, 5], 0.1, 9)
    stack = flow._native_stack()
    # 2^20 and 1310720 rows: 8 / 10 tiles per SIMD, which the grid runs on 4 / 5
    # waves per SIMD instead of 6 (cnf_sgpr.hip grid_for); 2^23 + 77 on all 6
    for B in (1, 1000, 1 << 20, 1310720, (1 << 23) + 77):
        x = _logits(B, 10, 11)
        y = torch.randint(0, 10, (B,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(5))
        terms, z, ld = stack.forward_loss(x, y, kind=kind, det=0.5, want_outputs=True)
        with torch.no_grad():
            z2, ld2 = flow.transform(x)
        assert torch.equal(z, z2) and torch.equal(ld, ld2.reshape(-1))
        lsm = torch.log_softmax(z.double(), dim=1)
        lpy = lsm.gather(1, y.view(-1, 1)).squeeze(1)
        ce = -torch.log(torch.exp(lpy) + 1e-7) if kind == 0 else -lpy
        loss = ce - (1.0 if kind == 0 else 0.5) * ld.double()
        ref = torch.stack([loss.sum(), ce.sum(), ld.double().sum()]).cpu().numpy()
        got = terms.double().cpu().numpy()
        assert np.all(np.abs(got - ref) <= 1e-5 * (np.abs(ref) + B)), (got, ref)
        t2, _, _ = stack.forward_loss(x, y, kind=kind, det=0.5)
        assert torch.equal(terms, t2), "non-deterministic reduction"


@pytest.mark.parametrize("D,L,hidden,flip,scale", [
    (100, 12, [100, 100], True, True),   # cfg4 shape with random_flip permutations
    (100, 4, [100], False, True),        # one hidden layer
    (100, 3, [], False, False),          # NICE, no hidden layer
    (32, 4, [64, 64], True, True),       # mid width, one partial state tile
])
def test_wide_kernel_matches_oracle_and_tile(D, L, hidden, flip, scale):
    """k_wide16 (cnf_wide16.hip, 16x16x4 register tiles): register-resident
    MFMA path against the numpy oracle, the round trip, and the LDS-tile
    kernel (k_tile) it replaces."""
    flow = _make_flow(D, L, hidden, 0.05, 21, random_flip=flip, scale=scale)
    assert flow._native_stack().kernel_name() == "mfma-wide"
    x = _logits(1000, D, 3)                     # ragged: 31 full waves + 8 rows
    with torch.no_grad():
        z, ld = flow.transform(x)
        xr, ild = flow.inverse_transform(z)
    ol = _oracle_layers(flow)
    if flip:
        for l, ly in enumerate(flow.layers):
            ol[l] = O.OracleLayer(D, ol[l].s_net, ol[l].t_net, ly.perm.reshape(-1).cpu().numpy())
    ozs, old = O.flow_forward(ol, x.cpu().numpy())
    assert rel_err(z.cpu().numpy(), ozs[-1]) <= TOL
    assert rel_err(ld.cpu().numpy(), old) <= TOL
    assert ((xr - x).abs() / (x.abs() + 1)).max().item() <= TOL
    assert ((ild + ld).abs() / (ld.abs() + 1)).max().item() <= TOL
    from cnf_hip import _lib
    flow.native_options = _lib.OPT_NO_WIDE        # the k_tile path
    assert flow._native_stack().kernel_name() == "mfma-tile"
    with torch.no_grad():
        zt, ldt = flow.transform(x)
    assert rel_err(z.cpu().numpy(), zt.cpu().numpy()) <= TOL
    assert rel_err(ld.cpu().numpy(), ldt.cpu().numpy()) <= TOL


@pytest.mark.parametrize("D,L,hidden", [(100, 2, [100, 100]), (32, 3, [64, 64])])
@pytest.mark.parametrize("B", [1, 40, 900])
def test_wide_kernel_partial_blocks(D, L, hidden, B):
    """k_wide16's last block with waves wholly past the batch (B = 900: one
    wave of 4 rows, three with none; B = 1, 40: the only block): those waves
    still take part in the block's LDS copies of the A stream and write
    nothing.  Forward / inverse against the oracle, predict against the
    reference formula (calibrators.py:40-44)."""
    flow = _make_flow(D, L, hidden, 0.05, 5, random_flip=True, scale=True)
    stack = flow._native_stack()
    assert stack.kernel_name() == "mfma-wide"
    x = _logits(B, D, 11)
    with torch.no_grad():
        z, ld = flow.transform(x)
        xr, ild = flow.inverse_transform(z)
    ol = _oracle_layers(flow)
    for l, ly in enumerate(flow.layers):
        ol[l] = O.OracleLayer(D, ol[l].s_net, ol[l].t_net, ly.perm.reshape(-1).cpu().numpy())
    ozs, old = O.flow_forward(ol, x.cpu().numpy())
    assert rel_err(z.cpu().numpy(), ozs[-1]) <= TOL
    # (the reference's log-det squeezes to 0-d at B = 1)
    assert rel_err(ld.reshape(-1).cpu().numpy(), old.reshape(-1)) <= TOL
    assert ((xr - x).abs() / (x.abs() + 1)).max().item() <= TOL
    lp = torch.log_softmax(torch.randn(D, device=x.device), 0)
    n0 = engine.stats["predict"]
    probs = stack.predict(x, lp)
    assert engine.stats["predict"] == n0 + 1  # the fused launch, not the fallback
    with torch.no_grad():
        zc, _ = flow.transform(x - x.mean(dim=1, keepdim=True))
    ref = torch.softmax(torch.log(torch.softmax(zc, 1) + 1e-7) - lp, 1)
    assert (probs - ref).abs().max().item() <= TOL


@pytest.mark.parametrize("name", [n for n in CASES if n != "g6_d4_nan"])
def test_final_only_inverse_matches_reference_fixture(name):
    """inverse_transform (final x and log-det only -- the cfg5 launch, k_sgpr
    for the narrow shapes) against the reference's Flow.backward fixture
    (flows/flows.py:27-37, 114-126)."""
    meta, state, d = load(name)
    if "inv_xs" not in d:
        pytest.skip("no inverse recorded")
    flow = build_flow(meta, state, DEV)
    z = torch.from_numpy(d["zs"][-1]).to(DEV)
    n0 = engine.stats["inverse"]
    with torch.no_grad():
        x, ld = flow.inverse_transform(z)
    assert engine.stats["inverse"] == n0 + 1, "native cnf_inverse did not run"
    assert tuple(ld.shape) == d["inv_ld"].shape
    _check_inverse(name, "final-only", x.cpu().numpy(), d["inv_xs"][-1], ld.cpu().numpy(),
                   d["inv_ld"], meta, state, d)


@pytest.mark.parametrize("name", [n for n in CASES if n not in ("g6_d4_nan",)])
def test_valu_family_matches_reference_fixture(name):
    """k_valu (the fallback family: misaligned views, permuted loss) held to the
    same fixtures once k_sgpr is switched off (cnf_desc.options)."""
    from cnf_hip import _lib
    meta, state, d = load(name)
    if meta["D"] > 16:
        pytest.skip("wide shape")
    flow = build_flow(meta, state, DEV)
    flow.native_options = _lib.OPT_NO_SGPR
    if flow._native_stack().kernel_name() != "valu-fused":
        pytest.skip("shape outside the k_valu table")
    x = torch.from_numpy(d["x"]).to(DEV)
    with torch.no_grad():
        zs, ld = flow(x)
        z, ld2 = flow.transform(x)
    assert rel_err(torch.stack(zs).cpu().numpy(), d["zs"]) <= TOL
    assert rel_err(ld.cpu().numpy(), d["ld"]) <= TOL
    assert rel_err(z.cpu().numpy(), d["zs"][-1]) <= TOL
    if "inv_xs" in d:
        with torch.no_grad():
            xr, ild = flow.inverse_transform(torch.from_numpy(d["zs"][-1]).to(DEV))
        _check_inverse(name, "valu", xr.cpu().numpy(), d["inv_xs"][-1], ild.cpu().numpy(),
                       d["inv_ld"], meta, state, d)


def test_every_layer_outputs_at_full_size():
    """The zs list (every layer's z, 284 B/row) at 2^20 rows with random_flip:
    its last entry agrees with the final-only output and the log-dets agree
    (different kernels: k_valu stores every layer, k_sgpr serves final-only
    launches with exp2 of log2(e)-scaled weights, so agreement is to fp32
    rounding, not bitwise)."""
    flow = _make_flow(10, 6, [5, 5], 0.1, 5, random_flip=True)
    x = _logits((1 << 20) + 33, 10, 7)
    with torch.no_grad():
        zs, ld = flow(x)
        z, ld2 = flow.transform(x)
        xs, ild = flow.backward(z)
    assert len(zs) == 6
    assert ((zs[-1] - z).abs() / (z.abs() + 1)).max().item() <= TOL
    assert ((ld - ld2).abs() / (ld2.abs() + 1)).max().item() <= TOL
    assert ((xs[-1] - x).abs() / (x.abs() + 1)).max().item() <= TOL
    assert ((ild + ld).abs() / (ld.abs() + 1)).max().item() <= TOL
    idx = torch.randperm(x.shape[0], generator=torch.Generator().manual_seed(2))[:1024].to(DEV)
    ol = _oracle_layers(flow)
    for l, ly in enumerate(flow.layers):
        ol[l] = O.OracleLayer(10, ol[l].s_net, ol[l].t_net, ly.perm.reshape(-1).cpu().numpy())
    ozs, _ = O.flow_forward(ol, x[idx].cpu().numpy())
    for l in range(6):
        assert rel_err(zs[l][idx].cpu().numpy(), ozs[l]) <= TOL


def test_random_flip_state_dict_reload_refreshes_native_tables():
    """load_state_dict of another random_flip flow (new permutations and
    weights) after the first native call: the kernels must see the new
    tables (flows/flows.py:92-99, 110-112)."""
    a = _make_flow(10, 4, [5, 5], 0.2, 1, random_flip=True)
    b = _make_flow(10, 4, [5, 5], 0.2, 2, random_flip=True)
    assert any(not torch.equal(la.perm, lb.perm) for la, lb in zip(a.layers, b.layers))
    x = _logits(1000, 10, 3)
    with torch.no_grad():
        a.transform(x)
    a.load_state_dict(b.state_dict())
    with torch.no_grad():
        z, ld = a.transform(x)
        xr, _ = a.inverse_transform(z)
    ol = _oracle_layers(b)
    for l, ly in enumerate(b.layers):
        ol[l] = O.OracleLayer(10, ol[l].s_net, ol[l].t_net, ly.perm.reshape(-1).cpu().numpy())
    ozs, old = O.flow_forward(ol, x.cpu().numpy())
    assert rel_err(z.cpu().numpy(), ozs[-1]) <= TOL
    assert rel_err(ld.cpu().numpy(), old) <= TOL
    assert ((xr - x).abs() / (x.abs() + 1)).max().item() <= TOL


def test_data_write_needs_invalidate_and_backward_checks_versions():
    """Writes through .data bypass version counters: invalidate_native() picks
    them up.  An in-place weight change between the native forward and its
    backward raises, as torch autograd does."""
    f = _make_flow(10, 2, [5, 5], 0.1, 1)
    x = _logits(256, 10, 1)
    with torch.no_grad():
        z0, _ = f.transform(x)
    f.layers[0].t.layers[0].bias.data.add_(0.5)
    f.invalidate_native()
    with torch.no_grad():
        z1, _ = f.transform(x)
    ozs, _ = O.flow_forward(_oracle_layers(f), x.cpu().numpy())
    assert rel_err(z1.cpu().numpy(), ozs[-1]) <= TOL and not torch.equal(z0, z1)
    z, ld = f.transform(x)           # grad-enabled: native autograd forward
    with torch.no_grad():
        f.layers[1].s.layers[0].weight.mul_(2.0)
    with pytest.raises(RuntimeError, match="modified by an inplace"):
        (z.sum() + ld.sum()).backward()


def test_out_of_range_labels_poison_the_loss_terms():
    """The reference's probs.gather(1, y) raises on a bad label; the fused
    kernels turn it into NaN terms and gradients instead of a silent wrong loss."""
    from cnf_hip import vjp as V
    f = _make_flow(10, 6, [5, 5], 0.1, 9)
    stack = f._native_stack()
    x = _logits(1000, 10, 1)
    y = torch.randint(0, 10, (1000,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(3))
    t_ok, _, _ = stack.forward_loss(x, y)
    assert torch.isfinite(t_ok).all()
    for bad in (10, -1, 1 << 33):
        yb = y.clone()
        yb[17] = bad
        t, _, _ = stack.forward_loss(x, yb)
        assert torch.isnan(t[0]) and torch.isnan(t[1]) and torch.isfinite(t[2])
        tg, g, _ = V.loss_and_grads(stack, x, yb, grad_scale=1e-3)
        assert torch.isnan(tg[0]) and torch.isnan(g).any()


@pytest.mark.parametrize("D,hidden,L,flip", [(10, [5, 5], 6, False), (3, [3, 3], 5, False),
                                             (10, [5, 5], 3, True), (100, [100, 100], 2, False)])
def test_fused_predict_matches_reference_formula(D, hidden, L, flip):
    """cnf_predict (one launch: centring, flow, softmax, prior correction) vs the
    reference's Calibrator.predict math (calibrators.py:40-44, 350-352) in fp64
    on the flow's fp32 outputs."""
    # 100-wide Linears at N(0, 0.1) make the flow chaotic: the last-ulp
    # difference between the kernel's in-launch centring and torch's mean
    # grows past 1e-5 in the probabilities; the wide case runs at N(0, 0.03)
    f = _make_flow(D, L, hidden, 0.1 if D <= 16 else 0.03, 4, random_flip=flip)
    stack = f._native_stack()
    g = torch.Generator(device=DEV).manual_seed(8)
    x = torch.randn(5000, D, device=DEV, generator=g) * 3 + 1
    pri = torch.rand(D, generator=torch.Generator().manual_seed(1)).double() + 0.1
    lp = torch.log(pri / pri.sum())
    n0 = engine.stats["predict"]
    probs = stack.predict(x, lp)
    fused = engine.stats["predict"] == n0 + 1
    assert fused  # one cnf_predict launch: k_sgpr (random_flip too) or k_wide (D=100)
    with torch.no_grad():
        z, _ = f.transform(x - x.mean(dim=1, keepdim=True))
    p = torch.softmax(z.double(), dim=1).cpu()
    ref = torch.softmax(torch.log(p + 1e-7) - lp, dim=1).numpy()
    assert np.max(np.abs(probs.cpu().numpy() - ref)) <= 1e-5


def test_fused_wide_predict_at_n01_within_the_references_own_fp32_error():
    """The wide fused predict (k_wide16's predict mode) at N(0, 0.1) weights,
    where the 100-wide flow amplifies last-ulp input differences: the fused
    probabilities must be as close to the fp64 evaluation of the reference
    formula (calibrators.py:40-44, 350-352; centring, flow and softmax all in
    fp64 on the CPU) as the reference's own fp32 evaluation is, with 1e-5 as
    the floor: tol = max(1e-5, 2 x |fp32 ref - fp64 ref|)."""
    D, hidden, L = 100, [100, 100], 2
    f = _make_flow(D, L, hidden, 0.1, 4)
    stack = f._native_stack()
    g = torch.Generator(device=DEV).manual_seed(8)
    x = torch.randn(5000, D, device=DEV, generator=g) * 3 + 1
    pri = torch.rand(D, generator=torch.Generator().manual_seed(1)).double() + 0.1
    lp = torch.log(pri / pri.sum())
    n0 = engine.stats["predict"]
    probs = stack.predict(x, lp).cpu().double()
    assert engine.stats["predict"] == n0 + 1
    import copy

    def formula(flow, xx):
        with torch.no_grad():
            z, _ = flow.transform(xx - xx.mean(dim=1, keepdim=True))
        p = torch.softmax(z.double(), dim=1).cpu()
        return torch.softmax(torch.log(p + 1e-7) - lp, dim=1)
    ref32 = formula(copy.deepcopy(f).cpu(), x.cpu())
    ref64 = formula(copy.deepcopy(f).cpu().double(), x.cpu().double())
    err_ref = (ref32 - ref64).abs().max().item()
    err_gpu = (probs - ref64).abs().max().item()
    tol = max(1e-5, 2 * err_ref)
    import conftest
    conftest.RECORDS.setdefault("predict_errors", []).append(
        {"test": "wide_predict_n01", "gpu_vs_fp64": err_gpu, "ref_fp32_vs_fp64": err_ref,
         "tol": tol})
    assert err_gpu <= tol, (err_gpu, err_ref)


@pytest.mark.parametrize("name", ["g2_nvp_d10_n02", "g6_d10_randflip", "g3_nvp_d100_n003",
                                  "g1_nice_d3_n02"])
@pytest.mark.parametrize("via_ops", [True, False])
def test_torch_ops_and_ctypes_boundaries_agree_with_fixture(name, via_ops, monkeypatch):
    """Both host boundaries -- the cnf::* torch.library operators (C++) and the
    ctypes calls -- reach the same kernels and match the reference fixture."""
    monkeypatch.setattr(engine, "USE_TORCH_OPS", via_ops)
    meta, state, d = load(name)
    flow = build_flow(meta, state, DEV)
    x = torch.from_numpy(d["x"]).to(DEV)
    n0 = engine.stats["torch_ops"]
    with torch.no_grad():
        zs, ld = flow(x)
        z, _ = flow.transform(x)
    assert (engine.stats["torch_ops"] - n0 == 2) == via_ops
    assert rel_err(torch.stack(zs).cpu().numpy(), d["zs"]) <= TOL
    assert rel_err(ld.cpu().numpy(), d["ld"]) <= TOL
    assert rel_err(z.cpu().numpy(), d["zs"][-1]) <= TOL


def test_torch_ops_autograd_matches_reference_gradients():
    """cnf::flow's C++ autograd kernel (backward = cnf_vjp) against the
    reference's own autograd gradients (g5 fixture, calibrators.py:288-291)."""
    from cnf_hip import _lib
    assert _lib.torch_ops() is not None
    meta, state, d = load("g5_grads_d10")
    flow = build_flow(meta, state, DEV)
    x = torch.from_numpy(d["x"]).to(DEV)
    y = torch.from_numpy(d["y"]).to(DEV)
    n0 = engine.stats["torch_ops"]
    zs, ld = flow(x)
    assert engine.stats["torch_ops"] == n0 + 1
    probs = torch.softmax(zs[-1], dim=1)
    ce = torch.log(probs.gather(1, y.view(-1, 1)) + 1e-7)
    loss = -torch.mean(ce.squeeze() + ld)
    flow.zero_grad()
    loss.backward()
    worst = 0.0
    for k, p in flow.named_parameters():
        if p.requires_grad:
            ref = d["gcal:" + k]
            worst = max(worst, float(np.max(np.abs(p.grad.cpu().numpy() - ref))) /
                        (float(np.max(np.abs(ref))) + 1e-3))
    assert worst <= 1e-4, worst
