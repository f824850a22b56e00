"""The device-side non-finite guard (cnf_guard_nonfinite, include/cnf.h; the
counterpart of the reference's NaN abort, run_experiment3D.py:129-131): the
flag bits for clean, NaN, inf and mixed data, unaligned views, ragged sizes,
accumulation over launches, and the data-parallel trainer's nan_guard."""
import pytest
import torch

from cnf_hip.guard import INF, NAN, NonFiniteGuard

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("n", [1, 3, 4, 1000, 1 << 20, (1 << 22) + 7])
@pytest.mark.parametrize("offset", [0, 1])
def test_guard_bits(n, offset):
    base = torch.randn(n + offset, device=DEV)
    a = base[offset:]  # offset 1: a 4-byte-aligned, not 16-byte-aligned view
    g = NonFiniteGuard(DEV)
    assert g.check(a).tripped() == 0
    for pos in (0, n // 2, n - 1):
        b = a.clone()
        b[pos] = float("nan")
        assert NonFiniteGuard(DEV).check(b).tripped() == NAN
        b[pos] = float("-inf")
        assert NonFiniteGuard(DEV).check(b).tripped() == INF
    if n >= 3:
        b = a.clone()
        b[0] = float("inf")
        b[-1] = float("nan")
        assert NonFiniteGuard(DEV).check(b).tripped() == NAN | INF


def test_guard_accumulates_until_reset():
    g = NonFiniteGuard(DEV)
    clean = torch.randn(4096, device=DEV)
    bad = clean.clone()
    bad[17] = float("nan")
    g.check(clean, bad, clean)
    assert g.tripped() == NAN
    g.check(clean)
    assert g.tripped() == NAN  # never cleared by the library
    g.reset()
    assert g.check(clean).tripped() == 0


def test_guard_on_flow_outputs():
    """z / log-det of a stack whose exp(s) overflows (the g6_d4_nan fixture in
    strict mode: NaN at masked positions, as the reference)."""
    from _golden import load
    from _model import build_flow
    meta, state, d = load("g6_d4_nan")
    f = build_flow(meta, state, DEV, strict_nan=True)
    with torch.no_grad():
        z, ld = f.transform(torch.from_numpy(d["x"]).to(DEV))
    assert NonFiniteGuard(DEV).check(z).tripped() & NAN
    f2 = build_flow(meta, state, DEV, strict_nan=False)
    with torch.no_grad():
        z2, ld2 = f2.transform(torch.from_numpy(d["x"]).to(DEV))
    assert NonFiniteGuard(DEV).check(z2).tripped() == 0 or torch.isinf(z2).any()


def test_trainer_nan_guard():
    from cnf_hip.dist import ShardedFlowTrainer
    from flows.flows import Flow, NvpCouplingLayer
    torch.manual_seed(3)
    flow = Flow([NvpCouplingLayer(10, [5, 5]) for _ in range(2)]).to(DEV)
    opt = torch.optim.Adam(flow.parameters(), lr=1e-3)
    tr = ShardedFlowTrainer(flow, opt, nan_guard=True)
    x = torch.randn(512, 10, device=DEV)
    y = torch.randint(0, 10, (512,), device=DEV)
    tr.step(x, y, 512)
    assert tr.guard is not None and tr.guard.tripped() == 0
    before = [p.detach().clone() for p in tr.params]
    m_before = tr._adam._m.clone()
    v_before = tr._adam._v.clone()
    x[5, 3] = float("nan")
    tr.step(x, y, 512)
    assert tr.guard.tripped() & NAN
    # the tripped step updated nothing: the last finite weights and moments
    # survive (the reference breaks before opt.step(), run_experiment3D.py:129-133)
    for a, b in zip(tr.params, before):
        assert torch.equal(a.detach(), b)
    assert torch.equal(tr._adam._m, m_before) and torch.equal(tr._adam._v, v_before)
    assert all(torch.isfinite(p).all() for p in tr.params)


def test_trainer_nan_guard_torch_optimizer():
    """A torch optimizer the native Adam does not reproduce (SGD) steps on the
    host path; with the guard on, a tripped step is skipped there too."""
    from cnf_hip.dist import ShardedFlowTrainer
    from flows.flows import Flow, NvpCouplingLayer
    torch.manual_seed(4)
    flow = Flow([NvpCouplingLayer(10, [5, 5]) for _ in range(2)]).to(DEV)
    opt = torch.optim.SGD(flow.parameters(), lr=1e-2)
    tr = ShardedFlowTrainer(flow, opt, nan_guard=True)
    x = torch.randn(256, 10, device=DEV)
    y = torch.randint(0, 10, (256,), device=DEV)
    tr.step(x, y, 256)
    before = [p.detach().clone() for p in tr.params]
    x[0, 0] = float("inf")
    tr.step(x, y, 256)
    assert tr.guard.tripped()
    for a, b in zip(tr.params, before):
        assert torch.equal(a.detach(), b)


def test_adam_step_guarded_abi():
    """cnf_adam_step_guarded: flag 0 gives cnf_adam_step's bits, a set flag
    leaves parameters and moments untouched; the sched form likewise."""
    import ctypes
    from cnf_hip import _lib
    from cnf_hip.adam import StackAdam
    from flows.flows import Flow, NvpCouplingLayer
    torch.manual_seed(5)
    flow = Flow([NvpCouplingLayer(10, [5, 5]) for _ in range(3)]).to(DEV)
    stack = flow._native_stack()
    P = stack.param_count()
    g = torch.randn(P, device=DEV) * 1e-2

    def run(flag_value, sched):
        f = Flow([NvpCouplingLayer(10, [5, 5]) for _ in range(3)]).to(DEV)
        f.load_state_dict(flow.state_dict())
        st = f._native_stack()
        ad = StackAdam(st, lr=1e-3)
        ad.step(g)  # moments non-zero
        ps, _ = ad._ensure_state()
        arr = (ctypes.c_void_p * len(ps))(*[p.data_ptr() for p in ps])
        flag = torch.full((1,), flag_value, dtype=torch.int32, device=DEV)
        sch = torch.tensor([1e-3 / (1 - 0.9 ** 2), (1 - 0.999 ** 2) ** 0.5], device=DEV)
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        rc = _lib.lib().cnf_adam_step_guarded(
            ctypes.byref(st.desc), arr, ctypes.c_void_p(g.data_ptr()),
            ctypes.c_void_p(ad._m.data_ptr()), ctypes.c_void_p(ad._v.data_ptr()),
            ctypes.c_int64(2), ctypes.c_double(1e-3),
            ctypes.c_void_p(sch.data_ptr()) if sched else None, ctypes.c_double(0.9),
            ctypes.c_double(0.999), ctypes.c_double(1e-8), ctypes.c_double(0.0),
            ctypes.c_void_p(flag.data_ptr()), stream)
        assert rc == 0
        torch.cuda.synchronize()
        return [p.detach().clone() for p in ps], ad._m.clone(), ad._v.clone(), ad

    for sched in (False, True):
        p0, m0, v0, ad0 = run(0, sched)
        # reference: the plain step 2 on a fresh copy
        f = Flow([NvpCouplingLayer(10, [5, 5]) for _ in range(3)]).to(DEV)
        f.load_state_dict(flow.state_dict())
        ref = StackAdam(f._native_stack(), lr=1e-3)
        ref.step(g)
        ref.step(g)
        ps_ref, _ = ref._ensure_state()
        for a, b in zip(p0, ps_ref):
            assert torch.equal(a, b.detach())
        assert torch.equal(m0, ref._m) and torch.equal(v0, ref._v)
        p1, m1, v1, ad1 = run(1, sched)
        f = Flow([NvpCouplingLayer(10, [5, 5]) for _ in range(3)]).to(DEV)
        f.load_state_dict(flow.state_dict())
        one = StackAdam(f._native_stack(), lr=1e-3)
        one.step(g)
        ps_one, _ = one._ensure_state()
        for a, b in zip(p1, ps_one):
            assert torch.equal(a, b.detach())
        assert torch.equal(m1, one._m) and torch.equal(v1, one._v)
