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
    x[5, 3] = float("nan")
    tr.step(x, y, 512)
    assert tr.guard.tripped() & NAN
