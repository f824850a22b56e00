"""Autograd through the INVERSE transform (Flow.backward, flows/flows.py:27-37,
114-126) on the native reverse mode (cnf_vjp_inverse) against CPU autograd of
the reference-semantics torch ops."""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "calibration-normalizing-flows_amd"))

from cnf_hip import engine  # noqa: E402
from flows.flows import Flow, NvpCouplingLayer  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _flow(D, L, hidden, sigma, seed, scale=True, shift=True, flip=False):
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


def _err(a, b):
    return (a - b).abs().max().item() / (b.abs().max().item() + 1e-3)


@pytest.mark.parametrize("D,L,hidden,scale,shift,flip", [
    (10, 6, [5, 5], True, True, False),
    (10, 5, [5, 5], True, True, True),    # odd L, random_flip
    (3, 2, [5, 5], False, True, False),   # NICE
    (17, 3, [], True, True, False),       # odd D, no hidden layer
    (100, 2, [100, 100], True, True, True),
])
@pytest.mark.parametrize("via_ops", [True, False])
def test_inverse_autograd_matches_cpu(D, L, hidden, scale, shift, flip, via_ops, monkeypatch):
    # via_ops: the cnf::inverse_flow operator (C++ autograd kernel); else the
    # Python autograd Function over ctypes
    monkeypatch.setattr(engine, "USE_TORCH_OPS", via_ops)
    f = _flow(D, L, hidden, 0.1 if D <= 20 else 0.05, 3, scale, shift, flip)
    z = torch.randn(333, D, generator=torch.Generator().manual_seed(1))
    w = torch.randn(L, 333, D, generator=torch.Generator().manual_seed(2))
    wl = torch.randn(333, generator=torch.Generator().manual_seed(3))

    def objective(flow, zz):
        xs, ld = flow.backward(zz)
        return sum((x * w[i].to(x.device)).sum() for i, x in enumerate(xs)) + \
            (ld * wl.to(ld.device)).sum()

    zc = z.clone().requires_grad_(True)
    objective(f, zc).backward()
    ref = {k: p.grad.clone() for k, p in f.named_parameters() if p.requires_grad}
    fg = f.to(DEV)
    fg.zero_grad()
    zg = z.to(DEV).requires_grad_(True)
    n0, t0 = engine.stats["vjp"], engine.stats["torch_ops"]
    objective(fg, zg).backward()
    if via_ops:
        assert engine.stats["torch_ops"] == t0 + 1 and engine.stats["vjp"] == n0, \
            "cnf::inverse_flow did not run"
    else:
        assert engine.stats["vjp"] == n0 + 1, "native cnf_vjp_inverse did not run"
    for k, p in fg.named_parameters():
        if p.requires_grad:
            assert _err(p.grad.cpu(), ref[k]) <= 1e-4, k
    assert _err(zg.grad.cpu(), zc.grad) <= 1e-4


def test_legacy_inverse_autograd():
    from flows.legacy import LegacyRealNvpFlow
    torch.manual_seed(0)
    f = LegacyRealNvpFlow(10, layers=3, hidden_size=[10], s_activation="tanh")
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for p in f.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.2)
    y = torch.randn(257, 10, generator=torch.Generator().manual_seed(4))
    yc = y.clone().requires_grad_(True)
    x, ld = f.backward(yc)
    (x.sum() * 0.5 + (x * x).sum() + ld.sum()).backward()
    ref = {k: p.grad.clone() for k, p in f.named_parameters()}
    fg = f.to(DEV)
    fg.zero_grad()
    yg = y.to(DEV).requires_grad_(True)
    x, ld = fg.backward(yg)
    (x.sum() * 0.5 + (x * x).sum() + ld.sum()).backward()
    for k, p in fg.named_parameters():
        assert _err(p.grad.cpu(), ref[k]) <= 1e-4, k
    assert _err(yg.grad.cpu(), yc.grad) <= 1e-4
