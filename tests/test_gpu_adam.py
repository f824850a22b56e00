"""cnf_adam_step (one-launch Adam over a stack's parameters, cnf_hip/adam.py)
against torch.optim.Adam on the same gradients: the optimizer half of the
calibrator's on-device training step (reference: calibrators.py:239-295 steps
torch.optim.Adam at its defaults)."""
import os
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "calibration-normalizing-flows_amd"))

from cnf_hip import vjp as V  # noqa: E402
from cnf_hip.adam import StackAdam  # noqa: E402
from flows.flows import Flow, NvpCouplingLayer  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _flow(D, L, hidden, seed=0):
    # 100-wide conditioners at N(0, 0.1) make the loss chaotic within a few
    # Adam steps (gradients grow 5x): rounding-level parameter differences then
    # grow past any tolerance, so the wide case starts near the smooth regime
    torch.manual_seed(seed)
    f = Flow([NvpCouplingLayer(D, hidden) for _ in range(L)])
    g = torch.Generator().manual_seed(seed)
    sigma = 0.1 if D <= 16 else 0.02
    with torch.no_grad():
        for p in f.parameters():
            if p.requires_grad:
                p.copy_(torch.randn(p.shape, generator=g) * sigma)
    return f


@pytest.mark.parametrize("D,L,hidden,wd", [(10, 6, [5, 5], 0.0), (100, 2, [100, 100], 0.01),
                                           (20, 24, [8, 8], 0.0),  # 288 tensors: 3 launches
                                           (10, 12, [5, 5], 0.0)])  # narrow, L > 8
def test_stack_adam_matches_torch_adam(D, L, hidden, wd):
    fa = _flow(D, L, hidden).to(DEV)
    fb = _flow(D, L, hidden).to(DEV)
    sa = fa._native_stack()
    ta = torch.optim.Adam([p for p in fb.parameters() if p.requires_grad], lr=3e-3,
                          weight_decay=wd)
    na = StackAdam.like(sa, torch.optim.Adam([p for p in fa.parameters() if p.requires_grad],
                                             lr=3e-3, weight_decay=wd))
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(4096, D, device=DEV, generator=g)
    y = torch.randint(0, D, (4096,), device=DEV, generator=g)
    for _ in range(5):
        _, ga, _ = V.loss_and_grads(sa, x, y, grad_scale=1.0 / 4096)
        na.step(ga)
        _, gb, _ = V.loss_and_grads(fb._native_stack(), x, y, grad_scale=1.0 / 4096)
        for p, gg in zip([p for p in fb.parameters() if p.requires_grad],
                         V._split(fb._native_stack(), gb)):
            p.grad = gg.view_as(p)
        ta.step()
    # Adam's step is ~lr per element whatever the gradient's size, so the scale
    # of a difference is the total movement (5 lr), not |p|
    for (k, p), (_, q) in zip(fa.named_parameters(), fb.named_parameters()):
        if p.requires_grad:
            assert ((p - q).abs() / (q.abs() + 5 * 3e-3)).max().item() <= 1e-4, k
    # the updated weights reach the kernels (the prepared-weight cache rebuilt)
    z1, _ = fa.transform(x)
    z2, _ = fb.transform(x)
    assert ((z1 - z2).abs() / (z2.abs() + 1)).max().item() <= 1e-5
