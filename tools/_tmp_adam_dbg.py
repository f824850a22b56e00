import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "calibration-normalizing-flows_amd"))
import torch
from test_gpu_adam import _flow, V, StackAdam, DEV
D, L, hidden, wd = 100, 2, [100, 100], 0.01
fa = _flow(D, L, hidden).to(DEV); fb = _flow(D, L, hidden).to(DEV)
sa = fa._native_stack()
pa = [p for p in fa.parameters() if p.requires_grad]; pb = [p for p in fb.parameters() if p.requires_grad]
ta = torch.optim.Adam(pb, lr=3e-3, weight_decay=wd)
na = StackAdam.like(sa, torch.optim.Adam(pa, lr=3e-3, weight_decay=wd))
g = torch.Generator(device=DEV).manual_seed(1)
x = torch.randn(4096, D, device=DEV, generator=g); y = torch.randint(0, D, (4096,), device=DEV, generator=g)
for step in range(5):
    _, ga, _ = V.loss_and_grads(sa, x, y, grad_scale=1.0 / 4096)
    _, gb, _ = V.loss_and_grads(fb._native_stack(), x, y, grad_scale=1.0 / 4096)
    print("step", step, "grad diff", (ga - gb).abs().max().item(), "grad max", gb.abs().max().item())
    na.step(ga)
    for p, gg in zip(pb, V._split(fb._native_stack(), gb)):
        p.grad = gg.view_as(p)
    ta.step()
    worst = max(((p - q).abs().max().item(), i) for i, (p, q) in enumerate(zip(pa, pb)))
    print("  param diff", worst)
