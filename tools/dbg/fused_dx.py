"""Debug: fused vs layer-at-a-time dx on the cfg4 shape; locate the worst rows
and check them against fp64 CPU autograd."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
sys.path.insert(0, "calibration-normalizing-flows_amd")
from test_gpu_vjp import _flow  # noqa
from cnf_hip import _lib
from cnf_hip import vjp as V

DEV = "cuda:0"
L = int(sys.argv[1]) if len(sys.argv) > 1 else 12
B = int(sys.argv[2]) if len(sys.argv) > 2 else (1 << 14) + 37
f = _flow(100, L, [100, 100], 0.03, 6, flip=False).to(DEV)
g = torch.Generator(device=DEV).manual_seed(2)
x = torch.randn(B, 100, device=DEV, generator=g) * 2
y = torch.randint(0, 100, (B,), device=DEV, generator=g)
t1, g1, d1 = V.loss_and_grads(f._native_stack(), x, y, grad_scale=1.0 / B, need_dx=True)
f.native_options = _lib.OPT_NO_WIDE
t2, g2, d2 = V.loss_and_grads(f._native_stack(), x, y, grad_scale=1.0 / B, need_dx=True)
d1, d2 = d1.cpu().double(), d2.cpu().double()
diff = (d1 - d2).abs()
rowmax = diff.max(1).values
print("L", L, "B", B, "max|dx|", d2.abs().max().item(), "maxdiff", diff.max().item())
worst = torch.argsort(rowmax, descending=True)[:8]
print("worst rows", worst.tolist(), rowmax[worst].tolist())
print("rows with diff > 1e-9:", int((rowmax > 1e-9).sum()), "hist of row//32:",
      np.unique((torch.nonzero(rowmax > 1e-9).squeeze(1) // 32).numpy())[:40])
# fp64 CPU autograd of the worst rows (per-row gradient * 1/B)
fc = _flow(100, L, [100, 100], 0.03, 6, flip=False).double()
xs = x[worst].cpu().double().requires_grad_(True)
zs, ld = fc(xs)
p = torch.softmax(zs[-1], 1).gather(1, y[worst].cpu().view(-1, 1)).squeeze(1)
loss = -(torch.log(p + 1e-7) + ld).sum() / B
loss.backward()
ref = xs.grad
print("fused err", (d1[worst] - ref).abs().max().item(), "layered err", (d2[worst] - ref).abs().max().item())
# relu kinks: the smallest |pre-activation| of each worst row over every hidden unit (fp64)
acts = []
hooks = [m.register_forward_hook(lambda m, i, o: acts.append(o.detach()))
         for m in fc.modules() if isinstance(m, torch.nn.Linear)]
with torch.no_grad():
    acts.clear()
    fc(x[worst].cpu().double())
for h in hooks:
    h.remove()
mins = torch.stack([a.abs().min(1).values for a in acts if a.shape[1] == 100]).min(0).values
print("min |pre-activation| per worst row:", mins.tolist())
