"""Calibrator training step on a wide stack (cfg4: D=100, 12 layers, [100,100],
2^18 rows): the native reverse mode (cnf_loss_vjp -> cnf_wvjp.hip) against
torch autograd through the reference's own ops (the layers' torch math on
the same GPU, cnf_hip/vjp.py _torch_forward).  Prints one JSON line."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "calibration-normalizing-flows_amd"))
import bench  # noqa: E402
from cnf_hip import vjp as V  # noqa: E402


def timed(fn, steps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "cfg4"
    w = bench.WORKLOADS[wl]
    dev = torch.device("cuda:0")
    B = w["B"]
    flow = bench.make_flow(w, dev)
    stack = flow._native_stack()
    x, y = bench.synthetic_logits(B, w["D"], dev, 99)

    def native():
        V.loss_and_grads(stack, x, y, grad_scale=1.0 / B)

    leaves = [p.detach().requires_grad_(True) for p in stack.param_tensors()]

    def autograd():
        zs, ld = V._torch_forward(stack, x, leaves)
        probs = torch.softmax(zs[-1], dim=1)
        ce = torch.log(probs.gather(1, y.view(-1, 1)) + 1e-7)
        loss = -torch.mean(ce.squeeze() + ld)          # calibrators.py:288-291
        torch.autograd.grad(loss, leaves)

    t0 = time.time()
    tn = timed(native, 5)
    ta = timed(autograd, 3)
    t_nat, g_nat, _ = V.loss_and_grads(stack, x, y, grad_scale=1.0 / B)
    zs, ld = V._torch_forward(stack, x, leaves)
    probs = torch.softmax(zs[-1], dim=1)
    loss = -torch.mean(torch.log(probs.gather(1, y.view(-1, 1)) + 1e-7).squeeze() + ld)
    g_ref = torch.cat([g.reshape(-1) for g in torch.autograd.grad(loss, leaves)])
    rel = ((g_nat - g_ref).abs().max() / (g_ref.abs().max() + 1e-3)).item()
    print(json.dumps({"workload": wl, "B": B, "native_ms": round(tn, 3),
                      "torch_autograd_ms": round(ta, 3), "speedup": round(ta / tn, 2),
                      "grad_rel_err": rel, "loss_native": t_nat[0].item() / B,
                      "loss_autograd": loss.item(), "wall_s": round(time.time() - t0, 1)}))


if __name__ == "__main__":
    main()
