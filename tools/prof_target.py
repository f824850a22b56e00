"""Lean profiling target: N launches of one fused pass (no CPU baseline, no
variants) so rocprofv3 kernel-trace / counter passes see only the kernels of
interest.  --mode loss: cnf_forward_loss (the bench step); forward: cnf_forward
/ cnf_inverse (cfg5); all: every layer's z (the zs list); train: the fused
calibrator training step cnf_loss_vjp (k_vjp + block-order reductions)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="cfg2")
ap.add_argument("--launches", type=int, default=40)
ap.add_argument("--batch", type=int, default=0)
ap.add_argument("--mode", default="loss", choices=["loss", "forward", "all", "train", "calib"])
ap.add_argument("--settle-s", type=float, default=0.3,
                help="untimed launches for this long first, as bench.py settles the clock; "
                     "tools/trace_stats.py keeps only the last --launches calls")
a = ap.parse_args()
w = dict(bench.WORKLOADS[a.workload])
if a.batch:
    w["B"] = a.batch
dev = torch.device("cuda:0")
if a.mode == "calib":  # the calibrator-fit epochs (graph replays), notebook shape
    import numpy as np
    import calibrators as C
    from flows.realNVP_torch import RealNvpFlow
    rs = np.random.RandomState(5)
    yy = rs.randint(0, 3, size=1500)
    xx = rs.standard_normal((1500, 3)) + 3.0 * np.eye(3)[yy]
    cal = C.TorchFlowCalibrator(RealNvpFlow, xx, yy, layers=5, hidden_size=[3, 3],
                                epochs=a.launches, dev=dev)
    name = "calibrator"
elif a.mode == "train":
    from cnf_hip import vjp as V
    flow = bench.make_flow(w, dev)
    stack = flow._native_stack()
    x, y = bench.synthetic_logits(w["B"], w["D"], dev, 4321)
    import time
    t0 = time.perf_counter()
    while a.settle_s > 0 and time.perf_counter() - t0 < a.settle_s:
        for _ in range(8):
            V.loss_and_grads(stack, x, y, grad_scale=1.0 / w["B"])
        torch.cuda.synchronize()
    for _ in range(a.launches):
        V.loss_and_grads(stack, x, y, grad_scale=1.0 / w["B"])
    name = stack.kernel_name()
else:
    mode = a.mode
    if mode == "loss" and (w["D"] > 16 or w["inverse"]):
        mode = "forward"
    r = bench.Runner(w, dev, 1.5e9, all_outputs=(mode == "all"),
                     mode="loss" if mode == "loss" else "forward")
    if a.settle_s > 0:
        r.settle(a.settle_s)
    for _ in range(a.launches):
        r.step()
    name = r.stack.kernel_name()
torch.cuda.synchronize()
print("done", a.mode, name, w)
