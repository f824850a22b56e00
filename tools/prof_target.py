"""Lean profiling target: N launches of one fused pass (no CPU baseline, no
variants) so rocprofv3 counter passes see only the kernel of interest."""
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
ap.add_argument("--all", action="store_true")
ap.add_argument("--batch", type=int, default=0)
ap.add_argument("--mode", default="loss", choices=["loss", "forward"])
a = ap.parse_args()
w = dict(bench.WORKLOADS[a.workload])
if a.batch:
    w["B"] = a.batch
mode = a.mode if (w["D"] <= 16 and not w["inverse"] and not a.all) else "forward"
r = bench.Runner(w, torch.device("cuda:0"), 1.5e9, all_outputs=a.all, mode=mode)
for _ in range(a.launches):
    r.step()
torch.cuda.synchronize()
print("done", r.stack.kernel_name(), w)
