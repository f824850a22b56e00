"""Launch time of one fused pass against the batch size: fits t = a + b*B so
the fixed cost of a launch (ramp-up, tail, the follow-up reduction) separates
from the steady-state cost per row.  usage: batch_sweep.py [mode] [options]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "loss"
opts = int(sys.argv[2]) if len(sys.argv) > 2 else 0
dev = torch.device("cuda:0")
rows = []
for lg in range(16, 25):
    w = dict(bench.WORKLOADS["cfg2"], B=1 << lg)
    r = bench.Runner(w, dev, 1.0e9, all_outputs=(mode == "all"),
                     mode="loss" if mode == "loss" else "forward")
    if opts:
        r.stack.options = opts
        r.stack._refresh_desc()
        r.desc = __import__("ctypes").byref(r.stack.desc)
    t = bench.kernel_only_seconds(r, 40)
    rows.append((1 << lg, t))
    del r
    torch.cuda.empty_cache()
B = np.array([b for b, _ in rows], dtype=np.float64)
T = np.array([t for _, t in rows])
b, a = np.polyfit(B[2:], T[2:], 1)
print(json.dumps({"mode": mode, "options": opts, "kernel_us": {int(k): round(v * 1e6, 2) for k, v in rows},
                  "fit_fixed_us": round(a * 1e6, 2), "fit_rows_per_s": round(1 / b, 1)}))
