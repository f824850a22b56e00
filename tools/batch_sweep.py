"""Device time of one fused pass against the batch size: fits t = a + b*B so
the fixed cost of a call (ramp-up, tail, the follow-up reduction) separates
from the steady-state cost per row.

Each batch size runs on a settled device (0.3 s of untimed calls, as
bench.py) and is timed twice: eager calls back to back (HIP events), and a
HIP graph of N calls replayed (the same ctypes launches captured once) --
below ~2^19 rows the eager loop is host-bound (the Python ctypes call and
the HIP launch take longer than the kernel), so only the graph timing shows
the device's fixed cost there.  The fit uses the graph times from 2^18 rows
up.  usage: batch_sweep.py [mode=loss|forward|all] [options]"""
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
N = 64  # calls per graph


def graph_seconds(r, reps=9):
    s = torch.cuda.Stream(dev)
    keep = r.stream
    r.stream = s
    with torch.cuda.stream(s):
        for _ in range(4):
            r.step()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(N):
                r.step()
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            g.replay()
            e1.record(s)
            torch.cuda.synchronize(dev)
            ts.append(e0.elapsed_time(e1) / 1e3 / N)
    r.stream = keep
    del g
    return float(np.median(ts))


rows = []
for lg in range(16, 25):
    w = dict(bench.WORKLOADS["cfg2"], B=1 << lg)
    r = bench.Runner(w, dev, 1.0e9, all_outputs=(mode == "all"),
                     mode="loss" if mode == "loss" else "forward")
    if opts:
        r.stack.options = opts
        r.stack._refresh_desc()
        r.desc = __import__("ctypes").byref(r.stack.desc)
    r.settle(0.3)
    te = bench.kernel_only_seconds(r, 40)
    tg = graph_seconds(r)
    rows.append((1 << lg, te, tg))
    print(json.dumps({"B": 1 << lg, "eager_us": round(te * 1e6, 2), "graph_us": round(tg * 1e6, 2)}),
          flush=True)
    del r
    torch.cuda.empty_cache()
B = np.array([b for b, _, _ in rows], dtype=np.float64)
T = np.array([t for _, _, t in rows])
sel = B >= (1 << 18)
b, a = np.polyfit(B[sel], T[sel], 1)
print(json.dumps({"mode": mode, "options": opts,
                  "eager_us": {int(k): round(v * 1e6, 2) for k, v, _ in rows},
                  "graph_us": {int(k): round(v * 1e6, 2) for k, _, v in rows},
                  "fit_from_rows": 1 << 18, "fit_fixed_us": round(a * 1e6, 2),
                  "fit_rows_per_s": round(1 / b, 1),
                  "at_2^20": {"graph_us": round(float(T[B == (1 << 20)][0]) * 1e6, 2),
                              "fixed_share": round(float(a / T[B == (1 << 20)][0]), 4)}}))
