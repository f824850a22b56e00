"""Host time per native call at the calibrator's sizes (N=1,500 rows per
training batch) and cfg1's B=4,096: wall-clock per call of
Flow.transform (forward + log-det) through the torch.library operators and
through ctypes, against the device time of the same launch."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "calibration-normalizing-flows_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import bench  # noqa: E402
from cnf_hip import engine  # noqa: E402

dev = torch.device("cuda:0")
res = []
for name, w, B in (("calibrator", dict(D=10, L=5, hidden=[3, 3], scale=True), 1500),
                   ("cfg1", dict(bench.WORKLOADS["cfg1"]), 4096),
                   ("cfg2_small", dict(bench.WORKLOADS["cfg2"]), 1500)):
    flow = bench.make_flow(dict(w, inverse=False), dev)
    x, _ = bench.synthetic_logits(B, w["D"], dev, 5)
    row = {"case": name, "B": B, "D": w["D"], "L": w["L"], "hidden": w["hidden"]}
    for label, ops in (("torch_ops", True), ("ctypes", False)):
        engine.USE_TORCH_OPS = ops
        with torch.no_grad():
            for _ in range(50):
                flow.transform(x)
            torch.cuda.synchronize()
            n = 2000
            t0 = time.perf_counter()
            for _ in range(n):
                flow.transform(x)
            host = (time.perf_counter() - t0) / n
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / n
        row[label + "_host_us"] = round(host * 1e6, 2)
        row[label + "_wall_us"] = round(wall * 1e6, 2)
    # device time of one launch
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.no_grad():
        e0.record()
        for _ in range(200):
            flow.transform(x)
        e1.record()
        torch.cuda.synchronize()
    row["device_us"] = round(e0.elapsed_time(e1) / 200 * 1e3, 2)
    res.append(row)
print(json.dumps(res))
