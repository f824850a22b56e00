"""Per-wave timeline of one k_sgpr launch (diagnostic build: `make -C
calibration-normalizing-flows_amd/csrc trace`, loaded via CNF_HIP_LIB).
Prints quantiles (us, from the first wave's start) of each mark."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CNF_HIP_LIB", os.path.join(ROOT, "calibration-normalizing-flows_amd",
                                                  "cnf_hip", "libcnf_hip_trace.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from cnf_hip import _lib  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "loss"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
w = dict(bench.WORKLOADS["cfg2"], B=B)
r = bench.Runner(w, torch.device("cuda:0"), 0.5e9, all_outputs=(mode == "all"),
                 mode="loss" if mode == "loss" else "forward")
for _ in range(20):
    r.step()
torch.cuda.synchronize()
lib = _lib.lib()
n = 16384 * 8
buf = (ctypes.c_ulonglong * n)()
lib.cnf_diag_trace.restype = ctypes.c_int
assert lib.cnf_diag_trace(buf, n) == n
a = np.frombuffer(buf, dtype=np.uint64).reshape(16384, 8).astype(np.float64)
ntiles = (B + 127) // 128
nw = int((a[:, 0] > 0).sum())
a = a[:nw]
t0 = a[:, 0].min()
us = lambda v: (v - t0) / 100.0  # 100 MHz
out = {"B": B, "waves": nw, "mode": mode}
names = ["start", "tile0_data", "tile0_done", "tile1_data", "tile1_done", "last_done", "end"]
for i, nm in enumerate(names):
    v = a[:, i]
    v = v[v > 0]
    if len(v):
        out[nm] = [round(float(np.quantile(us(v), q)), 2) for q in (0, 0.1, 0.5, 0.9, 1.0)]
d0 = (a[:, 2] - a[:, 1]) / 100.0
out["tile_compute_us"] = [round(float(np.quantile(d0[a[:, 2] > 0], q)), 2) for q in (0.1, 0.5, 0.9)]
print(json.dumps(out))
