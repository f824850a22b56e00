"""A/B of experimental k_valu builds (CNF_HIP_LIB=libcnf_hip_<v>.so): the
every-layer-output pass (the reference Flow.forward's zs list) of cfg2 at 2^20
rows: kernel time and a checksum of the outputs, one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
res = {"lib": os.path.basename(os.environ.get("CNF_HIP_LIB", "libcnf_hip.so"))}
for lg in (20, 23):
    w = dict(bench.WORKLOADS["cfg2"], B=1 << lg)
    r = bench.Runner(w, dev, 1.0e9, all_outputs=True)
    r.i = 0
    r.step()
    torch.cuda.synchronize()
    allt = r.sets[0][4]
    res["sum_2^%d" % lg] = float(allt.double().sum())
    t = min(bench.kernel_only_seconds(r, 30) for _ in range(3))
    res["us_2^%d" % lg] = round(t * 1e6, 2)
    res["TBs_2^%d" % lg] = round(w["B"] * 284 / t / 1e12, 3)
    del r
    torch.cuda.empty_cache()
print(json.dumps(res), flush=True)
