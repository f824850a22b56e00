"""A/B of experimental k_sgpr builds (CNF_HIP_LIB=libcnf_hip_<v>.so): the loss
terms of a seeded cfg2 batch (2^20 and a ragged 2^20+77 rows) and the kernel
time of the fused loss pass, one JSON line per build."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

res = {"lib": os.path.basename(os.environ.get("CNF_HIP_LIB", "libcnf_hip.so"))}
dev = torch.device("cuda:0")
for B in (1 << 20, (1 << 20) + 77, 5000):
    w = dict(bench.WORKLOADS["cfg2"], B=B)
    r = bench.Runner(w, dev, 1.0e9, mode="loss")
    r.i = 0
    r.step()
    r.step()
    torch.cuda.synchronize()
    t1 = r.terms.clone()
    r.i = 0
    r.step()
    torch.cuda.synchronize()
    res["terms_%d" % B] = [float(v) for v in r.terms.tolist()]
    res["repeat_equal_%d" % B] = bool(torch.equal(t1, r.terms))
    if B == 1 << 20:
        t = min(bench.kernel_only_seconds(r, 30) for _ in range(5))
        res["us"] = round(t * 1e6, 2)
        res["Grows"] = round(B / t / 1e9, 2)
    del r
    torch.cuda.empty_cache()
print(json.dumps(res), flush=True)
