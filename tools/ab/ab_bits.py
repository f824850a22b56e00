"""Output fingerprints of an experimental library build (CNF_HIP_LIB=...):
sha256 of z, ld and the loss terms of the cfg2 fused eval, the cfg2 forward and
the cfg5 inverse at a few batch sizes (full waves, ragged, small), so A/B
builds that must keep the arithmetic can be compared bit for bit across runs
(one JSON line per build; equal lines = bitwise-identical outputs)."""
import ctypes
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
h = lambda t: hashlib.sha256(t.detach().cpu().numpy().tobytes()).hexdigest()[:16]
res = {"lib": os.path.basename(os.environ.get("CNF_HIP_LIB", "libcnf_hip.so"))}
for wl, mode in (("cfg2", "loss"), ("cfg2", "forward"), ("cfg5", "forward")):
    for B in (1 << 20, 1000003, 4096 + 77):
        w = dict(bench.WORKLOADS[wl], B=B)
        r = bench.Runner(w, dev, 0.0, mode=mode)
        x, y, z, ld, _ = r.sets[0]
        z.fill_(float("nan"))
        ld.fill_(float("nan"))
        r.step()
        torch.cuda.synchronize()
        key = "%s_%s_%d" % (wl, mode, B)
        res[key] = [h(z), h(ld)] + ([h(r.terms)] if mode == "loss" else [])
        del r
print(json.dumps(res))
