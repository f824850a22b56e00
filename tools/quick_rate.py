"""Kernel time of the cfg2 bench pass at a few batch sizes, for A/B runs of
experimental library builds (CNF_HIP_LIB=... python tools/quick_rate.py [mode])."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

for mode in (sys.argv[1:] or ["loss"]):
    res = {"lib": os.path.basename(os.environ.get("CNF_HIP_LIB", "libcnf_hip.so")), "mode": mode}
    for lg in (20, 23):
        wl = bench.WORKLOADS["cfg5" if mode == "inverse" else "cfg2"]
        w = dict(wl, B=1 << lg)
        r = bench.Runner(w, torch.device("cuda:0"), 1.0e9, all_outputs=(mode == "all"),
                         mode="loss" if mode == "loss" else "forward")
        t = min(bench.kernel_only_seconds(r, 30) for _ in range(3))
        res["us_2^%d" % lg] = round(t * 1e6, 2)
        res["Grows_2^%d" % lg] = round(w["B"] / t / 1e9, 2)
        del r
        torch.cuda.empty_cache()
    print(json.dumps(res))
