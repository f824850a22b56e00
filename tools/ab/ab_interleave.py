"""Interleaved A/B timing of library builds in ONE process: every build in
tools/ab/lib*.so (plus the shipped libcnf_hip.so as "shipped") is loaded side
by side (ctypes, RTLD_LOCAL: each keeps its own kernels), and the same
pre-built launches (the shipped build's prepared blob: the builds must share
cnf_prepare's layout) are timed build after build, round after round, so
clock drift and box-to-box spread fall on every build alike.  Prints one JSON
line per (mode, B): the median and min per-launch time of each build.
usage: ab_interleave.py [modes=loss,forward (also inverse, all: every layer's z)] [Bs=1048576,8388608] [rounds=9]"""
import ctypes
import glob
import json
import os
import random
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from cnf_hip import _lib  # noqa: E402

modes = (sys.argv[1] if len(sys.argv) > 1 else "loss,forward").split(",")
Bs = [int(b) for b in (sys.argv[2] if len(sys.argv) > 2 else "1048576,8388608").split(",")]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 9
libs = {"shipped": _lib.lib()}
for p in sorted(glob.glob(os.path.join(ROOT, "tools", "ab", "lib*.so"))):
    name = os.path.basename(p)[3:-3]
    lib = ctypes.CDLL(p, mode=ctypes.RTLD_LOCAL)
    for fn in ("cnf_forward", "cnf_inverse", "cnf_forward_loss"):
        getattr(lib, fn).restype = ctypes.c_int
    libs[name] = lib
dev = torch.device("cuda:0")
for mode in modes:
    for B in Bs:
        wl = "cfg5" if mode == "inverse" else "cfg2"
        w = dict(bench.WORKLOADS[wl], B=B)
        r = bench.Runner(w, dev, 1.0e9, all_outputs=(mode == "all"),
                         mode="loss" if mode == "loss" else "forward")
        launches = max(24, (160 << 20) // B)
        r.settle(0.5)
        times = {k: [] for k in libs}
        ratios = {k: [] for k in libs}
        order = list(libs)
        rng = random.Random(1234 + B)
        for _ in range(rounds):
            rng.shuffle(order)  # a fresh order every round: no build always follows another
            got = {}
            for k in order:
                lib = libs[k]
                r.lib = lib
                r.fn = lib.cnf_inverse if w["inverse"] else lib.cnf_forward
                got[k] = bench.kernel_only_seconds(r, launches) * 1e6
                times[k].append(got[k])
            for k in libs:  # paired with the shipped build of the same round
                ratios[k].append(got[k] / got["shipped"])
        r.lib = libs["shipped"]
        out = {"mode": mode, "B": B, "rounds": rounds, "launches": launches,
               "median_us": {k: round(statistics.median(v), 2) for k, v in times.items()},
               "min_us": {k: round(min(v), 2) for k, v in times.items()}}
        # median over rounds of (build / shipped) timed in the same round
        out["vs_shipped"] = {k: round(statistics.median(v), 4) for k, v in ratios.items()}
        print(json.dumps(out), flush=True)
        del r
        torch.cuda.empty_cache()
