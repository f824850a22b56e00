"""Bitwise check of every A/B build in tools/ab/lib*.so against the shipped
library: the same pre-built launch (bench.Runner, set 0) run through each
build, z and log-det compared bit for bit; the loss sums by relative difference
(their summation order follows the grid size, which a build may change).  One JSON line
per (mode, B).  usage: ab_check.py [modes=loss,forward,inverse] [Bs=...]"""
import ctypes
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from cnf_hip import _lib  # noqa: E402

modes = (sys.argv[1] if len(sys.argv) > 1 else "loss,forward,inverse").split(",")
Bs = [int(b) for b in (sys.argv[2] if len(sys.argv) > 2 else "1048576,1000003,4099").split(",")]
libs = {"shipped": _lib.lib()}
for p in sorted(glob.glob(os.path.join(ROOT, "tools", "ab", "lib*.so"))):
    lib = ctypes.CDLL(p, mode=ctypes.RTLD_LOCAL)
    for fn in ("cnf_forward", "cnf_inverse", "cnf_forward_loss"):
        getattr(lib, fn).restype = ctypes.c_int
    libs[os.path.basename(p)[3:-3]] = lib
dev = torch.device("cuda:0")
bad = 0
for mode in modes:
    for B in Bs:
        w = dict(bench.WORKLOADS["cfg5" if mode == "inverse" else "cfg2"], B=B)
        r = bench.Runner(w, dev, 1.0, mode="loss" if mode == "loss" else "forward")
        x, y, out, ld, _ = r.sets[0]
        got = {}
        for k, lib in libs.items():
            r.lib = lib
            r.fn = lib.cnf_inverse if w["inverse"] else lib.cnf_forward
            out.fill_(float("nan"))
            ld.fill_(float("nan"))
            r.term_bufs.zero_()
            r.i = 0
            r.step()
            torch.cuda.synchronize(dev)
            got[k] = (out.clone(), ld.clone(), r.term_bufs[0, 0].clone())
        ref = got["shipped"]
        same = {k: all(torch.equal(a.view(torch.int32), b.view(torch.int32))
                       for a, b in zip(v[:2], ref[:2])) for k, v in got.items()}
        rel = {k: float(((v[2] - ref[2]).abs() / ref[2].abs().clamp_min(1e-30)).max())
               for k, v in got.items()}
        bad += sum(not s for s in same.values()) + sum(r_ > 1e-5 for r_ in rel.values())
        print(json.dumps({"mode": mode, "B": B, "z_ld_bitwise_equal": same,
                          "loss_sums_max_rel_diff": rel}), flush=True)
        del r
        torch.cuda.empty_cache()
sys.exit(1 if bad else 0)
