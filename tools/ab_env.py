"""A/B of environment switches in ONE process (interleaved rounds, median of 5).
Usage: python tools/ab_env.py 'CNF_SGPR_BAL=0,CNF_REDUCE4=0' 'CNF_SGPR_BAL=1' ...
Each argument is one configuration (comma-separated VAR=value); cases come
from CASES (default: cfg2 loss / forward at 1M and 8M, cfg5 inverse)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def parse(a):
    return dict(kv.split("=", 1) for kv in a.split(",") if kv)


def main():
    confs = [parse(a) for a in sys.argv[1:]] or [{}]
    keys = sorted({k for c in confs for k in c})
    dev = torch.device("cuda:0")
    W = bench.WORKLOADS
    cases = (("cfg2_loss", W["cfg2"], False, "loss"),
             ("cfg2", W["cfg2"], False, "forward"),
             ("cfg5", W["cfg5"], False, "forward"),
             ("cfg2_all", W["cfg2"], True, "forward"),
             ("cfg4", W["cfg4"], False, "forward"),
             ("cfg2_8M", dict(W["cfg2"], B=8 << 20), False, "forward"),
             ("cfg2_8M_loss", dict(W["cfg2"], B=8 << 20), False, "loss"))
    only = os.environ.get("CASES", "cfg2_loss,cfg2,cfg5,cfg2_8M,cfg2_8M_loss").split(",")
    launches = int(os.environ.get("LAUNCHES", "40"))
    for name, wl, allo, mode in cases:
        if name not in only:
            continue
        r = bench.Runner(dict(wl), dev, 1.5e9, all_outputs=allo, mode=mode)
        if mode == "loss":  # the partials area depends on the configuration's grid
            r.ws_bytes = 16 + 16 * (wl["B"] // 64 + 1)
            r.ws = torch.zeros(r.ws_bytes, dtype=torch.uint8, device=dev)
        res = [[] for _ in confs]
        for _ in range(5):
            for i, c in enumerate(confs):
                for k in keys:
                    os.environ.pop(k, None)
                os.environ.update(c)
                res[i].append(bench.kernel_only_seconds(r, launches))
        for i, c in enumerate(confs):
            t = float(np.median(res[i]))
            print("%-13s %-40s %9.2f us %8.3f Gvec/s (min %.2f)" %
                  (name, ",".join("%s=%s" % kv for kv in c.items()) or "default", t * 1e6,
                   wl["B"] / t / 1e9, min(res[i]) * 1e6), flush=True)
        del r
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
