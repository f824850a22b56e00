"""A/B of kernel variants in ONE process (interleaved rounds, median):
CNF_VALU_VARIANT=i selects rows-per-lane x launch-bound variants of the
fused VALU kernel for the headline shape (cnf_valu.hip kExp)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "0,1,2,3,4").split(",")]


def main():
    dev = torch.device("cuda:0")
    for name, wl, allo in (("cfg2", bench.WORKLOADS["cfg2"], False),
                           ("cfg5", bench.WORKLOADS["cfg5"], False),
                           ("cfg2_all", bench.WORKLOADS["cfg2"], True),
                           ("cfg2_8M", dict(bench.WORKLOADS["cfg2"], B=8 << 20), False)):
        r = bench.Runner(dict(wl), dev, 1.5e9, all_outputs=allo)
        res = {v: [] for v in VARIANTS}
        for rnd in range(5):
            for v in VARIANTS:
                os.environ["CNF_VALU_VARIANT"] = str(v)
                res[v].append(bench.kernel_only_seconds(r, 40))
        for v in VARIANTS:
            t = float(np.median(res[v]))
            print("%-9s variant %d: %8.2f us  %7.3f Gvec/s  (min %.2f)" %
                  (name, v, t * 1e6, wl["B"] / t / 1e9, min(res[v]) * 1e6), flush=True)
        del r
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
