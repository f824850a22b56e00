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

VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "1,2,4,5,6,7").split(",")]


def main():
    dev = torch.device("cuda:0")
    cases = (("cfg2_loss", bench.WORKLOADS["cfg2"], False, "loss"),
             ("cfg2", bench.WORKLOADS["cfg2"], False, "forward"),
             ("cfg5", bench.WORKLOADS["cfg5"], False, "forward"),
             ("cfg2_all", bench.WORKLOADS["cfg2"], True, "forward"),
             ("cfg2_8M", dict(bench.WORKLOADS["cfg2"], B=8 << 20), False, "forward"),
             ("cfg2_8M_loss", dict(bench.WORKLOADS["cfg2"], B=8 << 20), False, "loss"))
    only = os.environ.get("CASES")
    for name, wl, allo, mode in cases:
        if only and name not in only.split(","):
            continue
        r = bench.Runner(dict(wl), dev, 1.5e9, all_outputs=allo, mode=mode)
        if mode == "loss":  # the partials area depends on the variant's grid
            r.ws_bytes = 16 + 16 * (wl["B"] // 64 + 1)
            r.ws = torch.zeros(r.ws_bytes, dtype=torch.uint8, device=dev)
        res = {v: [] for v in VARIANTS}
        for rnd in range(5):
            for v in VARIANTS:
                if v in (97, 98, 99):  # pipelined-scalar kernel; 98/97: + LDS-DMA
                    os.environ["CNF_SGPR"] = "1"
                    os.environ["CNF_SGPR_PIPE"] = "0" if v == 99 else "1"
                    os.environ["CNF_LOSS_TICKET"] = "1" if v == 97 else "0"
                    os.environ.pop("CNF_VALU_VARIANT", None)
                else:
                    os.environ["CNF_SGPR"] = "0"
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
