"""Kernel time vs batch size (fixed-cost vs per-row cost), plus a torch copy
of the same bytes as a memory-only reference."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for var in os.environ.get("VARIANTS", "1,4").split(","):
        os.environ["CNF_VALU_VARIANT"] = var
        for B in (1 << 17, 1 << 18, 1 << 19, 1 << 20, 1 << 21, 1 << 22, 1 << 23):
            r = bench.Runner(dict(bench.WORKLOADS["cfg2"], B=B), dev, 1.5e9)
            t = float(np.median([bench.kernel_only_seconds(r, 30) for _ in range(3)]))
            print("variant %s B=%8d  %9.2f us  %7.3f Gvec/s  %.2f ns/1k rows" %
                  (var, B, t * 1e6, B / t / 1e9, t * 1e9 / (B / 1000)), flush=True)
            del r
            torch.cuda.empty_cache()
    for B in (1 << 20, 1 << 23):
        src = torch.empty(B * 10, device=dev)
        dst = torch.empty(B * 11, device=dev)
        for _ in range(3):
            dst[:B * 10].copy_(src)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(30):
            dst[:B * 10].copy_(src)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 30 / 1e3
        print("copy %d x 40B: %.2f us  %.1f GB/s" % (B, t * 1e6, B * 80 / t / 1e9))


if __name__ == "__main__":
    main()
