"""Per-block timeline of the persistent k_sgpr launch (diagnostic build
libcnf_hip_tl.so, `make -C calibration-normalizing-flows_amd/csrc timeline`).
Prints, relative to the earliest block start (us): start / first-tile-ready /
end percentiles, per-XCD spans, and the span vs the HIP-event launch time.
Usage: python tools/timeline.py [B] [mode]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["CNF_HIP_LIB"] = os.path.join(ROOT, "calibration-normalizing-flows_amd", "cnf_hip",
                                         "libcnf_hip_tl.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    mode = sys.argv[2] if len(sys.argv) > 2 else "forward"
    dev = torch.device("cuda:0")
    r = bench.Runner(dict(bench.WORKLOADS["cfg2"], B=B), dev, 1.5e9, mode=mode)
    t_ev = bench.kernel_only_seconds(r, 40)
    lib = r.lib
    lib.cnf_diag_timeline.restype = ctypes.c_int
    nblk = None
    spans = []
    for rep in range(5):
        r.step()
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (4096 * 4))()
        n = lib.cnf_diag_timeline(buf, 4096 * 4)
        a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 4)
        used = a[:, 0] != 0
        if nblk is None:
            nblk = int(used.sum())
        a = a[:nblk].astype(np.int64)
        t0 = a[:, 0].min()
        st, rd, en = [(a[:, k] - t0) / 100.0 for k in range(3)]  # 100 MHz -> us
        xcc = (a[:, 3] >> 32) & 0xF
        spans.append(en.max())
        if rep == 4:
            pct = lambda v: " ".join("%6.2f" % np.percentile(v, p) for p in (0, 10, 50, 90, 100))
            print("B=%d mode=%s blocks=%d  event-timed launch %.2f us" % (B, mode, nblk,
                                                                          t_ev * 1e6))
            print("percentiles          p0     p10    p50    p90    p100")
            print("start         ", pct(st))
            print("first ready   ", pct(rd))
            print("ready-start   ", pct(rd - st))
            print("end           ", pct(en))
            print("end-ready     ", pct(en - rd))
            for x in range(8):
                m = xcc == x
                if m.any():
                    print("xcc %d: %4d blocks start %.2f..%.2f  end %.2f..%.2f" %
                          (x, m.sum(), st[m].min(), st[m].max(), en[m].min(), en[m].max()))
            hist, edges = np.histogram(en, bins=20)
            print("end histogram:", " ".join("%.1f:%d" % (e, h) for e, h in zip(edges, hist)))
            # memrealtime is written before the tail stores drain: span is a floor
            print("in-kernel span (max end - min start): %.2f us, reps %s" %
                  (en.max(), " ".join("%.2f" % s for s in spans)))
        r.w["B"] = B


if __name__ == "__main__":
    main()
