"""Per-wave timeline of one k_sgpr launch (diagnostic build: `make -C
calibration-normalizing-flows_amd/csrc trace`, loaded via CNF_HIP_LIB).
Prints quantiles (us, from the first wave's start) of each mark, and the
per-SIMD picture: tiles owned vs finishing time, per XCD (HW_ID / XCC_ID
fields of the gfx9 hardware-id registers, as recorded in mark 7)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CNF_HIP_LIB", os.path.join(ROOT, "calibration-normalizing-flows_amd",
                                                  "cnf_hip", "libcnf_hip_trace.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from cnf_hip import _lib  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "loss"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
w = dict(bench.WORKLOADS["cfg2"], B=B)
r = bench.Runner(w, torch.device("cuda:0"), 0.5e9, all_outputs=(mode == "all"),
                 mode="loss" if mode == "loss" else "forward")
import time  # noqa: E402
t_end = time.perf_counter() + 2.0  # >= 2 s of back-to-back launches: the clock settles
while time.perf_counter() < t_end:
    for _ in range(50):
        r.step()
    torch.cuda.synchronize()
for _ in range(20):
    r.step()
torch.cuda.synchronize()
lib = _lib.lib()
n = 16384 * 8
buf = (ctypes.c_ulonglong * n)()
lib.cnf_diag_trace.restype = ctypes.c_int
assert lib.cnf_diag_trace(buf, n) == n
raw = np.frombuffer(buf, dtype=np.uint64).reshape(16384, 8)
cbuf = (ctypes.c_ulonglong * (16384 * 2))()
lib.cnf_diag_trace_clk.restype = ctypes.c_int
assert lib.cnf_diag_trace_clk(cbuf, 16384 * 2) == 16384 * 2
clk = np.frombuffer(cbuf, dtype=np.uint64).reshape(16384, 2).astype(np.float64)
a = raw.astype(np.float64)
ntiles = (B + 127) // 128
nw = int((a[:, 0] > 0).sum())
a = a[:nw]
raw = raw[:nw]
clk = clk[:nw]
# in-kernel shader clock per wave: memtime ticks over realtime ticks (100 MHz)
dt_real = a[:, 6] - a[:, 0]
ok = (dt_real > 0) & (clk[:, 1] > clk[:, 0])
ghz = (clk[ok, 1] - clk[ok, 0]) / dt_real[ok] * 0.1
t0 = a[:, 0].min()
us = lambda v: (v - t0) / 100.0  # 100 MHz
q5 = lambda v: [round(float(np.quantile(v, q)), 2) for q in (0, 0.1, 0.5, 0.9, 1.0)]
out = {"B": B, "waves": nw, "mode": mode,
       "clock_ghz": [round(float(np.quantile(ghz, q)), 3) for q in (0.1, 0.5, 0.9)] if len(ghz) else None}
names = ["start", "tile0_data", "tile0_done", "tile1_data", "tile1_done", "last_done", "end"]
for i, nm in enumerate(names):
    v = a[:, i]
    v = v[v > 0]
    if len(v):
        out[nm] = q5(us(v))
d0 = (a[:, 2] - a[:, 1]) / 100.0
out["tile_compute_us"] = [round(float(np.quantile(d0[a[:, 2] > 0], q)), 2) for q in (0.1, 0.5, 0.9)]

# per-SIMD: tiles owned by its waves (static walk t = gw, gw + nw, ...) and the
# time its last wave ended
hw = (raw[:, 7] & 0xffffffff).astype(np.int64)
xcc = ((raw[:, 7] >> 32) & 0xf).astype(np.int64)
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
gw = np.arange(nw)
tiles = np.where(gw < ntiles, (ntiles - 1 - gw) // nw + 1, 0)
end = us(a[:, 6])
start = us(a[:, 0])
ks, inv = np.unique(key, return_inverse=True)
n_s = len(ks)
t_s = np.bincount(inv, weights=tiles, minlength=n_s)
w_s = np.bincount(inv, minlength=n_s)
e_s = np.full(n_s, 0.0)
np.maximum.at(e_s, inv, end)
out["simds"] = n_s
out["waves_per_simd"] = {int(k): int(v) for k, v in zip(*np.unique(w_s, return_counts=True))}
out["tiles_per_simd"] = {int(k): int(v) for k, v in zip(*np.unique(t_s, return_counts=True))}
out["simd_end_us"] = q5(e_s)
for tv in np.unique(t_s):
    sel = t_s == tv
    out["simd_end_us_at_%d_tiles" % int(tv)] = q5(e_s[sel])
out["corr_tiles_end"] = round(float(np.corrcoef(t_s, e_s)[0, 1]), 3) if n_s > 2 else None
cu_key = key // 4
out["cus"] = int(len(np.unique(cu_key)))
out["per_xcc_end_us_median"] = {int(x): round(float(np.median(end[xcc == x])), 2)
                                for x in np.unique(xcc)}
out["per_xcc_start_us_median"] = {int(x): round(float(np.median(start[xcc == x])), 2)
                                  for x in np.unique(xcc)}
# start time of the waves by block index decile: how fast the dispatcher fills
blk = gw // 4
dec = np.minimum((blk * 10) // max(1, blk.max() + 1), 9)
out["start_us_by_block_decile"] = [round(float(np.median(start[dec == d])), 2) for d in range(10)]
# wave start / first data / end by the block's dispatch slot on its CU (0 =
# the CU's first block): how late the dispatcher places each resident block
blk_of = gw // 4
slot = np.zeros(nw, dtype=np.int64)
for k in np.unique(cu_key):
    bs = np.unique(blk_of[cu_key == k])
    for rnk, bb in enumerate(bs):
        slot[blk_of == bb] = rnk
out["by_cu_slot"] = {int(r): {"start": round(float(np.median(start[slot == r])), 2),
                             "data": round(float(np.median(us(a[slot == r, 1]))), 2),
                             "end": round(float(np.median(end[slot == r])), 2)}
                     for r in np.unique(slot)}
print(json.dumps(out))
if os.environ.get("CNF_TRACE_DUMP"):  # raw marks for offline analysis
    np.savez_compressed(os.environ["CNF_TRACE_DUMP"], marks=raw, clk=clk, B=B)
