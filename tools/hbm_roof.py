"""Practical HBM rates on this MI355X with stock torch kernels (no cnf code):
write-only (fill_), read-only (sum), read+write (copy_) over 1 GiB buffers,
for pricing the write-heavy every-layer-output pass (k_valu) against what the
memory system sustains, beside the 8 TB/s datasheet peak."""
import json

import torch

dev = torch.device("cuda:0")
n = (1 << 30) // 4
a = torch.empty(n, device=dev)
b = torch.empty(n, device=dev)
a.normal_()


def rate(fn, bytes_moved, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return bytes_moved * reps / (e0.elapsed_time(e1) / 1e3) / 1e9


out = {"buffer_GiB": 1,
       "write_GBs": round(rate(lambda: b.fill_(1.0), 4 * n), 1),
       "read_GBs": round(rate(lambda: a.sum(), 4 * n), 1),
       "copy_GBs": round(rate(lambda: b.copy_(a), 8 * n), 1)}
print(json.dumps(out), flush=True)
