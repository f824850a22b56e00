"""Loss-term check of an experimental library build (CNF_HIP_LIB=...): the
cfg2 fused eval's (loss, ce, ld) sums over 2^20 rows against an fp64 sum of
the same kernel's per-row outputs (z, ld) run through the reference's loss
formula (calibrators.py:288-291), on 8 different inputs, each launched 50
times back to back: every launch must give the same bits (deterministic
block-order sum) and the fp64 value to 2e-6 relative.  Catches a stale read
in an in-launch hand-off (a wrong or varying sum)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
w = dict(bench.WORKLOADS["cfg2"])
r = bench.Runner(w, dev, 0.0, mode="loss")
res = {"lib": os.path.basename(os.environ.get("CNF_HIP_LIB", "libcnf_hip.so")), "ok": True}
worst = 0.0
for i in range(8):
    x, y = bench.synthetic_logits(w["B"], w["D"], dev, 777 + i)
    z, ld, _ = r.sets[0][2], r.sets[0][3], None
    r.sets[0] = (x, y, z, ld, None)
    P = __import__("ctypes").c_void_p
    r.args[0] = (P(x.data_ptr()), P(z.data_ptr()), P(ld.data_ptr()), P(0), P(y.data_ptr()))
    got = []
    for _ in range(50):
        r.i = 0
        r.step()
        got.append(r.terms.clone())
    torch.cuda.synchronize()
    g = torch.stack(got)
    if not bool((g == g[0]).all()):
        res["ok"] = False
        res["nondeterministic_input"] = i
    zz, ll = z.double(), ld.double()
    p = torch.softmax(zz, 1).gather(1, y.view(-1, 1)).squeeze(1)
    ce = -torch.log(p + 1e-7)
    ref = torch.stack([(ce - ll).sum(), ce.sum(), ll.sum()])
    err = ((g[0].double() - ref).abs() / (ref.abs() + 1)).max().item()
    worst = max(worst, err)
res["worst_rel"] = worst
res["ok"] = res["ok"] and worst <= 2e-6
print(json.dumps(res))
