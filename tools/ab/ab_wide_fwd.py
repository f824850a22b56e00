"""A/B of experimental k_wide16 builds (CNF_HIP_LIB=<lib>.so): cfg4 forward,
inverse and predict kernel time (2^18 rows, ctypes path straight into the
library) and output checksums, one JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from cnf_hip import _lib  # noqa: E402
from cnf_hip.engine import _ptr, _stream  # noqa: E402

dev = torch.device("cuda:0")
w = bench.WORKLOADS["cfg4"]
stack = bench.make_flow(w, dev)._native_stack()
B = w["B"]
x, _ = bench.synthetic_logits(B, w["D"], dev, 4321)
blob = stack.prepared(dev)
lib = _lib.lib()
out = torch.empty_like(x)
ld = torch.empty(B, device=dev)
lp = torch.log_softmax(torch.randn(w["D"], device=dev), 0)


def call(kind):
    if kind == "predict":
        st = lib.cnf_predict(ctypes.byref(stack.desc), _ptr(blob), _ptr(x), _ptr(lp), _ptr(out),
                             _ptr(ld), ctypes.c_int64(B), _stream(dev))
    else:
        fn = lib.cnf_inverse if kind == "inverse" else lib.cnf_forward
        st = fn(ctypes.byref(stack.desc), _ptr(blob), _ptr(x), _ptr(out), _ptr(ld), None,
                ctypes.c_int64(B), _stream(dev))
    _lib.check(kind, st)


res = {"lib": os.path.basename(os.environ.get("CNF_HIP_LIB", "libcnf_hip.so"))}
for kind in ("forward", "inverse", "predict"):
    for _ in range(5):
        call(kind)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(30):
        call(kind)
    e1.record()
    torch.cuda.synchronize()
    res[kind + "_us"] = round(e0.elapsed_time(e1) * 1e3 / 30, 1)
    res[kind + "_sum"] = [float(out.double().sum()), float(out.double().abs().sum()),
                          float(ld.double().sum())]
print(json.dumps(res), flush=True)
