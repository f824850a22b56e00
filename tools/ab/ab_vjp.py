"""A/B of experimental k_vjp2 builds (CNF_HIP_LIB=libcnf_hip_<v>.so): cfg2
training-step time at 2^20 rows and a gradient checksum, one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from cnf_hip import vjp as V  # noqa: E402

dev = torch.device("cuda:0")
w = bench.WORKLOADS["cfg2"]
flow = bench.make_flow(w, dev)
x, y = bench.synthetic_logits(1 << 20, w["D"], dev, 4321)
terms, g, _ = V.loss_and_grads(flow._native_stack(), x, y, grad_scale=1.0 / (1 << 20))
r = bench.train_step_rate(dev)
print(json.dumps({"lib": os.path.basename(os.environ.get("CNF_HIP_LIB", "libcnf_hip.so")),
                  "ms": r["ms_per_step"], "terms": terms.tolist(),
                  "gsum": float(g.double().sum()), "gabs": float(g.double().abs().sum())}),
      flush=True)
