import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, bench
r = bench.train_step_rate(torch.device("cuda:0"))
print(json.dumps({"lib": os.path.basename(os.environ.get("CNF_HIP_LIB", "libcnf_hip.so")), "ms": r["ms_per_step"]}))
