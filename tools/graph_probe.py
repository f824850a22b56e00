"""Does graph replay shorten the cfg2 loss step (k_sgpr + the reduction
launch)?  The same Runner steps eager on the stream vs captured once into a
HIP graph of N steps and replayed; HIP-event time per step, interleaved."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
N = 100
r = bench.Runner(dict(bench.WORKLOADS["cfg2"]), dev, 1.0e9, mode="loss")
s = torch.cuda.Stream(dev)
r.stream = s
with torch.cuda.stream(s):
    r.settle(0.3)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(N):
            r.step()
    torch.cuda.synchronize()
    res = {"eager_us": [], "graph_us": []}
    for _ in range(7):
        for mode in ("eager", "graph"):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            if mode == "graph":
                g.replay()
            else:
                for _ in range(N):
                    r.step()
            e1.record(s)
            torch.cuda.synchronize()
            res[mode + "_us"].append(round(e0.elapsed_time(e1) * 1e3 / N, 3))
print(json.dumps(res))
