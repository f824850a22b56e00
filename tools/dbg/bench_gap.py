"""Debug: the bench step's device time vs host time per call, repeated."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import bench

dev = torch.device("cuda:0")
w = dict(bench.WORKLOADS["cfg2"])
r = bench.Runner(w, dev, 1.0e9, mode="loss")
for i in range(4):
    t1, wall1 = r.timed(200, 20)
    t2, wall2 = r.timed(100, 3)
    print(json.dumps({"dev200_us": round(t1 / 200 * 1e6, 2), "host200_us": round(wall1 / 200 * 1e6, 2),
                      "dev100_us": round(t2 / 100 * 1e6, 2), "host100_us": round(wall2 / 100 * 1e6, 2)}))
