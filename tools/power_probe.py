"""Board power and clocks while the cfg2 bench pass runs back to back: is the
device at its power cap (the shader clock then falls as memory traffic is
added, tools/sgpr_trace.py clock_ghz)?  Samples `rocm-smi` (read-only) idle
and under load.  usage: power_probe.py [loss|forward|train|train4] [seconds] [B]
(train / train4: the fused calibrator step, cnf_loss_vjp + reduction, on cfg2 /
cfg4)."""
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "loss"
secs = float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
B = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20


def smi():
    try:
        out = subprocess.run(["rocm-smi", "--showpower", "--showmaxpower", "--showclocks", "--json"],
                             capture_output=True, text=True, timeout=30).stdout
        return json.loads(out)
    except Exception as e:  # noqa: BLE001
        return {"error": str(e)}


dev = torch.device("cuda:0")
if mode in ("train", "train4"):
    from cnf_hip import vjp as V
    if mode == "train4" and B == 1 << 20:
        B = bench.WORKLOADS["cfg4"]["B"]

    class _Train:
        def __init__(self):
            w = bench.WORKLOADS["cfg2" if mode == "train" else "cfg4"]
            self.stack = bench.make_flow(w, dev)._native_stack()
            self.x, self.y = bench.synthetic_logits(B, w["D"], dev, 4321)

        def step(self):
            V.loss_and_grads(self.stack, self.x, self.y, grad_scale=1.0 / B)

    r = _Train()
else:
    r = bench.Runner(dict(bench.WORKLOADS["cfg2"], B=B), dev, 1.0e9, mode=mode)
res = {"lib": os.path.basename(os.environ.get("CNF_HIP_LIB", "libcnf_hip.so")), "mode": mode,
       "B": B, "idle": smi()}
stop = threading.Event()
samples = []


def sampler():
    time.sleep(1.0)
    while not stop.is_set():
        samples.append(smi())
        time.sleep(0.5)


th = threading.Thread(target=sampler)
th.start()
t0 = time.perf_counter()
t_end = t0 + secs
n = 0
per = {"train": max(1, (25 << 20) // B), "train4": 4}.get(mode, max(1, (200 << 20) // B))
while time.perf_counter() < t_end:
    for _ in range(per):
        r.step()
    n += per
    torch.cuda.synchronize()
el = time.perf_counter() - t0
stop.set()
th.join()


def num(d, key):
    for card in d.values():
        if isinstance(card, dict):
            for k, v in card.items():
                if key in k:
                    return float(str(v).strip("()Mhz"))
    return None


pw = [num(s_, "Current Socket Graphics Package Power") for s_ in samples]
pw = [p for p in pw if p is not None]
sclk = [num(s_, "sclk clock speed") for s_ in samples]
sclk = [c for c in sclk if c is not None]
us = el / n * 1e6
res["us_per_step"] = round(us, 2)
res["power_w"] = round(sum(pw) / len(pw), 1) if pw else None
res["sclk_mhz"] = round(sum(sclk) / len(sclk)) if sclk else None
res["idle_w"] = num(res["idle"], "Current Socket Graphics Package Power")
if pw:
    res["nJ_per_row"] = round(res["power_w"] * us * 1e-6 / B * 1e9, 3)
    res["nJ_per_row_above_idle"] = round((res["power_w"] - res["idle_w"]) * us * 1e-6 / B * 1e9, 3)
del res["idle"]
print(json.dumps(res))
