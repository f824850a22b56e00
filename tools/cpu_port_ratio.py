"""Cost ratio of the op-for-op torch CPU port (oracle/cnf_torch_port.py, the
bench's cpu_baseline) to the reference's own flows/flows.py, on the same cores.

BUILD-CONTAINER ONLY (test/bench infrastructure): imports the reference from
/root/reference, which does not exist on the GPU box.  Same weights, same
input, torch.no_grad(), median of repeated passes; prints one JSON line.
usage: PYTHONDONTWRITEBYTECODE=1 python tools/cpu_port_ratio.py [threads] [B]
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import cnf_torch_port as P  # noqa: E402


def median_rate(fn, B, seconds=8.0):
    fn()
    ts = []
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds or len(ts) < 5:
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return B / float(np.median(ts))


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 18
    torch.set_num_threads(threads)
    sys.path.insert(0, "/root/reference")
    from flows.flows import Flow, NvpCouplingLayer  # the reference itself
    torch.manual_seed(0)
    np.random.seed(0)
    D, L, hidden = 10, 6, [5, 5]
    ref = Flow([NvpCouplingLayer(D, hidden) for _ in range(L)])
    g = torch.Generator().manual_seed(0)
    with torch.no_grad():
        for p in ref.parameters():
            if p.requires_grad:
                p.copy_(torch.randn(p.shape, generator=g) * 0.1)
    st = {k: v.detach().numpy() for k, v in ref.state_dict().items()}
    port = P.layers_from_state(st, L, len(hidden) + 1, True, True)
    x = torch.randn(B, D)
    with torch.no_grad():
        zr, ldr = ref(x)
    zp, ldp = P.flow_forward(port, x)
    assert torch.equal(zr[-1], zp[-1]) and torch.equal(ldr, ldp), "port diverged from reference"
    # interleaved rounds (reference, port, reference, ...): host noise hits both
    rounds = int(os.environ.get("CNF_RATIO_ROUNDS", "7"))
    ratios, refs, ports = [], [], []
    for _ in range(rounds):
        with torch.no_grad():
            r_ref = median_rate(lambda: ref(x), B, seconds=2.0)
        r_port = median_rate(lambda: P.flow_forward(port, x), B, seconds=2.0)
        refs.append(r_ref)
        ports.append(r_port)
        ratios.append(r_ref / r_port)
    print(json.dumps({"threads": threads, "B": B, "shape": "D=10 L=6 h=[5,5]", "rounds": rounds,
                      "reference_vec_per_s": round(float(np.median(refs))),
                      "port_vec_per_s": round(float(np.median(ports))),
                      "port_over_reference_time": round(float(np.median(ratios)), 3),
                      "ratio_min_max": [round(min(ratios), 3), round(max(ratios), 3)],
                      "bitwise_equal_outputs": True}))


if __name__ == "__main__":
    main()
