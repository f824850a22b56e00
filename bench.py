"""Benchmark of the coupling-flow hot path on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 6-layer RealNVP affine
coupling, D=10 logits, conditioner hidden_size=[5,5] (reference default,
flows/flows.py:71), B=2^20 synthetic logit vectors per GPU, fp32.  One step =
one fused forward + per-sample log-det pass over one batch that also reduces
the batch's calibration NLL (cnf_forward_loss through the C ABI: writes the
final z [B,10] and log-det [B], and the sums of the per-row loss / ce / ld --
the eval pass of TorchFlowCalibrator.fit, calibrators.py:297-317).  With N>1
ranks every rank runs its own 2^20-vector shard (weak scaling: 8M vectors at
N=8 = configs[2]) and every batch's 3 NLL sums are summed across ranks by RCCL
over xGMI (configs[2]), bucketed: the sums of NLL_BUCKET consecutive batches
go in one all-reduce (a 12-B all-reduce is pure latency, ~14 us even on one
rank, half a step), the last partial bucket before the timed region closes;
at N=1 there is nothing to reduce.

Inputs are resident in HBM before timing; the step rotates through enough
distinct input/output buffers (>= --rotate-gb) that the 256 MB Infinity Cache
cannot serve repeated launches.  Timing: HIP events on the launch stream
around exactly --steps steps, barrier + synchronize on both sides, max over
ranks.  Rank 0 prints one JSON line.
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "calibration-normalizing-flows_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md chip table (spec)
VALU_PEAK_TFLOPS = 157.3  # FP32 vector peak (spec)
MFMA_F32_PEAK_TFLOPS = 157.3

WORKLOADS = {
    # name: (D, L, hidden, B per GPU, inverse)
    "cfg1": dict(D=3, L=2, hidden=[5, 5], B=4096, scale=False, inverse=False),
    "cfg2": dict(D=10, L=6, hidden=[5, 5], B=1 << 20, scale=True, inverse=False),
    # cfg4: the reference's own Linear init (N(0, 0.1) on 100-wide Linears
    # overflows exp(s) within a few layers: inf / NaN everywhere)
    "cfg4": dict(D=100, L=12, hidden=[100, 100], B=1 << 18, scale=True, inverse=False,
                 sigma=None),
    "cfg5": dict(D=10, L=6, hidden=[5, 5], B=1 << 20, scale=True, inverse=True),
}


def algo_flops_per_vec(D, L, hidden, scale=True):
    """mask-reduced MACs, 2 flops each, + elementwise."""
    dt, dc = D // 2, D - D // 2
    units = [dc] + list(hidden) + [dt]
    macs = sum(a * b for a, b in zip(units[:-1], units[1:]))
    nets = 2 if scale else 1
    per_layer = nets * 2 * macs + (3 * dt if scale else dt)
    return L * per_layer


def algo_bytes_per_vec(D, L, all_outputs=False, labels=False):
    """x in, z out (every layer's z with all_outputs), log-det out, int64 label in."""
    return 4 * D + 4 * D * (L if all_outputs else 1) + 4 + (8 if labels else 0)


def roofline(B, bytes_vec, flops_vec, seconds, mfma=False):
    """Roofline of one launch over B vectors: the attainable rate
    is min(HBM peak / bytes, compute peak / flops); `bound` names the roof that
    binds first and `frac` = achieved rate / attainable rate.  Compute is fp32
    VALU (packed FMA) for the narrow flows, fp32 MFMA for the wide ones."""
    comp_peak = MFMA_F32_PEAK_TFLOPS if mfma else VALU_PEAK_TFLOPS
    hbm_rate = HBM_PEAK_GBS * 1e9 / bytes_vec          # vectors/s if HBM-bound
    comp_rate = comp_peak * 1e12 / flops_vec           # vectors/s if compute-bound
    rate = B / seconds
    gbs = B * bytes_vec / seconds / 1e9
    tfs = B * flops_vec / seconds / 1e12
    if comp_rate <= hbm_rate:
        r = {"bound": "mfma" if mfma else "valu", "achieved": round(tfs, 2),
             "peak": comp_peak, "unit": "TFLOP/s"}
    else:
        r = {"bound": "hbm", "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s"}
    r["frac"] = round(rate / min(hbm_rate, comp_rate), 4)
    r["hbm_gbs"] = round(gbs, 2)
    r["hbm_frac"] = round(gbs / HBM_PEAK_GBS, 4)
    r["compute_tflops"] = round(tfs, 2)
    r["compute_frac"] = round(tfs / comp_peak, 4)
    return r


def make_flow(w, device, seed=0):
    from flows.flows import Flow, NvpCouplingLayer
    torch.manual_seed(seed)
    np.random.seed(seed)
    flow = Flow([NvpCouplingLayer(w["D"], w["hidden"], scale=w["scale"]) for _ in range(w["L"])])
    g = torch.Generator().manual_seed(seed)
    sigma = w.get("sigma", 0.1)
    with torch.no_grad():
        for p in flow.parameters():
            if p.requires_grad and sigma is not None:  # N(0, 0.1): SURVEY 8(d) synthetic weights
                p.copy_(torch.randn(p.shape, generator=g) * sigma)
    return flow.to(device)


def synthetic_logits(B, D, device, seed):
    """x = 2*onehot(y) + N(0,1), rows mean-centred (calibrators.py:17)."""
    g = torch.Generator(device=device).manual_seed(seed)
    x = torch.randn(B, D, device=device, generator=g)
    y = torch.randint(0, D, (B,), device=device, generator=g)
    x[torch.arange(B, device=device), y] += 2.0
    return x - x.mean(dim=1, keepdim=True), y


class Runner:
    """Pre-built C-ABI launches of one fused pass over rotating buffers.
    mode: "forward" (cnf_forward / cnf_inverse), "loss" (cnf_forward_loss)."""

    def __init__(self, w, device, rotate_bytes, all_outputs=False, mode="forward", data=None):
        from cnf_hip import _lib
        self.w = w
        self.dev = device
        self.flow = make_flow(w, device)
        self.stack = self.flow._native_stack()
        self.blob = self.stack.prepared(device)
        self.lib = _lib.lib()
        B, D, L = w["B"], w["D"], w["L"]
        self.mode = mode
        per_set = algo_bytes_per_vec(D, L, all_outputs, mode == "loss") * B
        # data: one caller-given (x [B, D], y [B]) set instead of rotating
        # synthetic ones (the sharded-eval test feeds each rank its shard)
        self.nsets = 1 if data is not None else max(1, min(64, math.ceil(rotate_bytes / per_set)))
        self.sets = []
        for i in range(self.nsets):
            x, y = data if data is not None else synthetic_logits(B, D, device, 1234 + i)
            ld = torch.empty(B, device=device)
            if all_outputs:
                out, allt = None, torch.empty(L, B, D, device=device)
            else:
                out, allt = torch.empty(B, D, device=device), None
            self.sets.append((x, y, out, ld, allt))
        self.fn = self.lib.cnf_inverse if w["inverse"] else self.lib.cnf_forward
        self.desc = ctypes.byref(self.stack.desc)
        P = ctypes.c_void_p
        vp = lambda t: P(t.data_ptr()) if t is not None else P(0)
        self.stream = torch.cuda.current_stream(device)
        self.args = [(vp(x), vp(out), vp(ld), vp(allt), vp(y)) for (x, y, out, ld, allt) in
                     self.sets]
        # loss-term buckets: batch i writes its sums to row i % NLL_BUCKET of
        # bucket (i // NLL_BUCKET) % 2 (two, so an overlapped all-reduce of one
        # bucket can run while the next fills); NllAllReduce reduces whole buckets
        # be in flight while batch i+1's kernel writes the next buffer
        self.term_bufs = torch.zeros(2, NLL_BUCKET, 3, device=device)
        self.terms = self.term_bufs[0, 0]
        if mode == "loss":
            n = ctypes.c_size_t()
            st = self.lib.cnf_forward_loss_workspace_bytes(self.desc, ctypes.c_int64(B),
                                                           ctypes.byref(n))
            if st != 0:
                raise RuntimeError("cnf_forward_loss unsupported for this shape: %d" % st)
            self.ws = torch.zeros(max(n.value, 16), dtype=torch.uint8, device=device)
            self.ws_bytes = n.value
        self.i = 0

    def kernel_symbol(self):
        return {"valu-fused": "k_valu", "sgpr-fused": "k_sgpr", "mfma-tile": "k_tile",
                "mfma-wide": "k_wide16"}.get(
            self.stack.kernel_name(), self.stack.kernel_name())

    def step(self):
        a = self.args[self.i % self.nsets]
        self.terms = self.term_bufs[(self.i // NLL_BUCKET) % 2, self.i % NLL_BUCKET]
        self.i += 1
        blob = ctypes.c_void_p(self.blob.data_ptr())
        stream = ctypes.c_void_p(self.stream.cuda_stream)
        if self.mode == "loss":
            st = self.lib.cnf_forward_loss(self.desc, blob, a[0], a[4], ctypes.c_int32(0),
                                           ctypes.c_float(1.0), a[1], a[2],
                                           ctypes.c_void_p(self.terms.data_ptr()),
                                           ctypes.c_int64(self.w["B"]),
                                           ctypes.c_void_p(self.ws.data_ptr()),
                                           ctypes.c_size_t(self.ws_bytes), stream)
        else:
            st = self.fn(self.desc, blob, a[0], a[1], a[2], a[3], ctypes.c_int64(self.w["B"]),
                         stream)
        if st != 0:
            raise RuntimeError("cnf launch failed: %d" % st)

    def settle(self, seconds):
        """Untimed steps until the device has run for `seconds` (the clock ramp
        and first touch of the rotating sets: a 2^20-row loss step measured
        36.3 us right after 20 warmup steps and 32.0 us once settled); returns
        the number of steps run."""
        n = 0
        t0 = time.perf_counter()
        while True:
            for _ in range(32):
                self.step()
            n += 32
            torch.cuda.synchronize(self.dev)
            if time.perf_counter() - t0 >= seconds:
                return n

    def timed(self, steps, warmup, collective=None):
        if collective:
            collective.realign()
        for _ in range(warmup):
            self.step()
            if collective:
                collective()
        if collective:
            collective.drain()
        torch.cuda.synchronize(self.dev)
        if dist.is_initialized():
            dist.barrier()
        torch.cuda.synchronize(self.dev)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(self.stream)
        t0 = time.perf_counter()
        for _ in range(steps):
            self.step()
            if collective:
                collective()
        if collective:
            collective.drain()  # every batch's all-reduce completes inside the timed region
        e1.record(self.stream)
        torch.cuda.synchronize(self.dev)
        wall = time.perf_counter() - t0
        if dist.is_initialized():
            dist.barrier()
        torch.cuda.synchronize(self.dev)
        return e0.elapsed_time(e1) / 1e3, wall


NLL_BUCKET = 50  # batches per NLL all-reduce (bench.py --nll-bucket)


class NllAllReduce:
    """The one real exchange of the sharded eval (configs[2]): every batch's
    (loss, ce, ld) sums, written by the fused kernel into its row of the
    runner's current bucket, summed across ranks by RCCL -- one all-reduce per
    full bucket of NLL_BUCKET batches (and one for the last partial bucket in
    drain()), so every batch's global sums exist once its bucket is reduced.
    A 12-B all-reduce per batch is all latency: measured on one MI355X (bench
    --dist-check, one rank) 46.2 us per step against ~32 us without it.
    overlap=True runs each bucket's all-reduce on RCCL's own stream (async_op)
    while the other bucket fills; the launch stream waits for it before that
    bucket is written again.  (Per batch and overlapped it measured 63.9 us per
    step on one rank: two cross-stream waits per batch.)"""

    def __init__(self, runner, overlap=False):
        self.runner = runner
        self.overlap = overlap
        self.pending = {}
        self.done = 0  # batches whose sums have been handed to an all-reduce

    def _reduce(self, b, n):
        t = self.runner.term_bufs[b, :n]
        if not self.overlap:  # the launch stream waits for it
            dist.all_reduce(t)
            return
        self.pending[b] = dist.all_reduce(t, async_op=True)

    def realign(self):
        """Start a bucket boundary at the runner's next batch: settle() and
        kernel_only_seconds() launch batches without the collective, so the
        batch counter need not sit on a bucket boundary when a collective run
        starts (rows of the partial bucket would then be reduced twice or not
        at all).  Outstanding all-reduces are waited for first."""
        for w in self.pending.values():
            w.wait()
        self.pending = {}
        r = self.runner
        r.i = -(-r.i // NLL_BUCKET) * NLL_BUCKET
        self.done = r.i

    def __call__(self):
        i = self.runner.i  # batches launched so far
        b = (i // NLL_BUCKET) % 2
        if b in self.pending and i % NLL_BUCKET == 0:
            self.pending.pop(b).wait()  # bucket b is about to be refilled
        if i % NLL_BUCKET == 0:  # a bucket just filled
            self._reduce((i // NLL_BUCKET - 1) % 2, NLL_BUCKET)
            self.done = i

    def drain(self):
        i = self.runner.i
        if i > self.done:  # the partial bucket (done sits on a bucket boundary)
            assert self.done % NLL_BUCKET == 0 and i - self.done < NLL_BUCKET
            self._reduce((i // NLL_BUCKET) % 2, i - self.done)
            self.done = i
        for w in self.pending.values():
            w.wait()
        self.pending = {}
        self.realign()  # the next batch starts a fresh bucket


def kernel_only_seconds(runner, launches):
    """Average device time per launch over `launches` back-to-back launches
    (HIP events on the launch stream, no collective in between)."""
    t, _ = runner.timed(launches, 3)
    return t / launches


def train_step_rate(dev, workload="cfg2", B=None, steps=20):
    """Fused calibrator training step (cnf_loss_vjp: forward + loss + reverse
    mode + fixed-order gradient reduction) on a workload's shape: vectors/s.
    Algorithmic training flops = 3x the forward's (forward, input gradients,
    weight gradients); the reverse mode's recompute is not counted."""
    from cnf_hip import vjp as V
    w = WORKLOADS[workload]
    B = B or w["B"]
    flow = make_flow(w, dev)
    stack = flow._native_stack()
    x, y = synthetic_logits(B, w["D"], dev, 4321)
    # untimed steps until the device has run ~0.3 s (the clock ramp, as
    # Runner.settle): 3 warmup steps timed 0.2007 ms per cfg2 step, the same
    # step back to back 0.179 ms at 2.39 GHz (tools/power_probe.py train)
    t0 = time.perf_counter()
    while True:
        for _ in range(8):
            V.loss_and_grads(stack, x, y, grad_scale=1.0 / B)
        torch.cuda.synchronize(dev)
        if time.perf_counter() - t0 >= 0.3:
            break
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        V.loss_and_grads(stack, x, y, grad_scale=1.0 / B)
    e1.record()
    torch.cuda.synchronize(dev)
    t = e0.elapsed_time(e1) / 1e3 / steps
    tf = 3 * algo_flops_per_vec(w["D"], w["L"], w["hidden"], w["scale"]) * B / t / 1e12
    peak = MFMA_F32_PEAK_TFLOPS if w["D"] >= 32 else VALU_PEAK_TFLOPS
    return {"vec_per_s": round(B / t, 1), "ms_per_step": round(t * 1e3, 4), "B": B,
            "tflops": round(tf, 2), "frac": round(tf / peak, 4),
            "note": "forward + calibrator loss + VJP + gradient reduction; optimizer excluded"}


def calibrator_epoch_rate(dev, epochs=400, cpu_epochs=20):
    """SURVEY 8(f) rank 1, the real workload: one TorchFlowCalibrator.fit epoch
    at the notebook's shape (notebooks/simulated-predictions-flows.ipynb
    L165, L213-215: RealNVP, 5 layers, hidden [3, 3], N = 1,500 3-class logits,
    full batch; the reference's 188.3 s / 5,000 epochs = 37.7 ms per epoch on
    an undocumented CPU).  Native: the fused kernels with every chunk of 50
    epochs replayed as one HIP graph, and the same epochs eager; CPU: the
    reference's own loop (calibrators._fit_torch, its DataLoader and autograd)
    on this host's cores."""
    import calibrators as C
    from flows.realNVP_torch import RealNvpFlow
    N, D = 1500, 3
    rs = np.random.RandomState(5)
    y = rs.randint(0, D, size=N)
    x = rs.standard_normal((N, D)) + 3.0 * np.eye(D)[y]
    out = {"N": N, "D": D, "layers": 5, "hidden_size": [3, 3], "batch": "full (N)",
           "reference_ms_per_epoch_notebook": 37.67}

    def timed(dev_, n_ep, graph):
        torch.manual_seed(0)
        cal = C.TorchFlowCalibrator(RealNvpFlow, x, y, layers=5, hidden_size=[3, 3], epochs=2,
                                    dev=torch.device(dev_), cnf_graph=graph)
        cal.fit(cal.logits, cal.target, epochs=2, batch_size=N)  # warm caches / graph pool
        if dev_ != "cpu":
            torch.cuda.synchronize(dev_)
        t = time.perf_counter()
        h = cal.fit(cal.logits, cal.target, epochs=n_ep, batch_size=N)
        float(h["loss"][-1])  # the history is device-resident: one sync at the end
        return (time.perf_counter() - t) / n_ep * 1e3

    out["native_graph_ms_per_epoch"] = round(timed(dev, epochs, True), 4)
    out["native_eager_ms_per_epoch"] = round(timed(dev, max(50, epochs // 4), False), 4)
    # tiny ops: one thread is usually fastest (37.7 ms/epoch on one build-container
    # core, the notebook's own figure); report the better of 1 and all threads
    nt = torch.get_num_threads()
    best = None
    for th in sorted({1, nt}):
        torch.set_num_threads(th)
        ms = timed("cpu", cpu_epochs, False)
        if best is None or ms < best[0]:
            best = (ms, th)
    torch.set_num_threads(nt)
    # the op-for-op CPU restatement of the reference's fit loop (_fit_torch:
    # DataLoader + autograd + torch Adam) -- the port, not the reference itself
    out["cpu_port_loop_ms_per_epoch"] = round(best[0], 3)
    out["cpu_threads"] = best[1]
    out["speedup_graph_vs_cpu"] = round(out["cpu_port_loop_ms_per_epoch"] /
                                        out["native_graph_ms_per_epoch"], 1)
    return out


def measured_traffic(workload, B, mode):
    """HBM bytes per launch of the bench kernel from the committed PMC summary
    (profiles/<round>_traffic_<workload>_<mode>.json, written by
    tools/pmc_traffic.py from rocprofv3 FETCH_SIZE / WRITE_SIZE passes,
    gfx950-corrected; tools/collect_profiles.sh), newest round first, or None."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic_%s_%s.json"
                                           % (workload, mode)))):
        try:
            with open(p) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if int(d.get("B", -1)) == B:
            d["source"] = "profiles/" + os.path.basename(p)
            best = d
    return best


def _cpu_share():
    """CPUs this process may use: the affinity mask, capped by a cgroup v2
    CPU quota when one is set (the GPU box grants a share of a larger host)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(w, seconds=10.0, rounds=7):
    """The op-for-op torch CPU port (oracle/cnf_torch_port.py) on host cores:
    `rounds` interleaved rounds over two thread counts -- torch's default
    (OMP_NUM_THREADS, 16 on the GPU box) and every CPU this process may use --
    one timed pass of the config's full batch per count and round; the
    reported value is the faster count's median, both medians are listed."""
    from oracle import cnf_torch_port as P
    flow = make_flow(w, "cpu")
    st = {k: v for k, v in flow.state_dict().items()}
    layers = P.layers_from_state(st, w["L"], len(w["hidden"]) + 1, w["scale"], True)
    B = w["B"]  # the config's own batch (2^20 for cfg2)
    x, _ = synthetic_logits(B, w["D"], "cpu", 99)
    default = torch.get_num_threads()
    counts = sorted({default, _cpu_share()})
    times = {c: [] for c in counts}
    for c in counts:  # warm each pool once
        torch.set_num_threads(c)
        P.flow_forward(layers, x)
    t_start = time.perf_counter()
    r = 0
    while r < rounds or (time.perf_counter() - t_start < seconds and r < 4 * rounds):
        for c in counts:
            torch.set_num_threads(c)
            t = time.perf_counter()
            P.flow_forward(layers, x)
            times[c].append(time.perf_counter() - t)
        r += 1
    torch.set_num_threads(default)
    med = {c: float(np.median(v)) for c, v in times.items()}
    best = min(med, key=med.get)
    return {"value": B / med[best], "unit": "logit-vectors/sec", "cores": best,
            "nproc": os.cpu_count(), "cpu_share": _cpu_share(),
            "by_threads": {str(c): round(B / med[c], 1) for c in counts},
            "kind": "port",
            "sample": "%d interleaved rounds x %d-vector forward passes (the config's B, D=%d, "
                      "L=%d, h=%s) with the op-for-op torch CPU port at %s torch threads (this "
                      "process's CPU share: %d of a %d-CPU host), median per thread count; "
                      "port/reference time ratio: profiles/*_cpu_port_ratio.jsonl, DESIGN.md"
                      % (r, B, w["D"], w["L"], w["hidden"], " and ".join(map(str, counts)),
                         _cpu_share(), os.cpu_count() or 0)}


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(n, argv):
    """`bench.py --gpus N` without a launcher: start N fresh rank processes
    (one per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in their env) as
    children of this process, which never touches the GPU, and exit with the
    worst child status.  torch.distributed.run sets WORLD_SIZE itself, so the
    driver's launcher path never comes here."""
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    for p in procs:
        c = p.wait()
        if c != 0 and rc == 0:
            rc = c if c > 0 else 128 - c
    return rc


def main():
    global NLL_BUCKET
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle-s", type=float, default=0.3,
                    help="untimed steps for this many seconds before the warmup (clock ramp)")
    ap.add_argument("--workload", default="cfg2", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=0, help="vectors per GPU (default: config)")
    ap.add_argument("--rotate-gb", type=float, default=1.0)
    ap.add_argument("--no-variants", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--overlap-allreduce", action="store_true",
                    help="run each NLL bucket's all-reduce under the next bucket's kernels")
    ap.add_argument("--nll-bucket", type=int, default=NLL_BUCKET,
                    help="batches whose NLL sums share one all-reduce (1: one per batch)")
    ap.add_argument("--dist-check", action="store_true",
                    help="one rank through the RCCL collective path (overlapped and "
                         "synchronous all-reduce timed side by side)")
    ap.add_argument("--launch-check", action="store_true",
                    help="rank wiring only: gloo process group, no GPU (CPU test of the launcher)")
    args = ap.parse_args()
    NLL_BUCKET = max(1, args.nll_bucket)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        if not args.launch_check and torch.cuda.device_count() < args.gpus:
            sys.exit("bench.py --gpus %d: only %d GPU(s) visible" % (args.gpus,
                                                                   torch.cuda.device_count()))
        sys.exit(self_launch(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if args.launch_check:
        dist.init_process_group("gloo", init_method="env://")
        t = torch.tensor([float(rank)])
        dist.all_reduce(t)
        if rank == 0:
            print(json.dumps({"n_gpus": dist.get_world_size(), "rank_sum": t.item()}))
        dist.destroy_process_group()
        return
    if args.dist_check and world == 1:
        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29533"), ("RANK", "0"),
                     ("WORLD_SIZE", "1")):
            os.environ.setdefault(k, v)
    if world > 1 or args.dist_check:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        assert dist.get_world_size() == args.gpus
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    w = dict(WORKLOADS[args.workload])
    if args.batch:
        w["B"] = args.batch
    mode = "loss" if (w["D"] <= 16 and not w["inverse"]) else "forward"
    runner = Runner(w, dev, args.rotate_gb * 1e9, mode=mode)

    collective = None
    if world > 1 or args.dist_check:
        # NLL all-reduce over xGMI (configs[2]), overlapped with the next batch
        collective = NllAllReduce(runner, overlap=args.overlap_allreduce)

    settle_steps = runner.settle(args.settle_s) if args.settle_s > 0 else 0
    t_dev, wall = runner.timed(args.steps, args.warmup, collective)
    sync_ms = None
    if args.dist_check:
        last = runner.terms.clone()
        ts, _ = runner.timed(args.steps, args.warmup,
                             NllAllReduce(runner, overlap=not args.overlap_allreduce))
        sync_ms = round(ts / args.steps * 1e3, 5)
    # SURVEY 8(e) as written: one NLL all-reduce per batch.  The bucketed run
    # above is the headline; the literal form is timed beside it on the same
    # ranks, so the first multi-GPU run answers both.
    literal = None
    if collective and NLL_BUCKET != 1:
        keep = NLL_BUCKET
        NLL_BUCKET = 1
        t_lit, _ = runner.timed(args.steps, args.warmup,
                                NllAllReduce(runner, overlap=args.overlap_allreduce))
        NLL_BUCKET = keep
        tl = torch.tensor([t_lit], dtype=torch.float64, device=dev)
        every_l = [round(t_lit / args.steps * 1e3, 5)]
        if world > 1:
            g = [torch.zeros_like(tl) for _ in range(world)]
            dist.all_gather(g, tl)
            every_l = [round(v.item() / args.steps * 1e3, 5) for v in g]
            dist.all_reduce(tl, op=dist.ReduceOp.MAX)
        literal = {"value": round(w["B"] * world * args.steps / tl.item(), 1),
                   "ms_per_step": round(tl.item() / args.steps * 1e3, 5),
                   "rank_ms_per_step": every_l,
                   "step": "fused forward + log-det + NLL sums + one RCCL all-reduce of the "
                           "batch's 3 sums per batch (SURVEY 8(e) literally)"}
    t = torch.tensor([t_dev], dtype=torch.float64, device=dev)
    rank_ms = [round(t_dev / args.steps * 1e3, 5)]
    if world > 1:
        every = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(every, t)
        rank_ms = [round(v.item() / args.steps * 1e3, 5) for v in every]
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_max = t.item()
    total_vecs = w["B"] * world * args.steps
    value = total_vecs / t_max

    # dominant kernel: average device time per launch, no collective in between
    k_avg = kernel_only_seconds(runner, max(50, args.steps // 2))
    # each rank's own kernel-only time beside its step time: on N > 1 the
    # difference is the NLL all-reduce, the spread across ranks is kernel spread
    rank_kernel_us = [round(k_avg * 1e6, 3)]
    if world > 1:
        kt = torch.tensor([k_avg], dtype=torch.float64, device=dev)
        every_k = [torch.zeros_like(kt) for _ in range(world)]
        dist.all_gather(every_k, kt)
        rank_kernel_us = [round(v.item() * 1e6, 3) for v in every_k]
    bytes_vec = algo_bytes_per_vec(w["D"], w["L"], labels=(mode == "loss"))
    flops_vec = algo_flops_per_vec(w["D"], w["L"], w["hidden"], w["scale"])
    mfma_bound = w["D"] >= 32
    roof = roofline(w["B"], bytes_vec, flops_vec, k_avg, mfma=mfma_bound)
    roof.update({
        "traffic": None,
        "kernel": runner.stack.kernel_name(),
        "kernel_avg_us": round(k_avg * 1e6, 3),
        "timed_kernels": ("%s + k_reduce_rows4 (block-order NLL sum): the whole cnf_forward_loss "
                          "call, HIP events on its stream" % runner.kernel_symbol()) if mode == "loss"
                         else runner.kernel_symbol(),
        "algo_bytes_per_vec": bytes_vec, "algo_flops_per_vec": flops_vec,
        "rotating_sets": runner.nsets,
    })
    tr = measured_traffic(args.workload, w["B"], mode)
    if tr is not None:
        roof["traffic"] = tr["traffic_bytes_per_launch"]
        roof["traffic_source"] = tr["source"]

    variants = {}
    if rank == 0 and world == 1 and not args.no_variants:
        for name, wl, allo in (("cfg2_forward_ld", WORKLOADS["cfg2"], False),
                               ("cfg2_all_zs", WORKLOADS["cfg2"], True),
                               ("cfg5_inverse", WORKLOADS["cfg5"], False),
                               ("cfg4_d100", WORKLOADS["cfg4"], False),
                               ("cfg1_nice_d3", WORKLOADS["cfg1"], False)):
            r = Runner(dict(wl), dev, args.rotate_gb * 1e9, all_outputs=allo)
            ka = kernel_only_seconds(r, 30)
            bv = algo_bytes_per_vec(wl["D"], wl["L"], allo)
            fv = algo_flops_per_vec(wl["D"], wl["L"], wl["hidden"], wl["scale"])
            rf = roofline(wl["B"], bv, fv, ka, mfma=wl["D"] >= 32)
            variants[name] = {"vec_per_s": round(wl["B"] / ka, 1), "kernel_avg_us": round(ka * 1e6, 2),
                              "B": wl["B"], "kernel": r.stack.kernel_name(allo),
                              "hbm_gbs": rf["hbm_gbs"], "tflops": rf["compute_tflops"],
                              "bound": rf["bound"], "frac": rf["frac"]}
            del r
            torch.cuda.empty_cache()
        variants["cfg2_train_step_fused_loss_vjp"] = train_step_rate(dev, steps=100)
        variants["cfg4_train_step_loss_vjp"] = train_step_rate(dev, "cfg4", steps=5)
        variants["calibrator_fit_epoch"] = calibrator_epoch_rate(dev)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(w, args.cpu_seconds)

    if rank == 0:
        out = {
            "metric": "logit-vectors/sec forward+log-det (6-layer RealNVP, D=10)"
                      if args.workload == "cfg2" else "logit-vectors/sec (%s)" % args.workload,
            "value": round(value, 1),
            "unit": "logit-vectors/sec",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            # untimed steps before the warmup, until the device has run this long
            "settle": {"seconds": args.settle_s, "steps": settle_steps},
            "ms_per_step": round(t_max / args.steps * 1e3, 5),
            # the rank count the process group reports, and each rank's own
            # ms/step (ms_per_step above is their max)
            "ranks": dist.get_world_size() if dist.is_initialized() else 1,
            "rank_ms_per_step": rank_ms,
            # each rank's kernel-only time per launch (no collective in between)
            "rank_kernel_us": rank_kernel_us,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic",
            "config": {"workload": "%s: %d-layer %s coupling, D=%d, hidden_size=%s, %d vectors "
                                   "per GPU%s" % (args.workload, w["L"],
                                                  "RealNVP" if w["scale"] else "NICE", w["D"],
                                                  w["hidden"], w["B"],
                                                  ", inverse" if w["inverse"] else ""),
                       "global_batch": w["B"] * world, "parallelism": "dp%d" % world,
                       "hidden_size": w["hidden"], "weights": ("N(0,%g) synthetic" % w.get("sigma", 0.1)) if w.get("sigma", 0.1) is not None
                       else "the reference's default Linear init (synthetic)"},
            "roofline": roof,
        "step": "fused forward + log-det + NLL sums (cnf_forward_loss)%s" % (
            " + RCCL all-reduce of every batch's NLL sums, %d batches per all-reduce%s" % (
                NLL_BUCKET, " (overlapping the next bucket)" if args.overlap_allreduce else "")
            if collective else "") if mode == "loss"
            else "fused pass (cnf_%s)" % ("inverse" if w["inverse"] else "forward"),
            "cpu_baseline": cpu,
            "wall_s": round(wall, 4),
        }
        if variants:
            out["variants"] = variants
        if literal is not None:
            out["per_batch_allreduce"] = literal
        if sync_ms is not None:
            ov = args.overlap_allreduce
            out["dist_check"] = {"overlapped_ms_per_step": out["ms_per_step"] if ov else sync_ms,
                                 "synchronous_ms_per_step": sync_ms if ov else out["ms_per_step"],
                                 "terms_after_all_reduce": last.tolist()}
        print(json.dumps(out))
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
