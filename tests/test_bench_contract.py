"""CPU checks of bench.py's workload table and algorithmic figures.

The roofline's `achieved` is algorithmic bytes (or flops) per vector times the
vectors per launch, so these per-vector figures are what DESIGN.md states for
SURVEY 8(d); pin them here so a bench edit cannot drift from the doc.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_workloads_match_baseline_configs():
    w = bench.WORKLOADS
    assert (w["cfg1"]["D"], w["cfg1"]["L"], w["cfg1"]["B"], w["cfg1"]["scale"]) == (3, 2, 4096, False)
    assert (w["cfg2"]["D"], w["cfg2"]["L"], w["cfg2"]["B"]) == (10, 6, 1 << 20)
    assert w["cfg2"]["hidden"] == [5, 5]  # flows/flows.py:71 default
    assert (w["cfg4"]["D"], w["cfg4"]["L"], w["cfg4"]["hidden"]) == (100, 12, [100, 100])
    assert w["cfg5"]["inverse"] and not w["cfg2"]["inverse"]


def test_cfg2_algorithmic_figures():
    # 6 layers x (2 nets x 2 x (5*5 + 5*5 + 5*5) MACs + 3*5 elementwise) = 1890
    assert bench.algo_flops_per_vec(10, 6, [5, 5]) == 1890
    # x in (40) + final z out (40) + log-det (4) + int64 label (8)
    assert bench.algo_bytes_per_vec(10, 6, labels=True) == 92
    assert bench.algo_bytes_per_vec(10, 6) == 84
    # every layer's z written (Flow.forward's zs list, flows/flows.py:17-25)
    assert bench.algo_bytes_per_vec(10, 6, all_outputs=True) == 40 + 240 + 4


def test_nice_has_no_scale_flops():
    # scale=False: one net, shift-only update (flows/flows.py:76-79)
    per_layer = 2 * (2 * 5 + 5 * 5 + 5 * 1) + 1
    assert bench.algo_flops_per_vec(3, 2, [5, 5], scale=False) == 2 * per_layer


def test_roofline_names_the_binding_roof():
    # cfg2 fused loss pass: 92 B and 1,890 flops per vector -> the VALU roof
    # (83.2 G vec/s) binds before HBM (87.0 G vec/s); SURVEY 8(d)
    r = bench.roofline(1 << 20, 92, 1890, 42.9e-6)
    assert r["bound"] == "valu" and r["unit"] == "TFLOP/s"
    rate = (1 << 20) / 42.9e-6
    assert abs(r["frac"] - rate / (157.3e12 / 1890)) < 1e-4
    assert abs(r["compute_frac"] - r["frac"]) < 1e-4
    # every-layer outputs (284 B) are HBM-bound
    r = bench.roofline(1 << 20, 284, 1890, 70e-6)
    assert r["bound"] == "hbm" and abs(r["frac"] - r["hbm_frac"]) < 1e-4
    # cfg4 is MFMA-bound
    assert bench.roofline(1 << 18, 804, 961800, 3e-3, mfma=True)["bound"] == "mfma"


def test_gpus_flag_self_launches_ranks():
    """`bench.py --gpus 2` with no launcher starts two rank processes itself
    (here with --launch-check: gloo wiring only, no GPU)."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--launch-check"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line == {"n_gpus": 2, "rank_sum": 1.0}


def test_gpus_flag_must_match_launcher_world():
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1",
                          "--launch-check"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode != 0 and "WORLD_SIZE=2" in out.stderr


def test_nll_all_reduce_buckets_cover_every_batch_once(monkeypatch):
    """bench.NllAllReduce (configs[2]'s exchange, bucketed): every batch's row
    is handed to exactly one all-reduce, after the kernel wrote it and before
    the row is written again, for the synchronous and the overlapped forms --
    checked with a recording stand-in for torch.distributed.all_reduce."""
    import torch

    class FakeRunner:
        def __init__(self):
            self.term_bufs = torch.zeros(2, bench.NLL_BUCKET, 3)
            self.i = 0

        def step(self):  # as bench.Runner.step: pick the row, then count the batch
            self.terms = self.term_bufs[(self.i // bench.NLL_BUCKET) % 2,
                                        self.i % bench.NLL_BUCKET]
            self.terms.fill_(float(self.i))
            self.i += 1

    class Work:
        def __init__(self, log, vals):
            self.log, self.vals = log, vals

        def wait(self):
            self.log.append(("wait", self.vals))

    for overlap in (False, True):
        for steps in (1, 7, bench.NLL_BUCKET, 2 * bench.NLL_BUCKET + 3, 5 * bench.NLL_BUCKET):
            log, reduced = [], []

            def fake_all_reduce(t, async_op=False):
                vals = tuple(int(v) for v in t[:, 0].tolist())
                reduced.extend(vals)
                log.append(("reduce", vals))
                return Work(log, vals) if async_op else None

            monkeypatch.setattr(bench.dist, "all_reduce", fake_all_reduce)
            r = FakeRunner()
            coll = bench.NllAllReduce(r, overlap=overlap)
            for _ in range(steps):
                r.step()
                coll()
            coll.drain()
            assert sorted(reduced) == list(range(steps)), (overlap, steps)
            if overlap:  # a bucket is waited for before its rows are written again
                for k, (what, vals) in enumerate(log):
                    if what == "reduce" and vals and vals[0] + 2 * bench.NLL_BUCKET < steps:
                        assert ("wait", vals) in log[k + 1:], (steps, vals)


def test_nll_all_reduce_realigns_after_uncollected_batches(monkeypatch):
    """The bench's own order: settle() and kernel_only_seconds()
    launch batches WITHOUT the collective, then timed() runs warmup + drain and
    the timed steps + drain.  Every batch launched under the collective must be
    reduced exactly once, and no batch launched without it may be reduced."""
    import torch

    class FakeRunner:
        def __init__(self):
            self.term_bufs = torch.zeros(2, bench.NLL_BUCKET, 3)
            self.i = 0

        def step(self):
            self.terms = self.term_bufs[(self.i // bench.NLL_BUCKET) % 2,
                                        self.i % bench.NLL_BUCKET]
            self.terms.fill_(float(self.i))
            self.i += 1

    reduced = []

    def fake_all_reduce(t, async_op=False):
        reduced.extend(int(v) for v in t[:, 0].tolist())

    monkeypatch.setattr(bench.dist, "all_reduce", fake_all_reduce)
    for pre in (0, 3, 17, bench.NLL_BUCKET + 9):
        for warm, steps in ((2, 7), (5, bench.NLL_BUCKET + 4), (0, 2 * bench.NLL_BUCKET)):
            reduced.clear()
            r = FakeRunner()
            coll = bench.NllAllReduce(r)
            for _ in range(pre):  # settle: no collective
                r.step()
            expect = []
            coll.realign()  # as timed(): once, then warmup + drain, steps + drain
            for n in (warm, steps):
                first = r.i
                for _ in range(n):
                    r.step()
                    coll()
                expect.extend(range(first, r.i))
                coll.drain()
            assert sorted(reduced) == expect, (pre, warm, steps)
