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
