import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "calibration-normalizing-flows_amd")
for p in (ROOT, PKG, os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: longer CPU test")


# Per-fixture numbers some tests record (e.g. the GPU inverse error next to
# the reference's own fp32 error, tests/test_gpu_parity.py), written as JSON
# lines to $CNF_RECORD_DIR/<name>.jsonl at the end of the session when that
# variable is set (tools/gpu_steps.sh sets it to gpurun_out/).
RECORDS = {}


def pytest_sessionfinish(session, exitstatus):
    out = os.environ.get("CNF_RECORD_DIR")
    if not out or not RECORDS:
        return
    import json
    os.makedirs(out, exist_ok=True)
    for name, rows in RECORDS.items():
        with open(os.path.join(out, name + ".jsonl"), "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
