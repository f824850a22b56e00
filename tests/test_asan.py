"""Host-side AddressSanitizer runs (GPU ASan is not
available on this pool, so only host code is instrumented): `make asan`
builds cnf_abi.hip / cnf_guard.hip's host pass and the torch.library shim
(cnf_torch_ops.cpp) with -fsanitize=address; here, in the build container
(no GPU), (1) tools/asan/abi_check drives the C ABI's descriptor validation
and plan sizing with seeded random and malformed descriptors, and (2) a
Python child with the same ASan runtime preloaded feeds the torch operators
malformed descriptor / permutation tables.  Any ASan report fails the test."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "calibration-normalizing-flows_amd", "csrc")
LIBDIR = os.path.join(ROOT, "calibration-normalizing-flows_amd", "cnf_hip")
BIN = os.path.join(ROOT, "tools", "asan", "abi_check")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0")


def _runtime():
    rt = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return rt[-1] if rt else None


@pytest.fixture(scope="module")
def asan_build():
    if _runtime() is None:
        pytest.skip("clang ASan runtime not found")
    r = subprocess.run(["make", "-C", CSRC, "-j8", "asan"], capture_output=True, text=True, timeout=1800)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return True


def test_abi_descriptor_validation_under_asan(asan_build):
    r = subprocess.run([BIN, "3000"], capture_output=True, text=True, timeout=600, env=ENV)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert '"failures": 0' in r.stdout


_CHILD = r'''
import sys, torch
torch.ops.load_library(sys.argv[1])
x = torch.zeros(4, 10)
blob = torch.zeros(64, dtype=torch.uint8)
good = [10, 6, 2, 5, 5, 0, 0, 0, 0, 0, 0, 1, 1, 0, 0]
cases = [
    (good[:14], None),                                     # short descriptor
    (good + [0], None),                                    # long descriptor
    (good, torch.zeros(5, 10, dtype=torch.int64)),         # perms: wrong layer count
    (good, torch.zeros(6, 9, dtype=torch.int64)),          # perms: wrong width
    (good, torch.arange(60).reshape(6, 10)),               # perms: out of range (CPU input)
    ([0] * 15, None),                                      # zero dim
    ([10, 6, 9] + [5] * 8 + [1, 1, 0, 0], None),           # too many hidden layers
    (good, None),                                          # CPU input
]
raised = 0
for desc, perms in cases:
    for op in ("forward", "flow", "forward_loss", "predict"):
        try:
            if op == "forward":
                torch.ops.cnf.forward(x, blob, desc, perms, False, False)
            elif op == "flow":
                torch.ops.cnf.flow(x, blob, desc, perms, False, [])
            elif op == "forward_loss":
                torch.ops.cnf.forward_loss(x, torch.zeros(4, dtype=torch.int64), blob, desc,
                                           perms, 0, 1.0)
            else:
                torch.ops.cnf.predict(x, blob, desc, perms, torch.zeros(10))
        except RuntimeError:
            raised += 1
print("raised", raised, "of", len(cases) * 4)
assert raised == len(cases) * 4
'''


def test_torch_ops_argument_parsing_under_asan(asan_build):
    lib = os.path.join(LIBDIR, "libcnf_torch_asan.so")
    env = dict(ENV, LD_PRELOAD=_runtime())
    r = subprocess.run([sys.executable, "-c", _CHILD, lib], capture_output=True, text=True,
                       timeout=600, env=env)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert "raised" in r.stdout
