"""C-ABI checks that need no GPU: libcnf_hip.so loads, exports every symbol
include/cnf.h declares, and the host-only entry points validate descriptors."""
import ctypes
import os
import re

import pytest
import torch

from cnf_hip import _lib
from cnf_hip.engine import CouplingStack
from flows.flows import NvpCouplingLayer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "cnf.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\**(cnf_\w+)\s*\(", src, re.M)))


def test_header_and_binding_agree():
    assert header_functions() == sorted(_lib.EXPORTS)


def test_library_exports_every_header_symbol():
    lib = _lib.lib()
    for name in header_functions():
        assert hasattr(lib, name), name
    assert lib.cnf_abi_version() == _lib.ABI_VERSION


def _count(desc):
    n = ctypes.c_int64()
    st = _lib.lib().cnf_param_count(ctypes.byref(desc), ctypes.byref(n))
    return st, n.value


def test_param_count_matches_state_dict():
    for dim, hidden, scale, shift in [(10, [5, 5], 1, 1), (100, [100, 100], 1, 1),
                                      (3, [5, 5], 0, 1), (10, [], 1, 0), (10, [4, 6, 3], 1, 1)]:
        layers = [NvpCouplingLayer(dim, hidden, scale=scale, shift=shift) for _ in range(3)]
        ref = sum(p.numel() for ly in layers for p in ly.parameters() if p.requires_grad)
        st, n = _count(_lib.make_desc(dim, 3, hidden, scale, shift))
        assert st == 0 and n == ref
        stack = CouplingStack(layers)
        assert stack.param_count() == ref
        nt = ctypes.c_int32()
        assert _lib.lib().cnf_param_tensor_count(ctypes.byref(stack.desc), ctypes.byref(nt)) == 0
        assert nt.value == len(stack.param_tensors())


def test_cfg2_param_count_is_1740_and_cfg4_727200():
    assert _count(_lib.make_desc(10, 6, [5, 5]))[1] == 1740
    assert _count(_lib.make_desc(100, 12, [100, 100]))[1] == 727200


def test_kernel_family_selection():
    name = lambda d: _lib.lib().cnf_kernel_name(ctypes.byref(d)).decode()
    assert name(_lib.make_desc(10, 6, [5, 5])) == "sgpr-fused"
    assert name(_lib.make_desc(3, 2, [5, 5], scale=0)) == "sgpr-fused"
    assert name(_lib.make_desc(10, 6, [5, 5], strict_nan=1)) == "valu-fused"
    assert name(_lib.make_desc(10, 6, [10, 10])) == "valu-fused"
    assert name(_lib.make_desc(100, 12, [100, 100])) == "mfma-wide"
    assert name(_lib.make_desc(10, 3, [4, 6, 3])) == "mfma-tile"


def test_legacy_kernel_family_selection():
    """Legacy stacks (CNF_OPT_ALT_MASK / S_TANH) of k_valu's shapes run on k_valu
    (never on k_sgpr), the rest on the MFMA-tile family."""
    name = lambda d: _lib.lib().cnf_kernel_name(ctypes.byref(d)).decode()
    alt, tanh = _lib.OPT_ALT_MASK, _lib.OPT_S_TANH
    assert name(_lib.make_desc(10, 4, [10], options=alt | tanh)) == "valu-fused"
    assert name(_lib.make_desc(10, 3, [5, 5], options=alt | tanh)) == "valu-fused"
    assert name(_lib.make_desc(3, 5, [3], options=alt | tanh)) == "valu-fused"
    assert name(_lib.make_desc(10, 4, [5, 5], options=alt)) == "valu-fused"      # not k_sgpr
    assert name(_lib.make_desc(10, 4, [10], scale=0, options=alt)) == "valu-fused"  # NICE v3
    assert name(_lib.make_desc(10, 4, [5, 5], options=tanh)) == "valu-fused"
    assert name(_lib.make_desc(10, 4, [7], options=alt | tanh)) == "mfma-tile"  # no tanh table
    assert name(_lib.make_desc(20, 1, [], options=alt | tanh)) == "mfma-tile"


@pytest.mark.parametrize("mutate,status", [
    (lambda d: setattr(d, "abi_version", 99), -2),
    (lambda d: setattr(d, "dim", 1), -2),
    (lambda d: setattr(d, "dim", 1000), -3),
    (lambda d: setattr(d, "n_layers", 0), -2),
    (lambda d: setattr(d, "n_hidden", 9), -2),
    (lambda d: setattr(d, "scale", 2), -2),
])
def test_bad_descriptors_are_rejected(mutate, status):
    d = _lib.make_desc(10, 6, [5, 5])
    mutate(d)
    assert _count(d)[0] == status
    assert _lib.lib().cnf_strerror(status)


def test_bad_permutation_rejected():
    p = torch.full((2, 4), -1, dtype=torch.int64)
    p[1] = torch.tensor([0, 1, 1, 3])
    assert _count(_lib.make_desc(4, 2, [3], perms=p))[0] == -2
    p[1] = torch.tensor([3, 1, 0, 2])
    assert _count(_lib.make_desc(4, 2, [3], perms=p))[0] == 0


def test_forward_argument_validation_without_gpu():
    lib = _lib.lib()
    d = _lib.make_desc(10, 6, [5, 5])
    P = ctypes.c_void_p
    # B < 0 and NULL pointers are rejected before any device work
    assert lib.cnf_forward(ctypes.byref(d), P(16), P(16), P(16), P(16), P(0),
                           ctypes.c_int64(-1), P(0)) == -4
    assert lib.cnf_forward(ctypes.byref(d), P(0), P(16), P(16), P(16), P(0),
                           ctypes.c_int64(8), P(0)) == -1
    assert lib.cnf_forward(ctypes.byref(d), P(16), P(18), P(16), P(16), P(0),
                           ctypes.c_int64(8), P(0)) == -6
    # B == 0 is a no-op
    assert lib.cnf_forward(ctypes.byref(d), P(0), P(0), P(0), P(0), P(0),
                           ctypes.c_int64(0), P(0)) == 0


def test_torch_library_operators_register():
    """csrc/cnf_torch_ops.cpp registers the cnf::* operators (TORCH_LIBRARY)
    over the same C ABI; loading needs no GPU."""
    from cnf_hip import _lib
    ops = _lib.torch_ops()
    assert ops is not None, "libcnf_torch.so was not built"
    names = {"forward", "flow", "forward_loss", "loss_and_grads", "vjp", "predict"}
    for n in names:
        assert hasattr(ops, n), n
    sch = str(torch.ops.cnf.flow.default._schema)
    assert "Tensor[] params" in sch and "int[] desc" in sch
    d = _lib.make_desc(10, 6, [5, 5])
    assert _lib.desc_list(d) == [10, 6, 2, 5, 5, 0, 0, 0, 0, 0, 0, 1, 1, 0, 0]


def _vjp_bytes(desc, B):
    n = ctypes.c_size_t()
    st = _lib.lib().cnf_vjp_workspace_bytes(ctypes.byref(desc), ctypes.c_int64(B), ctypes.byref(n))
    return st, n.value


def test_wide_training_workspace_plans():
    """cfg4 at 2^18 rows: the fused sweeps' plan holds the per-row tape (640
    floats per row and layer) and every layer's conditioner gradients (576), in
    whole 32-row blocks; OPT_NO_WIDE, strict_nan and the inverse take the
    layer-at-a-time plan (host-only sizing, no GPU)."""
    B, L = 1 << 18, 12
    st, fused = _vjp_bytes(_lib.make_desc(100, L, [100, 100]), B)
    assert st == 0
    tape_and_g = L * B * (640 + 576) * 4
    assert tape_and_g < fused < tape_and_g * 1.05
    st, layered = _vjp_bytes(_lib.make_desc(100, L, [100, 100], options=_lib.OPT_NO_WIDE), B)
    assert st == 0 and layered < tape_and_g
    st, strict = _vjp_bytes(_lib.make_desc(100, L, [100, 100], strict_nan=True), B)
    assert st == 0 and strict < tape_and_g
    n = ctypes.c_size_t()
    assert _lib.lib().cnf_vjp_inverse_workspace_bytes(
        ctypes.byref(_lib.make_desc(100, L, [100, 100])), ctypes.c_int64(B), ctypes.byref(n)) == 0
    assert n.value == layered
    # a ragged batch: the wave-tiled arrays hold whole 32-row blocks
    st, ragged = _vjp_bytes(_lib.make_desc(100, L, [100, 100]), B + 1)
    assert st == 0 and ragged > L * (B + 32) * (640 + 576) * 4


def test_guard_argument_validation_without_gpu():
    """cnf_guard_nonfinite rejects bad arguments before any launch."""
    import ctypes
    lib = _lib.lib()
    P = ctypes.c_void_p
    flag = ctypes.c_int32(0)
    buf = (ctypes.c_float * 8)()
    assert lib.cnf_guard_nonfinite(P(ctypes.addressof(buf)), ctypes.c_int64(-1),
                                   P(ctypes.addressof(flag)), P(0)) == -4
    assert lib.cnf_guard_nonfinite(P(ctypes.addressof(buf)), ctypes.c_int64(8), P(0), P(0)) == -1
    assert lib.cnf_guard_nonfinite(P(0), ctypes.c_int64(8), P(ctypes.addressof(flag)), P(0)) == -1
    assert lib.cnf_guard_nonfinite(P(ctypes.addressof(buf) + 2), ctypes.c_int64(4),
                                   P(ctypes.addressof(flag)), P(0)) == -6
    assert lib.cnf_guard_nonfinite(P(0), ctypes.c_int64(0), P(ctypes.addressof(flag)), P(0)) == 0


def test_adam_guarded_argument_validation_without_gpu():
    """cnf_adam_step_guarded needs its skip flag (NULL is rejected before any
    launch; the plain cnf_adam_step is the unguarded form)."""
    lib = _lib.lib()
    stack = CouplingStack([NvpCouplingLayer(10, [5, 5]) for _ in range(2)])
    P = ctypes.c_void_p
    arr = (P * 24)()  # 2 layers x 2 nets x 3 Linears x (W, b); never read
    st = lib.cnf_adam_step_guarded(ctypes.byref(stack.desc), arr, P(16), P(16), P(16),
                                   ctypes.c_int64(1), ctypes.c_double(1e-3), None,
                                   ctypes.c_double(0.9), ctypes.c_double(0.999),
                                   ctypes.c_double(1e-8), ctypes.c_double(0.0), None, P(0))
    assert st == -1


def test_roctx_build_exports_every_header_symbol():
    """`make roctx` (the traced diagnostic build): the same C ABI, with every
    launching entry point inside a roctx range, linked against the roctx
    library (checked by symbol tables only: no GPU, no tracer needed)."""
    import subprocess
    path = os.path.join(ROOT, "calibration-normalizing-flows_amd", "cnf_hip",
                        "libcnf_hip_roctx.so")
    if not os.path.exists(path):
        pytest.skip("make roctx was not run")
    syms = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True,
                          check=True).stdout
    for name in header_functions():
        assert re.search(r"\sT %s$" % name, syms, re.M), name
    undef = subprocess.run(["nm", "-D", "--undefined-only", path], capture_output=True,
                           text=True, check=True).stdout
    assert "roctxRangePushA" in undef and "roctxRangePop" in undef
