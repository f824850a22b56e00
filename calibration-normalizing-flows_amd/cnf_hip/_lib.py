"""ctypes binding of libcnf_hip.so (the C ABI declared in include/cnf.h).

The library is built in-tree by `make -C calibration-normalizing-flows_amd/csrc`
(or `__graft_entry__.build()`).  `torch` is imported first so the process has a
single HIP runtime: libcnf_hip.so's NEEDED libamdhip64.so.7 then resolves to
the copy torch already loaded (same SONAME).  There is no fallback: if the
library is missing, every native entry point raises.
"""
import ctypes
import os
import threading

import torch  # noqa: F401  (load torch's HIP runtime before ours)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CNF_HIP_LIB", os.path.join(_HERE, "libcnf_hip.so"))

ABI_VERSION = 2
MAX_HIDDEN = 8
MAX_DIM = 256
LOSS_CAL = 0
LOSS_CE = 1
OPT_NO_SGPR = 1   # cnf_desc.options (include/cnf.h)
OPT_NO_WIDE = 2
OPT_ALT_MASK = 4  # legacy code-old/realNVP.py semantics (flows/legacy.py)
OPT_S_TANH = 8

# Every symbol include/cnf.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "cnf_param_count", "cnf_param_tensor_count", "cnf_prepared_bytes", "cnf_prepare",
    "cnf_forward", "cnf_inverse", "cnf_forward_loss_workspace_bytes", "cnf_forward_loss",
    "cnf_predict", "cnf_vjp_workspace_bytes", "cnf_vjp", "cnf_loss_vjp", "cnf_adam_step",
    "cnf_adam_step_sched", "cnf_adam_step_guarded",
    "cnf_vjp_inverse_workspace_bytes", "cnf_vjp_inverse", "cnf_guard_nonfinite",
    "cnf_kernel_name", "cnf_strerror", "cnf_last_hip_error", "cnf_abi_version",
)


class CnfDesc(ctypes.Structure):
    """Mirror of `cnf_desc` (include/cnf.h)."""
    _fields_ = [
        ("abi_version", ctypes.c_int32),
        ("dim", ctypes.c_int32),
        ("n_layers", ctypes.c_int32),
        ("n_hidden", ctypes.c_int32),
        ("hidden", ctypes.c_int32 * MAX_HIDDEN),
        ("scale", ctypes.c_int32),
        ("shift", ctypes.c_int32),
        ("strict_nan", ctypes.c_int32),
        ("options", ctypes.c_int32),
        ("perms", ctypes.POINTER(ctypes.c_int64)),
    ]


class CnfError(RuntimeError):
    def __init__(self, fn, status, lib):
        msg = lib.cnf_strerror(status).decode()
        if status == -5:
            msg += " (hipError %d)" % lib.cnf_last_hip_error()
        super().__init__("%s failed: %s [%d]" % (fn, msg, status))
        self.status = status


class UnsupportedShape(CnfError):
    pass


_lib = None
_lock = threading.Lock()


def _bind(lib):
    P, I32, I64, F, DB = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float,
                          ctypes.c_double)
    D = ctypes.POINTER(CnfDesc)
    sig = {
        "cnf_param_count": (ctypes.c_int, [D, ctypes.POINTER(I64)]),
        "cnf_param_tensor_count": (ctypes.c_int, [D, ctypes.POINTER(I32)]),
        "cnf_prepared_bytes": (ctypes.c_int, [D, ctypes.POINTER(ctypes.c_size_t)]),
        "cnf_prepare": (ctypes.c_int, [D, ctypes.POINTER(P), P, P]),
        "cnf_forward": (ctypes.c_int, [D, P, P, P, P, P, I64, P]),
        "cnf_inverse": (ctypes.c_int, [D, P, P, P, P, P, I64, P]),
        "cnf_forward_loss_workspace_bytes": (ctypes.c_int,
                                             [D, I64, ctypes.POINTER(ctypes.c_size_t)]),
        "cnf_forward_loss": (ctypes.c_int, [D, P, P, P, I32, F, P, P, P, I64, P, ctypes.c_size_t,
                                            P]),
        "cnf_predict": (ctypes.c_int, [D, P, P, P, P, P, I64, P]),
        "cnf_vjp_workspace_bytes": (ctypes.c_int, [D, I64, ctypes.POINTER(ctypes.c_size_t)]),
        "cnf_vjp": (ctypes.c_int, [D, P, P, P, P, P, P, P, I64, P, ctypes.c_size_t, P]),
        "cnf_loss_vjp": (ctypes.c_int, [D, P, P, P, I32, F, F, P, P, P, I64, P, ctypes.c_size_t,
                                        P]),
        "cnf_vjp_inverse_workspace_bytes": (ctypes.c_int,
                                            [D, I64, ctypes.POINTER(ctypes.c_size_t)]),
        "cnf_vjp_inverse": (ctypes.c_int, [D, P, P, P, P, P, P, P, I64, P, ctypes.c_size_t, P]),
        "cnf_adam_step": (ctypes.c_int, [D, ctypes.POINTER(P), P, P, P, I64, DB, DB, DB, DB, DB,
                                         P]),
        "cnf_adam_step_sched": (ctypes.c_int, [D, ctypes.POINTER(P), P, P, P, P, DB, DB, DB, DB,
                                               P]),
        "cnf_adam_step_guarded": (ctypes.c_int, [D, ctypes.POINTER(P), P, P, P, I64, DB, P, DB,
                                                 DB, DB, DB, P, P]),
        "cnf_guard_nonfinite": (ctypes.c_int, [P, I64, P, P]),
        "cnf_kernel_name": (ctypes.c_char_p, [D]),
        "cnf_strerror": (ctypes.c_char_p, [ctypes.c_int]),
        "cnf_last_hip_error": (ctypes.c_int, []),
        "cnf_abi_version": (ctypes.c_int, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def lib():
    """The loaded library; raises (never falls back) if it cannot be loaded."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(
                        "libcnf_hip.so not found at %s -- build it with "
                        "`make -C calibration-normalizing-flows_amd/csrc` or "
                        "`python -c 'import __graft_entry__ as g; g.build()'`" % LIB_PATH)
                l = _bind(ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL))
                if l.cnf_abi_version() != ABI_VERSION:
                    raise RuntimeError("libcnf_hip ABI %d != %d" % (l.cnf_abi_version(),
                                                                   ABI_VERSION))
                _lib = l
    return _lib


TORCH_LIB_PATH = os.environ.get("CNF_TORCH_LIB", os.path.join(_HERE, "libcnf_torch.so"))
_ops = None
_ops_tried = False


def torch_ops():
    """torch.ops.cnf (the TORCH_LIBRARY operators of csrc/cnf_torch_ops.cpp over
    the same C ABI), or None when libcnf_torch.so was not built.  Loaded after
    libcnf_hip.so so both resolve to the one in-tree copy."""
    global _ops, _ops_tried
    if not _ops_tried:
        with _lock:
            if not _ops_tried:
                lib()
                if os.path.exists(TORCH_LIB_PATH):
                    torch.ops.load_library(TORCH_LIB_PATH)
                    _ops = torch.ops.cnf
                _ops_tried = True
    return _ops


def desc_list(d):
    """cnf_desc as the int[] the torch operators take."""
    return [d.dim, d.n_layers, d.n_hidden] + [d.hidden[i] for i in range(MAX_HIDDEN)] + \
        [d.scale, d.shift, d.strict_nan, d.options]


def check(fn, status):
    if status != 0:
        l = lib()
        raise (UnsupportedShape if status == -3 else CnfError)(fn, status, l)


def make_desc(dim, n_layers, hidden, scale=True, shift=True, strict_nan=False, perms=None,
              options=0):
    """Build a CnfDesc; `perms` is an int64 host tensor [L, D] (row[0] < 0: no perm)
    that must stay alive while the descriptor is used."""
    hidden = list(hidden)
    if len(hidden) > MAX_HIDDEN:
        raise ValueError("at most %d hidden layers" % MAX_HIDDEN)
    d = CnfDesc()
    d.abi_version = ABI_VERSION
    d.dim = int(dim)
    d.n_layers = int(n_layers)
    d.n_hidden = len(hidden)
    for i, h in enumerate(hidden):
        d.hidden[i] = int(h)
    d.scale = int(bool(scale))
    d.shift = int(bool(shift))
    d.strict_nan = int(bool(strict_nan))
    d.options = int(options)
    d.perms = None
    if perms is not None:
        assert perms.dtype == torch.int64 and perms.is_contiguous() and not perms.is_cuda
        d.perms = ctypes.cast(perms.data_ptr(), ctypes.POINTER(ctypes.c_int64))
    return d
