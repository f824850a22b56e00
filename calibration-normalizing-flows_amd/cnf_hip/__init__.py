"""Native (HIP, gfx950) coupling-flow engine: ctypes binding of libcnf_hip.so
and the torch-side orchestration (prepared-weight cache, streams, autograd)."""
from ._lib import CnfError, UnsupportedShape, lib  # noqa: F401
from .engine import CouplingStack, stats  # noqa: F401
