"""On-device Adam over a coupling stack's parameters in ONE launch
(cnf_adam_step, include/cnf.h), fed by the flat gradient of cnf_loss_vjp:
the optimizer half of the calibrator's fused training step (SURVEY 8(f) rank 1;
the reference steps torch.optim.Adam at its defaults, calibrators.py:239-295).
Same update as torch.optim.Adam (amsgrad off)."""
import ctypes

import torch

from . import _lib
from .engine import _ptr, _stream, stats


class StackAdam:
    """Adam state (two flat moment buffers) for one CouplingStack."""

    def __init__(self, stack, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        self.stack = stack
        self.lr, self.betas, self.eps, self.weight_decay = lr, tuple(betas), eps, weight_decay
        self.t = 0
        self._m = self._v = None

    @classmethod
    def like(cls, stack, torch_adam):
        """Hyper-parameters of an existing torch.optim.Adam (first group)."""
        g = torch_adam.param_groups[0]
        if g.get("amsgrad") or g.get("maximize"):
            raise ValueError("StackAdam: amsgrad / maximize are not supported")
        return cls(stack, g["lr"], g["betas"], g["eps"], g["weight_decay"])

    def step(self, flat_grads):
        ps = self.stack.param_tensors()
        dev = ps[0].device
        if self._m is None:
            n = self.stack.param_count()
            self._m = torch.zeros(n, dtype=torch.float32, device=dev)
            self._v = torch.zeros(n, dtype=torch.float32, device=dev)
        for p in ps:
            if not p.is_contiguous():
                raise ValueError("StackAdam needs contiguous parameters")
        self.t += 1
        arr = (ctypes.c_void_p * len(ps))(*[p.data_ptr() for p in ps])
        lib = _lib.lib()
        st = lib.cnf_adam_step(ctypes.byref(self.stack.desc), arr, _ptr(flat_grads), _ptr(self._m),
                               _ptr(self._v), ctypes.c_int64(self.t), ctypes.c_float(self.lr),
                               ctypes.c_float(self.betas[0]), ctypes.c_float(self.betas[1]),
                               ctypes.c_float(self.eps), ctypes.c_float(self.weight_decay),
                               _stream(dev))
        _lib.check("cnf_adam_step", st)
        # the kernel wrote the parameters behind autograd's back: bump their
        # version counters, so every prepared-weight cache keyed on them (this
        # stack's and any other binding's) rebuilds
        for p in ps:
            torch.autograd.graph.increment_version(p)
        stats["adam"] = stats.get("adam", 0) + 1
