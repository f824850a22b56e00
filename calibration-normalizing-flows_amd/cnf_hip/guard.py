"""Device-side non-finite guard (cnf_guard_nonfinite, include/cnf.h): the
counterpart of the reference's NaN abort in its experiment loop,

    if (preds != preds).any():                    run_experiment3D.py:129-131
        print('Aborting training due to nan values'); break

without synchronising the host every step.  A guard owns one zeroed device
int32; check() ORs into it (1: a NaN was seen, 2: an inf) on the current
stream; the host reads it when it chooses (tripped(), one sync), e.g. once
per epoch or every N steps.  ROCm tensors only (the product path has no CPU
fallback: the library must be loaded)."""
import ctypes

import torch

from . import _lib

NAN = 1
INF = 2


class NonFiniteGuard:
    def __init__(self, device):
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("NonFiniteGuard: ROCm device tensors only")
        self.flag = torch.zeros(1, dtype=torch.int32, device=self.device)

    def check(self, *tensors):
        """Scan every given fp32 device tensor (views are made contiguous);
        returns self so calls chain."""
        lib = _lib.lib()
        stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        for t in tensors:
            if t is None:
                continue
            if t.device != self.device or t.dtype != torch.float32:
                raise ValueError("NonFiniteGuard.check: fp32 tensors on %s" % self.device)
            t = t.contiguous()
            st = lib.cnf_guard_nonfinite(ctypes.c_void_p(t.data_ptr()), ctypes.c_int64(t.numel()),
                                         ctypes.c_void_p(self.flag.data_ptr()), stream)
            _lib.check("cnf_guard_nonfinite", st)
        return self

    def tripped(self):
        """The accumulated bits (0: clean; NAN | INF otherwise). Syncs the host."""
        return int(self.flag.item())

    def reset(self):
        self.flag.zero_()
