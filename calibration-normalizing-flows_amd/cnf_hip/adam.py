"""On-device Adam over a coupling stack's parameters in ONE launch
(cnf_adam_step, include/cnf.h), fed by the flat gradient of cnf_loss_vjp:
the optimizer half of the calibrator's fused training step (SURVEY 8(f) rank 1;
the reference steps torch.optim.Adam at its defaults, calibrators.py:239-295).
Same update as torch.optim.Adam (amsgrad off), with torch's scalar rounding
(the hyper-parameters cross the ABI as doubles).

`StackAdam.like(stack, torch_adam)` takes the torch optimizer's CURRENT
hyper-parameters and, when it already holds state for the stack's parameters
(an earlier fit), its step count and moments; `store_into(torch_adam)` writes
the state back, so the torch optimizer and the native one never diverge
across fit() calls."""
import ctypes

import torch

from . import _lib
from .engine import _ptr, _stream, stats


def supports(opt):
    """True when `opt` is an optimizer whose update cnf_adam_step reproduces:
    exactly torch.optim.Adam (not a subclass such as AdamW, whose decay is
    decoupled), with amsgrad, maximize and decoupled weight decay off."""
    if type(opt) is not torch.optim.Adam:
        return False
    return not any(g.get("amsgrad") or g.get("maximize") or g.get("decoupled_weight_decay")
                   for g in opt.param_groups)


def group_hparams(torch_adam, stack):
    """The CURRENT (lr, betas, eps, weight_decay) of the param group holding
    the stack's parameters, as Python floats -- a scheduler may have changed
    any of them since the last step (OneCycleLR and CyclicLR cycle beta1 as
    well as lr).  None when one of them is a tensor: reading it would sync the
    host, so the caller hands that group to torch's own optimizer.step()."""
    ids = {id(p) for p in stack.param_tensors()}
    for g in torch_adam.param_groups:
        if any(id(p) in ids for p in g["params"]):
            vals = (g["lr"], g["betas"][0], g["betas"][1], g["eps"], g["weight_decay"])
            if any(torch.is_tensor(v) for v in vals):
                return None
            return (float(g["lr"]), (float(g["betas"][0]), float(g["betas"][1])),
                    float(g["eps"]), float(g["weight_decay"]))
    raise ValueError("StackAdam: the optimizer holds none of the stack's parameters")


class StackAdam:
    """Adam state (two flat moment buffers) for one CouplingStack."""

    def __init__(self, stack, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        self.stack = stack
        self.lr, self.betas, self.eps, self.weight_decay = (float(lr), tuple(map(float, betas)),
                                                            float(eps), float(weight_decay))
        self.t = 0
        self._m = self._v = None

    @classmethod
    def like(cls, stack, torch_adam):
        """Hyper-parameters (and state, if any) of an existing torch.optim.Adam.
        Every stack parameter must sit in one param group."""
        ps = stack.param_tensors()
        ids = {id(p) for p in ps}
        groups = [g for g in torch_adam.param_groups if any(id(p) in ids for p in g["params"])]
        if len(groups) != 1:
            raise ValueError("StackAdam: the stack's parameters must share one param group")
        g = groups[0]
        if g.get("amsgrad") or g.get("maximize"):
            raise ValueError("StackAdam: amsgrad / maximize are not supported")
        lr = g["lr"].item() if torch.is_tensor(g["lr"]) else g["lr"]
        if not supports(torch_adam):
            raise ValueError("StackAdam: only a plain torch.optim.Adam (coupled weight decay) "
                             "is supported, got %s" % type(torch_adam).__name__)
        self = cls(stack, lr, g["betas"], g["eps"], g["weight_decay"])
        st = [torch_adam.state.get(p) for p in ps]
        have = [s is not None and "exp_avg" in s for s in st]
        if any(have) and not all(have):
            raise ValueError("StackAdam: the torch optimizer holds state for some of the "
                             "stack's parameters but not all (%d of %d)" % (sum(have), len(have)))
        if all(have):
            steps = {int(s["step"]) for s in st}
            if len(steps) != 1:
                raise ValueError("StackAdam: parameters at different step counts")
            self.t = steps.pop()
            dev = ps[0].device
            self._m = torch.cat([s["exp_avg"].reshape(-1).to(dev, torch.float32) for s in st])
            self._v = torch.cat([s["exp_avg_sq"].reshape(-1).to(dev, torch.float32) for s in st])
        return self

    def set_hparams(self, hp):
        """Adopt group_hparams()'s (lr, betas, eps, weight_decay)."""
        self.lr, self.betas, self.eps, self.weight_decay = hp

    def store_into(self, torch_adam):
        """Write step count and moments into the torch optimizer's state (the
        layout torch.optim.Adam keeps: per parameter, a 0-d float32 `step` and
        moments shaped like the parameter)."""
        if self._m is None:
            return
        off = 0
        for p in self.stack.param_tensors():
            n = p.numel()
            torch_adam.state[p] = {
                "step": torch.tensor(float(self.t), dtype=torch.float32),
                "exp_avg": self._m[off:off + n].view_as(p).clone(),
                "exp_avg_sq": self._v[off:off + n].view_as(p).clone(),
            }
            off += n

    def sched_values(self, t):
        """torch.optim.Adam's two step-dependent scalars for step t, formed as
        torch forms them (Python doubles, torch/optim/adam.py
        _single_tensor_adam), for cnf_adam_step_sched: [lr / (1 - beta1^t),
        (1 - beta2^t) ** 0.5]."""
        b1, b2 = self.betas
        return (self.lr / (1 - b1 ** t), (1 - b2 ** t) ** 0.5)

    def _ensure_state(self):
        ps = self.stack.param_tensors()
        dev = ps[0].device
        if self._m is None:
            n = self.stack.param_count()
            self._m = torch.zeros(n, dtype=torch.float32, device=dev)
            self._v = torch.zeros(n, dtype=torch.float32, device=dev)
        elif self._m.device != dev:
            self._m, self._v = self._m.to(dev), self._v.to(dev)
        return ps, dev

    def step_sched(self, flat_grads, sched):
        """One step whose scalars come from the device tensor `sched` [2]
        (graph capture: replays any step).  Advances the host step count."""
        ps, dev = self._ensure_state()
        self.t += 1
        arr = (ctypes.c_void_p * len(ps))(*[p.data_ptr() for p in ps])
        st = _lib.lib().cnf_adam_step_sched(
            ctypes.byref(self.stack.desc), arr, _ptr(flat_grads), _ptr(self._m), _ptr(self._v),
            _ptr(sched), ctypes.c_double(self.betas[0]), ctypes.c_double(self.betas[1]),
            ctypes.c_double(self.eps), ctypes.c_double(self.weight_decay), _stream(dev))
        _lib.check("cnf_adam_step_sched", st)
        for p in ps:
            torch.autograd.graph.increment_version(p)
        stats["adam"] = stats.get("adam", 0) + 1

    def step(self, flat_grads, skip=None):
        """One step.  skip: a device int32 flag (NonFiniteGuard.flag) read by
        the kernel: non-zero leaves the parameters and moments untouched
        (cnf_adam_step_guarded), with no host sync."""
        ps, dev = self._ensure_state()
        for p in ps:
            if not p.is_contiguous():
                raise ValueError("StackAdam needs contiguous parameters")
        self.t += 1
        arr = (ctypes.c_void_p * len(ps))(*[p.data_ptr() for p in ps])
        lib = _lib.lib()
        if skip is not None:
            if skip.dtype != torch.int32 or skip.device != dev:
                raise ValueError("StackAdam.step: skip must be a device int32 flag on %s" % dev)
            st = lib.cnf_adam_step_guarded(
                ctypes.byref(self.stack.desc), arr, _ptr(flat_grads), _ptr(self._m),
                _ptr(self._v), ctypes.c_int64(self.t), ctypes.c_double(self.lr), None,
                ctypes.c_double(self.betas[0]), ctypes.c_double(self.betas[1]),
                ctypes.c_double(self.eps), ctypes.c_double(self.weight_decay), _ptr(skip),
                _stream(dev))
            _lib.check("cnf_adam_step_guarded", st)
        else:
            st = lib.cnf_adam_step(ctypes.byref(self.stack.desc), arr, _ptr(flat_grads),
                                   _ptr(self._m), _ptr(self._v), ctypes.c_int64(self.t),
                                   ctypes.c_double(self.lr), ctypes.c_double(self.betas[0]),
                                   ctypes.c_double(self.betas[1]), ctypes.c_double(self.eps),
                                   ctypes.c_double(self.weight_decay), _stream(dev))
            _lib.check("cnf_adam_step", st)
        # the kernel wrote the parameters behind autograd's back: bump their
        # version counters, so every prepared-weight cache keyed on them (this
        # stack's and any other binding's) rebuilds
        for p in ps:
            torch.autograd.graph.increment_version(p)
        stats["adam"] = stats.get("adam", 0) + 1
