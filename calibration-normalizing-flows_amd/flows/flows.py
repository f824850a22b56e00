"""Drop-in replacement for the reference's flows/flows.py.

Same classes, constructor arguments, attributes, state_dict keys and return
conventions as the reference (SergioAlvarezB/calibration-normalizing-flows,
flows/flows.py), so `from flows.flows import Flow, NvpCouplingLayer` works
unchanged.  On a ROCm device a Flow made of NvpCouplingLayers runs as ONE fused
HIP launch per call (libcnf_hip.so, include/cnf.h):

  Flow.forward(x)  -> (zs, cum_log_det)   fused cnf_forward, zs = views of one
                                           [L, B, D] buffer       (flows.py:17-25)
  Flow.backward(z) -> (xs, cum_log_det)   fused cnf_inverse        (flows.py:27-37)
  NvpCouplingLayer.forward / .backward    the same kernels, L = 1  (flows.py:101-126)

`backward` is the reference's name for the INVERSE transform; gradients come
from torch autograd, which calls the native VJP kernel.

Host tensors (CPU) run the same math with torch ops, as the reference does.
Layers the native engine does not cover (AffineConstantLayer, PlanarLayer,
RadialLayer -- out of the hot-path scope) also run as torch ops.
"""
import os
import warnings

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from .utils import MLP

# Reproduce the reference's `0 * inf = NaN` at masked positions when exp(s)
# overflows there (flows/flows.py:107).  Off by default: it costs the kernel
# the masked half of the last Linear; finite results are identical either way.
STRICT_NAN = os.environ.get("CNF_STRICT_NAN", "0") == "1"
# Raise instead of running torch ops when a ROCm tensor cannot take the
# native path (unsupported shape or activation).
STRICT_NATIVE = os.environ.get("CNF_STRICT_NATIVE", "0") == "1"

_warned = set()


def _not_native(reason):
    if STRICT_NATIVE:
        raise RuntimeError("native coupling path unavailable: " + reason)
    if reason not in _warned:
        _warned.add(reason)
        warnings.warn("cnf: running torch ops on the GPU (%s)" % reason, RuntimeWarning)


def _needs_grad(x, module):
    if not torch.is_grad_enabled():
        return False
    return x.requires_grad or any(p.requires_grad for p in module.parameters())


def _native_eligible(layers, x):
    """True when these layers can run as one fused native stack on x."""
    if not (isinstance(x, torch.Tensor) and x.is_cuda):
        return False
    if x.dtype != torch.float32 or x.dim() != 2:
        return False
    if not layers or not all(isinstance(ly, NvpCouplingLayer) for ly in layers):
        return False
    for ly in layers:
        for net in (ly.s, ly.t):
            if isinstance(net, MLP) and net.activation is not F.relu:
                _not_native("conditioner activation %r" % (net.activation,))
                return False
    from cnf_hip.engine import CouplingStack
    if not CouplingStack.compatible(layers):
        return False
    if x.shape[1] != layers[0].dim:
        return False
    return True


def _squeeze_ld(ld):
    # torch.sum(..., dim=1).squeeze(): 0-d for a single row (flows/flows.py:109)
    return ld.squeeze()


class Flow(nn.Module):
    """Sequential flow (reference flows/flows.py:8-37)."""

    def __init__(self, layers, **kwargs):
        super().__init__()
        self.layers = nn.ModuleList(layers)
        # a flow is computationally invertible iff every layer is
        self.invertible = all(ly.invertible for ly in self.layers)
        self.strict_nan = kwargs.get("strict_nan", None)
        # cnf_desc.options bits (cnf_hip._lib.OPT_*): keep launches off a kernel
        # family, for A/B runs and tests; 0 = the fastest kernel
        self.native_options = int(kwargs.get("native_options", 0))
        self._stack = None
        self._stack_key = None

    def __getstate__(self):
        # the native binding (ctypes descriptor, device blobs) is rebuilt lazily
        st = self.__dict__.copy()
        st["_stack"] = None
        st["_stack_key"] = None
        return st

    # -- native plumbing --------------------------------------------------
    def _native_stack(self):
        key = (tuple(id(ly) for ly in self.layers), self._strict(), self.native_options)
        if self._stack is None or self._stack_key != key:
            from cnf_hip.engine import CouplingStack
            self._stack = CouplingStack(list(self.layers), strict_nan=self._strict(),
                                        options=self.native_options)
            self._stack_key = key
        return self._stack

    def invalidate_native(self):
        """Drop the native binding's prepared weights.  Needed only after writes
        that bypass torch's version counters (`p.data.copy_(...)`); optimizer
        steps, `load_state_dict` and in-place ops are tracked automatically."""
        self._stack = None
        self._stack_key = None
        for ly in self.layers:
            if isinstance(ly, NvpCouplingLayer):
                ly._stack = None

    def _strict(self):
        return STRICT_NAN if self.strict_nan is None else bool(self.strict_nan)

    def _try_native(self, x, inverse, want_all=True):
        """(zs list | final z, log-det) from one fused launch, or None."""
        if not _native_eligible(list(self.layers), x):
            return None
        from cnf_hip._lib import UnsupportedShape
        stack = self._native_stack()
        try:
            if torch.is_grad_enabled() and (x.requires_grad or stack.requires_grad()):
                if inverse:  # cnf_vjp_inverse (strict_nan included)
                    out, ld = stack.inverse_autograd(x, want_all=want_all)
                else:
                    out, ld = stack.forward_autograd(x, want_all=want_all)
            else:
                fin, ld, allt = stack.run(x, inverse=inverse, want_all=want_all)
                out = allt if want_all else fin
            return (list(out.unbind(0)) if want_all else out), _squeeze_ld(ld)
        except UnsupportedShape as e:
            _not_native(str(e))
            return None

    def transform(self, x):
        """Final output and log-det only -- (zs[-1], cum_log_det) without
        materialising the intermediate layer outputs."""
        out = self._try_native(x, inverse=False, want_all=False)
        if out is not None:
            return out
        zs, ld = Flow.forward(self, x)
        return zs[-1], ld

    def inverse_transform(self, z):
        """(xs[-1], cum_log_det) of Flow.backward without the intermediates."""
        if not self.invertible:
            raise ValueError('Flow inverse not tractable!')
        out = self._try_native(z, inverse=True, want_all=False)
        if out is not None:
            return out
        xs, ld = Flow.backward(self, z)
        return xs[-1], ld

    # -- reference API ----------------------------------------------------
    def forward(self, x):
        out = self._try_native(x, inverse=False)
        if out is not None:
            return out
        cum_log_det = 0.0
        zs = []
        for layer in self.layers:
            x, log_det = layer(x)
            zs.append(x)
            cum_log_det += log_det
        return zs, cum_log_det

    def backward(self, z):
        if not self.invertible:
            raise ValueError('Flow inverse not tractable!')
        out = self._try_native(z, inverse=True)
        if out is not None:
            return out
        cum_log_det = 0.0
        xs = []
        for layer in reversed(self.layers):
            z, log_det = layer.backward(z)
            xs.append(z)
            cum_log_det += log_det
        return xs, cum_log_det


class AffineConstantLayer(nn.Module):
    """z = x*exp(s) + t with per-feature constants (reference flows/flows.py:40-65).
    Not a coupling layer: torch ops on every device."""

    def __init__(self, dim, scale=True, shift=True):
        super().__init__()
        self.s = nn.Parameter(torch.zeros(1, dim, requires_grad=True)) if scale else None
        self.t = nn.Parameter(torch.zeros(1, dim, requires_grad=True)) if shift else None
        self.invertible = True

    def _st(self, x):
        s = self.s if self.s is not None else x.new_zeros(x.size())
        t = self.t if self.t is not None else x.new_zeros(x.size())
        return s, t

    def forward(self, x):
        s, t = self._st(x)
        return x * torch.exp(s) + t, torch.sum(s, dim=1)

    def backward(self, z):
        s, t = self._st(z)
        return (z - t) * torch.exp(-s), torch.sum(-s, dim=1)


class NvpCouplingLayer(nn.Module):
    """RealNVP affine coupling (NICE additive when scale=False), fixed half
    mask, feature flip after the layer, optional random permutation
    (reference flows/flows.py:68-126)."""

    def __init__(self, dim, hidden_size=[5, 5], scale=True, shift=True, random_flip=False):
        super().__init__()
        # conditioner nets; the reference draws their init in this order
        self.s = MLP(dim, hidden_size, wscale=0.001) if scale \
            else (lambda x: x.new_zeros(x.size()))
        self.t = MLP(dim, hidden_size, wscale=0.001) if shift \
            else (lambda x: x.new_zeros(x.size()))
        mask = np.zeros((1, dim))
        mask[:, dim // 2:] = 1
        self.mask = nn.Parameter(torch.as_tensor(mask.copy(), dtype=torch.float),
                                 requires_grad=False)
        self.invertible = True
        self.random_flip = random_flip
        # shape record used by the native engine (not part of the state_dict)
        self.dim = dim
        self.hidden_size = list(hidden_size)
        self.scale = bool(scale)
        self.shift = bool(shift)
        self.strict_nan = None
        self._stack = None
        if random_flip:
            perm = np.random.permutation(dim)
            rev = np.zeros(dim)
            rev[perm] = np.arange(dim)
            self.perm = nn.Parameter(torch.as_tensor(perm[None], dtype=torch.long),
                                     requires_grad=False)
            self.rev_perm = nn.Parameter(torch.as_tensor(rev[None], dtype=torch.long),
                                         requires_grad=False)

    def __getstate__(self):
        st = self.__dict__.copy()
        st["_stack"] = None
        return st

    def _native(self, x, inverse):
        if not _native_eligible([self], x):
            return None
        from cnf_hip._lib import UnsupportedShape
        from cnf_hip.engine import CouplingStack
        strict = STRICT_NAN if self.strict_nan is None else bool(self.strict_nan)
        if self._stack is None or self._stack.strict_nan != strict:
            self._stack = CouplingStack([self], strict_nan=strict)
        try:
            if _needs_grad(x, self):
                if inverse:  # cnf_vjp_inverse (strict_nan included)
                    z, ld = self._stack.inverse_autograd(x, want_all=False)
                else:
                    z, ld = self._stack.forward_autograd(x, want_all=False)
            else:
                z, ld, _ = self._stack.run(x, inverse=inverse)
            return z, _squeeze_ld(ld)
        except UnsupportedShape as e:
            _not_native(str(e))
            return None

    def forward(self, x):
        out = self._native(x, inverse=False)
        if out is not None:
            return out
        keep = self.mask * x              # conditioning half (mask = 1)
        free = 1 - self.mask              # transformed half
        s, t = self.s(keep), self.t(keep)
        z = keep + free * (x * torch.exp(s) + t)
        log_det = torch.sum(free * s, dim=1).squeeze()
        if self.random_flip:
            z = z[:, self.perm.reshape(-1)]
        return z.flip((1,)), log_det

    def backward(self, z):
        out = self._native(z, inverse=True)
        if out is not None:
            return out
        z = z.flip((1,))
        if self.random_flip:
            z = z[:, self.rev_perm.reshape(-1)]
        keep = self.mask * z
        free = 1 - self.mask
        s, t = self.s(keep), self.t(keep)
        x = keep + free * (z - t) * torch.exp(-s)
        log_det = torch.sum(free * (-s), dim=1).squeeze()
        return x, log_det


class PlanarLayer(nn.Module):
    """Planar flow (reference flows/flows.py:129-165); non-invertible.
    Torch ops on every device (outside the coupling hot path)."""

    def __init__(self, dim=0, params=None):
        super().__init__()
        if params is not None:
            self.w = params['w'].squeeze()
            self.u = params['u'].squeeze()
            self.b = params['b'].squeeze()
        else:
            if dim < 1:
                raise ValueError('Either dim of params must be provided!')
            self.w = nn.Parameter(torch.rand(dim))
            self.u = nn.Parameter(torch.rand(dim))
            self.b = nn.Parameter(torch.rand(1))
        self.invertible = False

    def forward(self, x):
        wtu = torch.dot(self.w, self.u)
        m = -1 + torch.log1p(torch.exp(wtu))   # keeps w.u_hat >= -1
        u_hat = self.u + (m - wtu) * self.w / torch.norm(self.w)
        h = torch.tanh(torch.matmul(x, self.w) + self.b)
        z = x + torch.matmul(h.view(-1, 1), u_hat.view(1, -1))
        psi = torch.matmul((1 - h ** 2).view(-1, 1), self.w.view(1, -1))
        det = torch.abs(1 + torch.matmul(psi, u_hat.view(-1, 1)))
        return z, torch.log(det.squeeze())


class RadialLayer(nn.Module):
    """Radial flow (reference flows/flows.py:168-193); non-invertible.  Its
    log-det is the constant log(1) = 0, as in the reference."""

    def __init__(self, dim):
        super().__init__()
        self.z0 = nn.Parameter(torch.rand(dim))
        self.a = nn.Parameter(torch.rand(1))
        self.b = nn.Parameter(torch.rand(1))
        self.invertible = False

    def forward(self, x):
        b_hat = -self.a + torch.log1p(torch.exp(self.b))
        diff = x - self.z0
        h = 1. / (self.a + torch.norm(diff, dim=1, keepdim=True))
        z = x + b_hat * h.expand_as(diff) * diff
        return z, torch.log(torch.tensor(1.0))
