"""Legacy (TensorFlow-era) RealNVP semantics of the reference, restated in
torch and served by the native MFMA-tile kernels on a ROCm device.

The reference's `code-old/realNVP.py:8-92` (Keras; TensorFlow is absent here,
so parity is UNPINNED: the torch restatement below is the only check, see
DESIGN.md) differs from the maintained `flows/flows.py` coupling flow in two
ways, exposed as options:

* mask_mode='alternate_mask' (code-old/realNVP.py:66-76): layer l uses the
  mask b = [0]*(D//2) + [1]*(D-D//2) for even l and its flip for odd l; the
  data are never flipped.  (`flows.flows` keeps one mask and flips the data.)
* s_activation='tanh' (code-old/realNVP.py:58-64): the s-net's hidden layers
  use tanh, the t-net's use `activation` (ReLU by default).

Everything else follows code-old/realNVP.py:19-38 (`NvpCoupling.call`):
    y = x_b + (1-b) * (x * exp(s(x_b)) + t(x_b)),      x_b = b * x
    x = y_b + (1-b) * (y - t(y_b)) / exp(s(y_b))       (backward=True)
with the conditioners `MLP(dim, hidden, act)` = Dense(h, act)... Dense(dim)
(code-old/realNVP.py:8-16).  The Keras model returns no log-det; this module
also returns ld = sum((1-b) * s) (the maintained flow's convention) so the
calibrator losses apply.

Native path: the stack runs as cnf_desc options CNF_OPT_ALT_MASK (| S_TANH) on
the flip-based kernels with odd layers' weights reversed at prepare time
(include/cnf.h); gradients come back in this module's parameter layout.
"""
import torch
import torch.nn.functional as F
from torch import nn

from .utils import MLP

_ACT = {"relu": F.relu, "tanh": torch.tanh}


class LegacyNvpCoupling(nn.Module):
    """One Keras-era coupling layer (code-old/realNVP.py:19-38) with an
    explicit mask parity (0: transform the first D//2 features)."""

    def __init__(self, dim, hidden_size, parity, s_activation="tanh", activation="relu"):
        super().__init__()
        self.dim = dim
        self.hidden_size = list(hidden_size)
        self.parity = int(parity) & 1
        self.s_activation = s_activation
        self.activation = activation
        self.s = MLP(dim, self.hidden_size, _ACT[s_activation])
        self.t = MLP(dim, self.hidden_size, _ACT[activation])
        b = torch.zeros(1, dim)
        b[:, dim // 2:] = 1.0
        if self.parity:
            b = b.flip(1)  # np.flip(b) (code-old/realNVP.py:73)
        self.register_buffer("mask", b)
        # the native stack reads these (cnf_hip/engine.py CouplingStack)
        self.scale = True
        self.shift = True
        self.random_flip = False
        self.invertible = True

    def forward(self, x):
        b = self.mask
        x_b = b * x
        s = self.s(x_b)
        y = x_b + (1 - b) * (x * torch.exp(s) + self.t(x_b))
        return y, torch.sum((1 - b) * s, dim=1)

    def backward(self, y):
        b = self.mask
        y_b = b * y
        s = self.s(y_b)
        x = y_b + (1 - b) * ((y - self.t(y_b)) / torch.exp(s))
        return x, -torch.sum((1 - b) * s, dim=1)


class LegacyRealNvpFlow(nn.Module):
    """`RealNvpFlow` of code-old/realNVP.py:44-92 in torch: `layers` coupling
    layers with alternating masks, tanh s-nets and `activation` t-nets.
    forward(x) -> (y, ld);  backward(y) -> (x, ld)."""

    def __init__(self, dim, layers=4, hidden_size=None, activation="relu", s_activation="tanh",
                 **kwargs):
        super().__init__()
        hidden_size = [dim] if hidden_size is None else list(hidden_size)  # :50-51
        self.dim = dim
        self.layers = nn.ModuleList([
            LegacyNvpCoupling(dim, hidden_size, l, s_activation, activation)
            for l in range(layers)])
        self.invertible = True
        self._stack = None

    # -- native plumbing --------------------------------------------------
    def _native_ok(self, x):
        if not (isinstance(x, torch.Tensor) and x.is_cuda and x.dtype == torch.float32
                and x.dim() == 2 and x.shape[1] == self.dim):
            return False
        ly = self.layers[0]
        # the kernels' t-net is ReLU; the s-net ReLU or tanh
        return ly.activation == "relu" and ly.s_activation in ("relu", "tanh")

    def _native_stack(self):
        if self._stack is None:
            from cnf_hip import _lib
            from cnf_hip.engine import CouplingStack
            opts = _lib.OPT_ALT_MASK | (_lib.OPT_S_TANH if self.layers[0].s_activation == "tanh"
                                        else 0)
            self._stack = CouplingStack(list(self.layers), options=opts)
        return self._stack

    def invalidate_native(self):
        self._stack = None

    def __getstate__(self):
        st = self.__dict__.copy()
        st["_stack"] = None
        return st

    def forward(self, x):
        if self._native_ok(x):
            stack = self._native_stack()
            if torch.is_grad_enabled() and (x.requires_grad or stack.requires_grad()):
                y, ld = stack.forward_autograd(x, want_all=False)
            else:
                y, ld, _ = stack.run(x)
            return y, ld
        ld = torch.zeros(x.shape[0], dtype=x.dtype, device=x.device)
        for ly in self.layers:
            x, l = ly(x)
            ld = ld + l
        return x, ld

    def backward(self, y):
        if self._native_ok(y):
            stack = self._native_stack()
            if torch.is_grad_enabled() and (y.requires_grad or stack.requires_grad()):
                return stack.inverse_autograd(y, want_all=False)  # cnf_vjp_inverse
            x, ld, _ = stack.run(y, inverse=True)
            return x, ld
        ld = torch.zeros(y.shape[0], dtype=y.dtype, device=y.device)
        for ly in reversed(self.layers):
            y, l = ly.backward(y)
            ld = ld + l
        return y, ld
