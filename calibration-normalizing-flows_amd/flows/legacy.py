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

The Keras-era NICE flows of code-old/nice.py are restated here too
(`LegacyNiceFlow`, version=1/2/3), additive (log-det 0, as the Keras models
have none):

* version 1, `NiceFlow` (code-old/nice.py:101-145) with the split coupling
  `AddCouplingLayer` (:55-77): x1 = x[:, :D//2], x2 = x[:, D//2:]; layer l
  even ('odd' mode): x2 += f_l(x1), f_l: D//2 -> D-D//2; layer l odd ('even'
  mode): x1 += f_l(x2), f_l: D-D//2 -> D//2.  No permutation.
* version 2, `NiceFlow_v2` (:158-211): every layer 'even' mode (x1 += f(x2))
  followed by a full reversal (`ReIndex`), one more reversal at the end for
  odd L.
* version 3, `NiceFlow_v3` (:214-263) with `AddCouplingLayer_v2` (:80-98):
  y = b*x + (1-b)*(x + f(b*x)), f = MLP(D -> D), the mask b = [0]*(D//2) +
  [1]*(D-D//2) flipped every layer; no data permutation.

`backward` is the true inverse for every version.  (The Keras v3 inverse
model, code-old/nice.py:232-245, applies the coupling functions in FORWARD
order with the reversed mask sequence -- it inverts only when every f_l is the
same function; that quirk is not reproduced.)

Versions 1 and 2 keep Keras' half-width conditioners and run natively by
zero-embedding them into the maintained NICE layer (_EmbeddedNice):
* version 2: its layer IS the maintained additive layer (x1 += f(x2) on the
  first D//2 features, conditioned on the rest, then a full reversal) whose
  t-net's first Linear sees only the conditioning columns and whose last
  Linear's transformed rows are f's; one more reversal ends an odd-L stack;
* version 1 (even D): with R the full reversal, a split layer in 'odd' mode
  is M_g(R x) and in 'even' mode R M_f(x), where M is the maintained layer and
  g is f with its input columns and output rows reversed; the stack is
  R^[L even] M_{f_{L-1}} ... M_{f_1} M_{g_0} (R x);
* version 1, odd D = 2h+1 (code-old/nice.py:140-155: its 'odd' layers add
  f(x1) to the LARGER half x2, h+1 features, which no mask of width D can
  express): the same stack over D+1 features, x' = [x1, 0, x2] -- a zero
  feature d appended to x1.  Both halves then hold h+1 features; in an 'odd'
  layer d is an input of f (a zero weight column), in an 'even' layer an
  output (a zero weight row and bias, so d stays exactly 0); the output drops
  d again.
Version 3 is the alternate-mask stack of the RealNVP path with the s-net
absent, so it runs natively as CNF_OPT_ALT_MASK on the shift-only kernels.
"""
import torch
import torch.nn.functional as F
from torch import nn

from .utils import MLP


class UnsupportedShape(Exception):
    """Stand-in until the native library is imported (CPU-only use)."""


def _not_native(why):
    from .flows import _not_native as nn_
    nn_(why)


def _bind_unsupported():
    global UnsupportedShape
    try:
        from cnf_hip._lib import UnsupportedShape as U
        UnsupportedShape = U
    except ImportError:
        pass


_bind_unsupported()

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
            try:
                stack = self._native_stack()
                if torch.is_grad_enabled() and (x.requires_grad or stack.requires_grad()):
                    if not stack.has_native_vjp():
                        # the torch VJP restates the maintained layer only
                        raise UnsupportedShape("cnf_vjp", -3, __import__("cnf_hip").lib())
                    return stack.forward_autograd(x, want_all=False)
                y, ld, _ = stack.run(x)
                return y, ld
            except UnsupportedShape as e:
                _not_native("legacy RealNVP %s" % e)
        ld = torch.zeros(x.shape[0], dtype=x.dtype, device=x.device)
        for ly in self.layers:
            x, l = ly(x)
            ld = ld + l
        return x, ld

    def backward(self, y):
        if self._native_ok(y):
            try:
                stack = self._native_stack()
                if torch.is_grad_enabled() and (y.requires_grad or stack.requires_grad()):
                    return stack.inverse_autograd(y, want_all=False)  # cnf_vjp_inverse
                x, ld, _ = stack.run(y, inverse=True)
                return x, ld
            except UnsupportedShape as e:
                _not_native("legacy RealNVP %s" % e)
        ld = torch.zeros(y.shape[0], dtype=y.dtype, device=y.device)
        for ly in reversed(self.layers):
            y, l = ly.backward(y)
            ld = ld + l
        return y, ld


def _mlp(n_in, hidden, n_out, act):
    """Keras MLP(input_dim, output_dim, hidden_size, activation)
    (code-old/nice.py:8-16): Dense(h, act) ... Dense(output_dim)."""
    widths = [n_in, *hidden, n_out]
    lins = nn.ModuleList(nn.Linear(a, b) for a, b in zip(widths[:-1], widths[1:]))
    return lins


def _run_mlp(lins, act, x):
    *hidden, last = lins
    for lin in hidden:
        x = act(lin(x))
    return last(x)


class LegacySplitCoupling(nn.Module):
    """AddCouplingLayer (code-old/nice.py:55-77): split x into x1 (first D//2)
    and x2 (rest); mode 'odd': x2 + f(x1); mode 'even': x1 + f(x2); inverse
    subtracts."""

    def __init__(self, dim, hidden_size, mode, activation="relu"):
        super().__init__()
        self.dim = dim
        self.mode = mode
        self.activation = activation
        h = dim // 2
        n_in, n_out = (h, dim - h) if mode == "odd" else (dim - h, h)
        self.f_hidden = list(hidden_size)
        self.f = _mlp(n_in, list(hidden_size), n_out, _ACT[activation])

    def _couple(self, x, sign):
        h = self.dim // 2
        x1, x2 = x[:, :h], x[:, h:]
        if self.mode == "odd":
            x2 = x2 + sign * _run_mlp(self.f, _ACT[self.activation], x1)
        else:
            x1 = x1 + sign * _run_mlp(self.f, _ACT[self.activation], x2)
        return torch.cat([x1, x2], dim=1)

    def forward(self, x):
        return self._couple(x, 1.0)

    def backward(self, y):
        return self._couple(y, -1.0)


class LegacyAddCoupling(nn.Module):
    """AddCouplingLayer_v2 (code-old/nice.py:80-98): y = b*x + (1-b)*(x +
    f(b*x)), f = MLP(dim -> dim); inverse: (1-b)*(y - f(b*y)).  The mask
    parity follows NiceFlow_v3 (:214-230): [0]*(D//2)+[1]*(D-D//2), flipped on
    odd layers.  Attributes the native stack reads: scale False (no s-net),
    shift True, t = the conditioner."""

    def __init__(self, dim, hidden_size, parity, activation="relu"):
        super().__init__()
        self.dim = dim
        self.hidden_size = list(hidden_size)
        self.parity = int(parity) & 1
        self.activation = activation
        self.s_activation = activation
        self.s = None
        self.t = MLP(dim, self.hidden_size, _ACT[activation])
        b = torch.zeros(1, dim)
        b[:, dim // 2:] = 1.0
        if self.parity:
            b = b.flip(1)
        self.register_buffer("mask", b)
        self.scale = False
        self.shift = True
        self.random_flip = False
        self.invertible = True

    def forward(self, x):
        b = self.mask
        x_b = b * x
        y = x_b + (1 - b) * (x + self.t(x_b))
        return y, torch.zeros(x.shape[0], dtype=x.dtype, device=x.device)

    def backward(self, y):
        b = self.mask
        y_b = b * y
        x = y_b + (1 - b) * (y - self.t(y_b))
        return x, torch.zeros(y.shape[0], dtype=y.dtype, device=y.device)


class _Lin:
    """What CouplingStack reads of an nn.Linear: .weight, .bias."""

    def __init__(self, weight, bias):
        self.weight, self.bias = weight, bias


class _Net:
    def __init__(self, lins):
        self.layers = lins


class _VirtualLayer:
    """A maintained NICE layer (flows/flows.py:68-126 with scale=False) as
    CouplingStack reads it, over zero-embedded full-width t-net tensors."""

    def __init__(self, dim, hidden, lins):
        self.dim, self.hidden_size = dim, list(hidden)
        self.scale, self.shift, self.random_flip = False, True, False
        self.s, self.t = None, _Net(lins)


class _EmbeddedNice:
    """Native plumbing of LegacyNiceFlow versions 1 / 2 (see the module
    docstring): full-width first / last t-net Linears kept in device buffers,
    refreshed from the half-width Keras conditioners whenever one of their
    parameters changed (in-place version counters); hidden Linears are the
    conditioners' own tensors.  rev[l]: layer l's conditioner enters with its
    input columns and output rows reversed (version 1, even layers).  pad:
    version 1 with odd D runs over D + 1 features (the zero feature d after
    x1; module docstring)."""

    def __init__(self, flow, device):
        self.flow = flow
        self.pad = 1 if (flow.version == 1 and flow.dim % 2) else 0
        D = flow.dim + self.pad  # the virtual stack's width
        h = D // 2
        self.D, self.h = D, h
        self.rev = [flow.version == 1 and l % 2 == 0 for l in range(len(flow.layers))]
        vls, self.fparams, self.bufs = [], [], []
        for ly in flow.layers:
            lins = list(ly.f)
            first, last = lins[0], lins[-1]
            bL = torch.zeros(D, device=device)
            if len(lins) > 1:
                W0 = torch.zeros(first.weight.shape[0], D, device=device)
                WL = torch.zeros(D, last.weight.shape[1], device=device)
                vl = [_Lin(W0, first.bias)] + [_Lin(l.weight, l.bias) for l in lins[1:-1]]
                vl.append(_Lin(WL, bL))
            else:  # no hidden layer: ONE Linear, embedded on both sides
                W0 = torch.zeros(D, D, device=device)
                WL = None
                vl = [_Lin(W0, bL)]
            vls.append(_VirtualLayer(D, ly.f_hidden, vl))
            self.bufs.append((W0, WL, bL))
            self.fparams.extend([l.weight for l in lins] + [l.bias for l in lins])
        from cnf_hip.engine import CouplingStack
        self.stack = CouplingStack(vls)
        self._key = None

    def key(self):
        return tuple((p.data_ptr(), p._version) for p in self.fparams)

    def _cols(self, rev):
        """First column of the conditioning block that holds f's inputs: with
        the pad, a reversed ('odd' mode) layer sees [d, x1 reversed] there."""
        return self.h + (self.pad if rev else 0)

    @torch.no_grad()
    def refresh(self):
        k = self.key()
        if k == self._key:
            return
        for ly, (W0, WL, bL), rev in zip(self.flow.layers, self.bufs, self.rev):
            lins = list(ly.f)
            first, last = lins[0], lins[-1]
            c0, n_out = self._cols(rev), last.weight.shape[0]
            if len(lins) > 1:
                W0[:, c0:].copy_(first.weight.flip(1) if rev else first.weight)
                WL[:n_out].copy_(last.weight.flip(0) if rev else last.weight)
                bL[:n_out].copy_(last.bias.flip(0) if rev else last.bias)
            else:
                w = first.weight.flip(0).flip(1) if rev else first.weight
                W0.zero_()
                W0[:n_out, c0:].copy_(w)
                bL.zero_()
                bL[:n_out].copy_(first.bias.flip(0) if rev else first.bias)
        self._key = k

    def grads_back(self, flat):
        """Flat gradient of the virtual stack (ABI order) -> per-parameter
        gradients of the Keras conditioners (fparams order)."""
        out_w, out_b = [], []
        off = 0
        for ly, rev in zip(self.flow.layers, self.rev):
            lins = list(ly.f)
            gw, gb = [], []
            c0, n_out = self._cols(rev), lins[-1].weight.shape[0]
            for i, lin in enumerate(lins):
                n_out_full = self.D if (i == len(lins) - 1) else lin.weight.shape[0]
                n_in_full = self.D if i == 0 else lin.weight.shape[1]
                W = flat[off:off + n_out_full * n_in_full].view(n_out_full, n_in_full)
                off += n_out_full * n_in_full
                b = flat[off:off + n_out_full]
                off += n_out_full
                if i == 0:
                    W = W[:, c0:]
                if i == len(lins) - 1:
                    W, b = W[:n_out], b[:n_out]
                if rev and i == 0:
                    W = W.flip(1)
                if rev and i == len(lins) - 1:
                    W, b = W.flip(0), b.flip(0)
                gw.append(W.contiguous())
                gb.append(b.contiguous())
            out_w.extend(gw)
            out_b.extend(gb)
        # fparams order per layer: weights then biases
        res, iw, ib = [], 0, 0
        for ly in self.flow.layers:
            n = len(list(ly.f))
            res.extend(out_w[iw:iw + n] + out_b[ib:ib + n])
            iw += n
            ib += n
        return res


class _EmbedFn(torch.autograd.Function):
    """The virtual stack's transform (inverse=False) or inverse as one native
    launch, gradients through cnf_vjp / cnf_vjp_inverse mapped back onto the
    half-width conditioners."""

    @staticmethod
    def forward(ctx, emb, inverse, x, *fparams):
        emb.refresh()
        fin, ld, _ = emb.stack.run(x, inverse=inverse)
        ctx.emb, ctx.inverse, ctx.key = emb, inverse, emb.key()
        ctx.save_for_backward(x)
        return fin, ld

    @staticmethod
    def backward(ctx, g_out, g_ld):
        from cnf_hip.vjp import stack_vjp, stack_vjp_inverse
        (x,) = ctx.saved_tensors
        emb = ctx.emb
        if emb.key() != ctx.key:
            raise RuntimeError("one of the variables needed for gradient computation has been "
                               "modified by an inplace operation: a legacy NICE conditioner "
                               "changed between the native pass and its backward")
        fn = stack_vjp_inverse if ctx.inverse else stack_vjp
        dx, grads = fn(emb.stack, x, g_out, g_ld, False, ctx.needs_input_grad[2])
        flat = torch.cat([g.reshape(-1) for g in grads])
        return (None, None, dx) + tuple(emb.grads_back(flat))


class LegacyNiceFlow(nn.Module):
    """The NICE flows of code-old/nice.py in torch (see the module docstring):
    version 1 `NiceFlow`, 2 `NiceFlow_v2`, 3 `NiceFlow_v3`; default hidden
    [dim], 4 layers (:104-111).  forward(x) -> (y, ld = 0); backward(y) ->
    (x, ld = 0)."""

    def __init__(self, dim, layers=4, hidden_size=None, activation="relu", version=1, **kwargs):
        super().__init__()
        hidden_size = [dim] if hidden_size is None else list(hidden_size)
        if version not in (1, 2, 3):
            raise ValueError("LegacyNiceFlow version must be 1, 2 or 3")
        self.dim = dim
        self.version = version
        self.n_layers = layers
        if version == 1:
            mods = [LegacySplitCoupling(dim, hidden_size, "even" if l % 2 else "odd", activation)
                    for l in range(layers)]
        elif version == 2:
            mods = [LegacySplitCoupling(dim, hidden_size, "even", activation) for _ in range(layers)]
        else:
            mods = [LegacyAddCoupling(dim, hidden_size, l, activation) for l in range(layers)]
        self.layers = nn.ModuleList(mods)
        self.invertible = True
        self._stack = None
        self._emb = None

    # -- native plumbing ---------------------------------------------------
    def _native_ok(self, x):
        if not (isinstance(x, torch.Tensor) and x.is_cuda and x.dtype == torch.float32
                and x.dim() == 2 and x.shape[1] == self.dim):
            return False
        from flows.flows import _not_native
        if self.layers[0].activation != "relu":
            _not_native("legacy NICE activation %r" % self.layers[0].activation)
            return False
        return True

    def _native_stack(self):
        if self._stack is None:
            from cnf_hip import _lib
            from cnf_hip.engine import CouplingStack
            self._stack = CouplingStack(list(self.layers), options=_lib.OPT_ALT_MASK)
        return self._stack

    def _embedded(self, device):
        emb = self._emb
        if emb is None or emb.bufs[0][0].device != device:
            emb = self._emb = _EmbeddedNice(self, device)
        return emb

    def _native_split(self, x, inverse):
        """Versions 1 / 2 on the virtual maintained stack (module docstring)."""
        emb = self._embedded(x.device)
        L = len(self.layers)
        pre = self.version == 1          # R before the stack (after, for the inverse)
        post = (self.version == 1 and L % 2 == 0) or (self.version == 2 and L % 2 == 1)
        if inverse:
            pre, post = post, pre
        h0 = self.dim // 2
        if emb.pad:  # x' = [x1, d = 0, x2]
            x = torch.cat([x[:, :h0], x.new_zeros(x.shape[0], 1), x[:, h0:]], dim=1)
        if pre:
            x = x.flip(1)
        fparams = emb.fparams
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in fparams)):
            y, ld = _EmbedFn.apply(emb, inverse, x.contiguous(), *fparams)
        else:
            emb.refresh()
            y, ld, _ = emb.stack.run(x.contiguous(), inverse=inverse)
        if post:
            y = y.flip(1)
        if emb.pad:  # drop d (exactly 0 throughout)
            y = torch.cat([y[:, :h0], y[:, h0 + 1:]], dim=1)
        return y, ld

    def invalidate_native(self):
        self._stack = None
        self._emb = None

    def __getstate__(self):
        st = self.__dict__.copy()
        st["_stack"] = None
        st["_emb"] = None
        return st

    @staticmethod
    def _rev(x):
        return x.flip(1)  # ReIndex() with the default index (code-old/nice.py:38-51)

    def forward(self, x):
        if self._native_ok(x) and self.version != 3:
            try:
                return self._native_split(x, inverse=False)
            except UnsupportedShape as e:
                _not_native("legacy NICE %s" % e)
        elif self._native_ok(x):
            try:
                stack = self._native_stack()
                if torch.is_grad_enabled() and (x.requires_grad or stack.requires_grad()):
                    if not stack.has_native_vjp():
                        # the torch VJP restates the maintained layer only
                        raise UnsupportedShape("cnf_vjp", -3, __import__("cnf_hip").lib())
                    return stack.forward_autograd(x, want_all=False)
                y, ld, _ = stack.run(x)
                return y, ld
            except UnsupportedShape as e:
                _not_native("legacy NICE %s" % e)
        ld = torch.zeros(x.shape[0], dtype=x.dtype, device=x.device)
        for ly in self.layers:
            x = ly(x)[0] if self.version == 3 else ly(x)
            if self.version == 2:
                x = self._rev(x)
        if self.version == 2 and len(self.layers) % 2 == 1:
            x = self._rev(x)
        return x, ld

    def backward(self, y):
        if self._native_ok(y) and self.version != 3:
            try:
                return self._native_split(y, inverse=True)
            except UnsupportedShape as e:
                _not_native("legacy NICE %s" % e)
        elif self._native_ok(y):
            try:
                stack = self._native_stack()
                if torch.is_grad_enabled() and (y.requires_grad or stack.requires_grad()):
                    return stack.inverse_autograd(y, want_all=False)
                x, ld, _ = stack.run(y, inverse=True)
                return x, ld
            except UnsupportedShape as e:
                _not_native("legacy NICE %s" % e)
        ld = torch.zeros(y.shape[0], dtype=y.dtype, device=y.device)
        if self.version == 2 and len(self.layers) % 2 == 1:
            y = self._rev(y)
        for ly in reversed(self.layers):
            if self.version == 2:
                y = self._rev(y)
            y = ly.backward(y)[0] if self.version == 3 else ly.backward(y)
        return y, ld
