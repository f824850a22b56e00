"""Host side of the native coupling-flow path: descriptor, prepared-weight
cache, launches on torch's current HIP stream, and the autograd binding.

`CouplingStack` binds a run of identically-shaped NvpCouplingLayers to ONE
fused launch (cnf_forward / cnf_inverse / cnf_vjp in include/cnf.h).  All
buffers are torch allocations on the input's device; the stream is
`torch.cuda.current_stream()`, so launches order with surrounding torch work
and can be captured into a CUDA(HIP) graph.

Cache validity.  The prepared blob (weights re-laid out for the kernels, the
flip / random_flip permutation folded into gather tables) is rebuilt whenever
a parameter's or a permutation's storage or in-place version changes: optimizer
steps, `load_state_dict` and `copy_` all bump `_version`.  Writes through
`.data` do not (torch hides them from autograd too); after such a write call
`Flow.invalidate_native()` (or `CouplingStack.invalidate()`).  A backward whose
weights changed in place since its forward raises, as autograd does.
"""
import ctypes

import torch

from . import _lib

# counts of native launches (tests assert the HIP path really ran); "torch_ops"
# counts the launches that went through the torch.library operators
stats = {"forward": 0, "inverse": 0, "prepare": 0, "vjp": 0, "loss_vjp": 0, "predict": 0,
         "torch_ops": 0}

# Dispatch through torch.ops.cnf (C++ operators, autograd in C++) when
# libcnf_torch.so is built; False: the ctypes calls of the same C ABI.
USE_TORCH_OPS = True


def _ops():
    return _lib.torch_ops() if USE_TORCH_OPS else None


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _stream_key(device):
    return (device, torch.cuda.current_stream(device).cuda_stream)


class CouplingStack:
    """A fused stack of NvpCouplingLayers (flows/flows.py:68-126) sharing
    dim / hidden_size / scale / shift.  Layers keep owning their parameters;
    the stack only reads them (state_dict order) through cnf_prepare."""

    def __init__(self, layers, strict_nan=False, options=0):
        layers = list(layers)
        l0 = layers[0]
        self.layers = layers
        self.dim = l0.dim
        self.hidden = list(l0.hidden_size)
        self.scale = bool(l0.scale)
        self.shift = bool(l0.shift)
        self.strict_nan = bool(strict_nan)
        self.options = int(options)
        self.L = len(layers)
        self._perm_key = None
        self._perms = None
        # the Parameter objects are fixed for the stack's life (load_state_dict
        # and .to() update them in place); nn.Module attribute lookups cost
        # ~4 us each, so the list is gathered once
        self._params = self._gather_params()
        self._refresh_desc()
        self._cache = {}
        self._loss_ws = {}
        self._vjp_ok = None
        self._vjp_inv_ok = None

    # -- descriptor and permutations ----------------------------------------
    def _perm_tensors(self):
        return [ly.perm for ly in self.layers if ly.random_flip]

    def _perm_state(self):
        return tuple((p.data_ptr(), p._version) for p in self._perm_tensors())

    def _refresh_desc(self):
        """(Re)build the host permutation table and the descriptor from the
        layers' current `perm` values (one small D2H copy, only on change)."""
        self._perm_key = self._perm_state()
        if any(ly.random_flip for ly in self.layers):
            p = torch.full((self.L, self.dim), -1, dtype=torch.int64)
            for i, ly in enumerate(self.layers):
                if ly.random_flip:
                    p[i] = ly.perm.detach().reshape(-1).cpu()
            self._perms = p.contiguous()
        else:
            self._perms = None
        self.desc = _lib.make_desc(self.dim, self.L, self.hidden, self.scale, self.shift,
                                   self.strict_nan, self._perms, self.options)
        self.desc_ints = _lib.desc_list(self.desc)

    def invalidate(self):
        """Forget every prepared blob (after writes the version counters do
        not see, e.g. through `.data`)."""
        self._cache.clear()
        self._perm_key = None

    @staticmethod
    def compatible(layers):
        l0 = layers[0]
        return all(ly.dim == l0.dim and list(ly.hidden_size) == list(l0.hidden_size)
                   and ly.scale == l0.scale and ly.shift == l0.shift for ly in layers)

    def kernel_name(self, all_outputs=False):
        """Kernel family serving this stack; every-layer-output calls of an
        sgpr-fused stack run on valu-fused (cnf_valu.hip valu_run)."""
        name = _lib.lib().cnf_kernel_name(ctypes.byref(self.desc)).decode()
        return "valu-fused" if all_outputs and name == "sgpr-fused" else name

    def has_native_vjp(self):
        """True when cnf_vjp serves this descriptor (every shape within the
        ABI's limits, strict_nan included, except strict stacks under the legacy
        alternate mask or tanh s-net).  Cached: support depends only on the
        shape and options."""
        if self._vjp_ok is None:
            n = ctypes.c_size_t()
            st = _lib.lib().cnf_vjp_workspace_bytes(ctypes.byref(self.desc), ctypes.c_int64(1),
                                                    ctypes.byref(n))
            self._vjp_ok = st == 0
        return self._vjp_ok

    def param_tensors(self):
        """ABI order (include/cnf.h cnf_param_tensor_count)."""
        return self._params

    def _gather_params(self):
        out = []
        for ly in self.layers:
            for net, on in ((ly.s, self.scale), (ly.t, self.shift)):
                if on:
                    for lin in net.layers:
                        out.append(lin.weight)
                        out.append(lin.bias)
        return out

    def param_count(self):
        n = ctypes.c_int64()
        _lib.check("cnf_param_count", _lib.lib().cnf_param_count(ctypes.byref(self.desc),
                                                                  ctypes.byref(n)))
        return n.value

    def state_key(self):
        """Identity of everything the prepared blob encodes."""
        return (tuple([(p.data_ptr(), p._version) for p in self._params]), self._perm_state())

    def requires_grad(self):
        return any([p.requires_grad for p in self._params])

    def prepared(self, device):
        """Device blob for this stack, rebuilt only when a parameter or a
        permutation changed (storage or in-place version counter)."""
        if self._perm_state() != self._perm_key:
            self._refresh_desc()
            self._cache.clear()
        key = self.state_key()
        ent = self._cache.get(device)
        if ent is not None and ent[0] == key:
            return ent[1]
        ps = self._params
        for p in ps:
            if p.device != device or p.dtype != torch.float32:
                raise TypeError("native coupling path needs fp32 parameters on %s" % device)
        lib = _lib.lib()
        nbytes = ctypes.c_size_t()
        _lib.check("cnf_prepared_bytes", lib.cnf_prepared_bytes(ctypes.byref(self.desc),
                                                                 ctypes.byref(nbytes)))
        blob = torch.empty(max(nbytes.value, 16), dtype=torch.uint8, device=device)
        cps = [p.detach().contiguous() for p in ps]
        arr = (ctypes.c_void_p * max(len(cps), 1))(*[c.data_ptr() for c in cps])
        _lib.check("cnf_prepare", lib.cnf_prepare(ctypes.byref(self.desc), arr, _ptr(blob),
                                                  _stream(device)))
        stats["prepare"] += 1
        # keep the parameter tensors referenced so the key's pointers stay theirs
        self._cache[device] = (key, blob, cps)
        return blob

    # ---------------------------------------------------------------- launches
    def _check_input(self, x):
        if not x.is_cuda:
            raise RuntimeError("native coupling path needs a ROCm device tensor")
        if x.dtype != torch.float32:
            raise TypeError("native coupling path is fp32 (the reference's nn.Linear weights "
                            "are fp32); got %s" % x.dtype)
        if x.dim() != 2 or x.shape[1] != self.dim:
            raise ValueError("expected [B, %d] logits, got %s" % (self.dim, tuple(x.shape)))
        return x.contiguous()

    def run(self, x, inverse=False, want_all=False, want_final=True, blob=None):
        """Returns (final [B,D] or None, logdet [B], all [L,B,D] or None)."""
        x = self._check_input(x)
        B = x.shape[0]
        dev = x.device
        if blob is None:
            blob = self.prepared(dev)
        ops = _ops()
        if ops is not None:
            out, ld = ops.forward(x, blob, self.desc_ints, self._perms, inverse, want_all)
            stats["inverse" if inverse else "forward"] += 1
            stats["torch_ops"] += 1
            if want_all:
                return (out[-1] if want_final else None), ld, out
            return out, ld, None
        ld = torch.empty(B, dtype=torch.float32, device=dev)
        allt = torch.empty(self.L, B, self.dim, dtype=torch.float32, device=dev) \
            if want_all else None
        fin = torch.empty(B, self.dim, dtype=torch.float32, device=dev) \
            if (want_final and not want_all) else None
        lib = _lib.lib()
        fn = lib.cnf_inverse if inverse else lib.cnf_forward
        st = fn(ctypes.byref(self.desc), _ptr(blob), _ptr(x), _ptr(fin), _ptr(ld), _ptr(allt),
                ctypes.c_int64(B), _stream(dev))
        _lib.check("cnf_inverse" if inverse else "cnf_forward", st)
        stats["inverse" if inverse else "forward"] += 1
        if want_all and want_final:
            fin = allt[-1]
        return fin, ld, allt

    def forward_loss(self, x, y, kind=_lib.LOSS_CAL, det=1.0, want_outputs=False,
                     terms_out=None):
        """Fused forward + log-det + loss terms (cnf_forward_loss): returns
        (terms[3] = sums over the rows of (loss, ce, log-det), z or None, ld or None).
        A label outside [0, D) makes the terms NaN (the reference raises).
        terms_out: a caller-provided fp32 [3] destination on x's device."""
        x = self._check_input(x)
        y = y.contiguous().to(torch.int64)
        B = x.shape[0]
        dev = x.device
        blob = self.prepared(dev)
        lib = _lib.lib()
        n = ctypes.c_size_t()
        _lib.check("cnf_forward_loss_workspace_bytes",
                   lib.cnf_forward_loss_workspace_bytes(ctypes.byref(self.desc),
                                                        ctypes.c_int64(B), ctypes.byref(n)))
        # one workspace per (device, stream): launches on two streams never share
        # the partial-sum records
        sk = _stream_key(dev)
        ws = self._loss_ws.get(sk)
        if ws is None or ws.numel() < n.value:
            ws = torch.zeros(max(n.value, 16), dtype=torch.uint8, device=dev)
            self._loss_ws[sk] = ws
        terms = torch.empty(3, dtype=torch.float32, device=dev) if terms_out is None else terms_out
        if terms.numel() != 3 or terms.dtype != torch.float32 or terms.device != dev:
            raise ValueError("forward_loss: terms_out must be fp32 [3] on %s" % dev)
        z = torch.empty_like(x) if want_outputs else None
        ld = torch.empty(B, dtype=torch.float32, device=dev) if want_outputs else None
        st = lib.cnf_forward_loss(ctypes.byref(self.desc), _ptr(blob), _ptr(x), _ptr(y),
                                  ctypes.c_int32(kind), ctypes.c_float(det), _ptr(z), _ptr(ld),
                                  _ptr(terms), ctypes.c_int64(B), _ptr(ws),
                                  ctypes.c_size_t(n.value), _stream(dev))
        _lib.check("cnf_forward_loss", st)
        stats["forward"] += 1
        return terms, z, ld

    def predict(self, x, log_priors, want_logdet=False):
        """Calibrated probabilities softmax(log(softmax(flow(x - mean x)) + 1e-7)
        - log_priors) (Calibrator.predict, calibrators.py:40-44, 330-353):
        one fused cnf_predict launch (k_sgpr, random_flip included; k_wide),
        or -- for shapes it does not cover (strict_nan, legacy options, wide
        shapes outside k_wide's table) -- cnf_forward followed by the same
        math as device torch ops."""
        x = self._check_input(x)
        B = x.shape[0]
        dev = x.device
        lp = torch.as_tensor(log_priors, dtype=torch.float32, device=dev).reshape(-1).contiguous()
        if lp.numel() != self.dim:
            raise ValueError("log_priors must have %d entries" % self.dim)
        blob = self.prepared(dev)
        probs = torch.empty_like(x)
        ld = torch.empty(B, dtype=torch.float32, device=dev) if want_logdet else None
        st = _lib.lib().cnf_predict(ctypes.byref(self.desc), _ptr(blob), _ptr(x), _ptr(lp),
                                    _ptr(probs), _ptr(ld), ctypes.c_int64(B), _stream(dev))
        if st == 0:
            stats["predict"] += 1
            return (probs, ld) if want_logdet else probs
        if st != -3:
            _lib.check("cnf_predict", st)
        xc = x - x.mean(dim=1, keepdim=True)
        z, ld, _ = self.run(xc, blob=blob)
        p = torch.softmax(z, dim=1)
        probs = torch.softmax(torch.log(p + 1e-7) - lp, dim=1)
        return (probs, ld) if want_logdet else probs

    # -------------------------------------------------------------- autograd
    def forward_autograd(self, x, want_all):
        """Forward with gradients w.r.t. x and every parameter (cnf_vjp): the
        cnf::flow operator (autograd kernel in C++) or the Python Function.
        Stacks whose reverse mode the ABI reports unsupported (legacy strict
        options) take the Python Function, whose backward falls back to torch
        autograd (vjp._torch_vjp); the C++ kernel would raise there."""
        ps = self.param_tensors()
        ops = _ops()
        if ops is not None and self.has_native_vjp():
            x = self._check_input(x)
            blob = self.prepared(x.device)
            stats["forward"] += 1
            stats["torch_ops"] += 1
            return ops.flow(x, blob, self.desc_ints, self._perms, want_all, ps)
        return _StackFn.apply(self, want_all, x, *ps)


    def has_native_vjp_inverse(self):
        """True when cnf_vjp_inverse serves this descriptor (strict_nan included)."""
        if self._vjp_inv_ok is None:
            n = ctypes.c_size_t()
            st = _lib.lib().cnf_vjp_inverse_workspace_bytes(ctypes.byref(self.desc),
                                                            ctypes.c_int64(1), ctypes.byref(n))
            self._vjp_inv_ok = st == 0
        return self._vjp_inv_ok

    def inverse_autograd(self, z, want_all):
        """Inverse with gradients w.r.t. z and every parameter
        (cnf_vjp_inverse, the layer-at-a-time reverse mode): the
        cnf::inverse_flow operator (autograd kernel in C++) or the Python
        Function."""
        ps = self.param_tensors()
        ops = _ops()
        if ops is not None and self.has_native_vjp_inverse():
            z = self._check_input(z)
            blob = self.prepared(z.device)
            stats["inverse"] += 1
            stats["torch_ops"] += 1
            return ops.inverse_flow(z, blob, self.desc_ints, self._perms, want_all, ps)
        return _InvStackFn.apply(self, want_all, z, *ps)


class _InvStackFn(torch.autograd.Function):
    """Flow.backward (the inverse transform) under autograd: cnf_inverse
    forward, cnf_vjp_inverse backward."""

    @staticmethod
    def forward(ctx, stack, want_all, z, *params):
        blob = stack.prepared(z.device)
        fin, ld, allt = stack.run(z, inverse=True, want_all=want_all, blob=blob)
        ctx.stack = stack
        ctx.want_all = want_all
        ctx.blob = blob
        ctx.key = stack.state_key()
        ctx.save_for_backward(z)
        return (allt if want_all else fin), ld

    @staticmethod
    def backward(ctx, g_out, g_ld):
        from .vjp import stack_vjp_inverse
        (z,) = ctx.saved_tensors
        stack = ctx.stack
        if stack.state_key() != ctx.key:
            raise RuntimeError(
                "one of the variables needed for gradient computation has been modified by an "
                "inplace operation: a coupling-layer weight or permutation changed between the "
                "native inverse and its backward")
        dz, grads = stack_vjp_inverse(stack, z, g_out, g_ld, all_grads=ctx.want_all,
                                      need_dz=ctx.needs_input_grad[2], blob=ctx.blob)
        out = [None, None, dz]
        for p, g in zip(stack.param_tensors(), grads):
            out.append(g.view_as(p))
        return tuple(out)


class _StackFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, stack, want_all, x, *params):
        blob = stack.prepared(x.device)
        fin, ld, allt = stack.run(x, inverse=False, want_all=want_all, blob=blob)
        ctx.stack = stack
        ctx.want_all = want_all
        ctx.blob = blob
        ctx.key = stack.state_key()
        ctx.save_for_backward(x)
        return (allt if want_all else fin), ld

    @staticmethod
    def backward(ctx, g_out, g_ld):
        from .vjp import stack_vjp
        (x,) = ctx.saved_tensors
        stack = ctx.stack
        if stack.state_key() != ctx.key:
            raise RuntimeError(
                "one of the variables needed for gradient computation has been modified by an "
                "inplace operation: a coupling-layer weight or permutation changed between the "
                "native forward and its backward")
        dx, grads = stack_vjp(stack, x, g_out, g_ld, all_grads=ctx.want_all,
                              need_dx=ctx.needs_input_grad[2], blob=ctx.blob)
        ps = stack.param_tensors()
        out = [None, None, dx]
        for p, g in zip(ps, grads):
            out.append(g.view_as(p))
        return tuple(out)
