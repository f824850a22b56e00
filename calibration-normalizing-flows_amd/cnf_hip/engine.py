"""Host side of the native coupling-flow path: descriptor, prepared-weight
cache, launches on torch's current HIP stream, and the autograd binding.

`CouplingStack` binds a run of identically-shaped NvpCouplingLayers to ONE
fused launch (cnf_forward / cnf_inverse / cnf_vjp in include/cnf.h).  All
buffers are torch allocations on the input's device; the stream is
`torch.cuda.current_stream()`, so launches order with surrounding torch work
and can be captured into a CUDA(HIP) graph.
"""
import ctypes

import torch

from . import _lib

# counts of native launches (tests assert the HIP path really ran)
stats = {"forward": 0, "inverse": 0, "prepare": 0, "vjp": 0, "loss_vjp": 0}


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class CouplingStack:
    """A fused stack of NvpCouplingLayers (flows/flows.py:68-126) sharing
    dim / hidden_size / scale / shift.  Layers keep owning their parameters;
    the stack only reads them (state_dict order) through cnf_prepare."""

    def __init__(self, layers, strict_nan=False):
        layers = list(layers)
        l0 = layers[0]
        self.layers = layers
        self.dim = l0.dim
        self.hidden = list(l0.hidden_size)
        self.scale = bool(l0.scale)
        self.shift = bool(l0.shift)
        self.strict_nan = bool(strict_nan)
        self.L = len(layers)
        self._perms = None
        if any(ly.random_flip for ly in layers):
            p = torch.full((self.L, self.dim), -1, dtype=torch.int64)
            for i, ly in enumerate(layers):
                if ly.random_flip:
                    p[i] = ly.perm.detach().reshape(-1).cpu()
            self._perms = p.contiguous()
        self.desc = _lib.make_desc(self.dim, self.L, self.hidden, self.scale, self.shift,
                                   self.strict_nan, self._perms)
        self._cache = {}
        self._loss_ws = {}

    @staticmethod
    def compatible(layers):
        l0 = layers[0]
        return all(ly.dim == l0.dim and list(ly.hidden_size) == list(l0.hidden_size)
                   and ly.scale == l0.scale and ly.shift == l0.shift for ly in layers)

    def kernel_name(self):
        return _lib.lib().cnf_kernel_name(ctypes.byref(self.desc)).decode()

    def param_tensors(self):
        """ABI order (include/cnf.h cnf_param_tensor_count)."""
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

    def prepared(self, device):
        """Device blob for this stack, rebuilt only when a parameter changed
        (data pointer or in-place version counter)."""
        ps = self.param_tensors()
        for p in ps:
            if p.device != device or p.dtype != torch.float32:
                raise TypeError("native coupling path needs fp32 parameters on %s" % device)
        key = tuple((p.data_ptr(), p._version) for p in ps)
        ent = self._cache.get(device)
        if ent is not None and ent[0] == key:
            return ent[1]
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

    def run(self, x, inverse=False, want_all=False, want_final=True):
        """Returns (final [B,D] or None, logdet [B], all [L,B,D] or None)."""
        x = self._check_input(x)
        B = x.shape[0]
        dev = x.device
        blob = self.prepared(dev)
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

    def forward_loss(self, x, y, kind=_lib.LOSS_CAL, det=1.0, want_outputs=False):
        """Fused forward + log-det + loss terms (cnf_forward_loss): returns
        (terms[3] = sums over the rows of (loss, ce, log-det), z or None, ld or None)."""
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
        ws = self._loss_ws.get(dev)
        if ws is None or ws.numel() < n.value:
            ws = torch.zeros(max(n.value, 16), dtype=torch.uint8, device=dev)  # ticket = 0
            self._loss_ws[dev] = ws
        terms = torch.empty(3, dtype=torch.float32, device=dev)
        z = torch.empty_like(x) if want_outputs else None
        ld = torch.empty(B, dtype=torch.float32, device=dev) if want_outputs else None
        st = lib.cnf_forward_loss(ctypes.byref(self.desc), _ptr(blob), _ptr(x), _ptr(y),
                                  ctypes.c_int32(kind), ctypes.c_float(det), _ptr(z), _ptr(ld),
                                  _ptr(terms), ctypes.c_int64(B), _ptr(ws),
                                  ctypes.c_size_t(n.value), _stream(dev))
        _lib.check("cnf_forward_loss", st)
        stats["forward"] += 1
        return terms, z, ld

    # -------------------------------------------------------------- autograd
    def forward_autograd(self, x, want_all):
        """Forward with gradients w.r.t. x and every parameter (cnf_vjp)."""
        ps = self.param_tensors()
        return _StackFn.apply(self, want_all, x, *ps)


class _StackFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, stack, want_all, x, *params):
        fin, ld, allt = stack.run(x, inverse=False, want_all=want_all)
        ctx.stack = stack
        ctx.want_all = want_all
        ctx.save_for_backward(x)
        return (allt if want_all else fin), ld

    @staticmethod
    def backward(ctx, g_out, g_ld):
        from .vjp import stack_vjp
        (x,) = ctx.saved_tensors
        stack = ctx.stack
        dx, grads = stack_vjp(stack, x, g_out, g_ld, all_grads=ctx.want_all,
                              need_dx=ctx.needs_input_grad[2])
        ps = stack.param_tensors()
        out = [None, None, dx]
        for p, g in zip(ps, grads):
            out.append(g.view_as(p))
        return tuple(out)
