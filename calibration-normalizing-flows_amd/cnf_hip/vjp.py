"""Reverse mode of the fused coupling stack (cnf_vjp / cnf_loss_vjp, include/cnf.h).

`stack_vjp` is what torch autograd calls for Flow.forward on a ROCm device;
`loss_and_grads` is the fused calibrator step (forward + loss + reverse mode in
one launch plus a fixed-order reduction), used by the native
TorchFlowCalibrator and by the data-parallel trainer.
"""
import ctypes
import warnings

import torch

from . import _lib
from .engine import _ptr, _stream, _stream_key, stats

_ws_cache = {}


def _workspace(stack, B, device):
    """Per-block gradient partials: one buffer per (device, stream), so launches
    on different streams never share it; grown on demand."""
    lib = _lib.lib()
    n = ctypes.c_size_t()
    _lib.check("cnf_vjp_workspace_bytes",
               lib.cnf_vjp_workspace_bytes(ctypes.byref(stack.desc), ctypes.c_int64(B),
                                           ctypes.byref(n)))
    key = _stream_key(device)
    buf = _ws_cache.get(key)
    if buf is None or buf.numel() < n.value:
        buf = torch.empty(max(n.value, 16), dtype=torch.uint8, device=device)
        _ws_cache[key] = buf
    return buf, n.value


def _split(stack, flat):
    out = []
    off = 0
    for p in stack.param_tensors():
        out.append(flat[off:off + p.numel()].view_as(p))
        off += p.numel()
    return out


def stack_vjp(stack, x, g_out, g_ld, all_grads, need_dx, blob=None):
    """(dx or None, [grad per parameter]) for the upstream gradients of
    (z_all if all_grads else z_final, log-det); `blob`: the prepared weights
    the forward ran with."""
    x = x.contiguous()
    B = x.shape[0]
    dev = x.device
    try:
        if blob is None:
            blob = stack.prepared(dev)
        ws, nws = _workspace(stack, B, dev)
    except _lib.UnsupportedShape:
        return _torch_vjp(stack, x, g_out, g_ld, all_grads, need_dx)
    P = stack.param_count()
    grads = torch.empty(P, dtype=torch.float32, device=dev)
    dx = torch.empty_like(x) if need_dx else None
    gz = gza = None
    if g_out is not None:
        g_out = g_out.contiguous().float()
        if all_grads:
            gza = g_out
        else:
            gz = g_out
    gld = g_ld.contiguous().float().reshape(-1) if g_ld is not None else None
    if gld is not None and gld.numel() == 1 and B != 1:
        gld = gld.expand(B).contiguous()
    lib = _lib.lib()
    st = lib.cnf_vjp(ctypes.byref(stack.desc), _ptr(blob), _ptr(x), _ptr(gz), _ptr(gza),
                     _ptr(gld), _ptr(grads), _ptr(dx), ctypes.c_int64(B), _ptr(ws),
                     ctypes.c_size_t(nws), _stream(dev))
    if st == -3:
        return _torch_vjp(stack, x, g_out, g_ld, all_grads, need_dx)
    _lib.check("cnf_vjp", st)
    stats["vjp"] += 1
    return dx, _split(stack, grads)


def stack_vjp_inverse(stack, z, g_out, g_ld, all_grads, need_dz, blob=None):
    """(dz or None, [grad per parameter]) of the INVERSE transform for the
    upstream gradients of (x_all if all_grads else x_final, log-det)
    (cnf_vjp_inverse, include/cnf.h)."""
    z = z.contiguous()
    B = z.shape[0]
    dev = z.device
    if blob is None:
        blob = stack.prepared(dev)
    lib = _lib.lib()
    n = ctypes.c_size_t()
    _lib.check("cnf_vjp_inverse_workspace_bytes",
               lib.cnf_vjp_inverse_workspace_bytes(ctypes.byref(stack.desc), ctypes.c_int64(B),
                                                   ctypes.byref(n)))
    key = ("inv",) + _stream_key(dev)
    ws = _ws_cache.get(key)
    if ws is None or ws.numel() < n.value:
        ws = torch.empty(max(n.value, 16), dtype=torch.uint8, device=dev)
        _ws_cache[key] = ws
    grads = torch.empty(stack.param_count(), dtype=torch.float32, device=dev)
    dz = torch.empty_like(z) if need_dz else None
    gx = gxa = None
    if g_out is not None:
        g_out = g_out.contiguous().float()
        if all_grads:
            gxa = g_out
        else:
            gx = g_out
    gld = g_ld.contiguous().float().reshape(-1) if g_ld is not None else None
    if gld is not None and gld.numel() == 1 and B != 1:
        gld = gld.expand(B).contiguous()
    st = lib.cnf_vjp_inverse(ctypes.byref(stack.desc), _ptr(blob), _ptr(z), _ptr(gx), _ptr(gxa),
                             _ptr(gld), _ptr(grads), _ptr(dz), ctypes.c_int64(B), _ptr(ws),
                             ctypes.c_size_t(n.value), _stream(dev))
    _lib.check("cnf_vjp_inverse", st)
    stats["vjp"] += 1
    return dz, _split(stack, grads)


def loss_and_grads(stack, x, y, kind=_lib.LOSS_CAL, det=1.0, grad_scale=1.0, need_dx=False,
                   grads_out=None, terms_out=None):
    """Fused forward + loss + reverse mode.  Returns (terms[3], flat grads, dx)
    where terms = (sum of per-row loss, sum of ce, sum of log-det) over THIS
    batch and grads = grad_scale * d(sum of per-row loss)/d(params).
    grads_out / terms_out: caller-provided contiguous fp32 destinations (e.g.
    the two parts of one all-reduce buffer)."""
    x = x.contiguous()
    y = y.contiguous().to(torch.int64)
    B = x.shape[0]
    dev = x.device
    blob = stack.prepared(dev)
    ws, nws = _workspace(stack, B, dev)
    grads = torch.empty(stack.param_count(), dtype=torch.float32, device=dev) \
        if grads_out is None else grads_out
    terms = torch.empty(3, dtype=torch.float32, device=dev) if terms_out is None else terms_out
    for t, n in ((grads, stack.param_count()), (terms, 3)):
        if t.numel() != n or not t.is_contiguous() or t.dtype != torch.float32 or t.device != dev:
            raise ValueError("loss_and_grads: output buffer must be contiguous fp32 [%d] on %s"
                             % (n, dev))
    dx = torch.empty_like(x) if need_dx else None
    lib = _lib.lib()
    st = lib.cnf_loss_vjp(ctypes.byref(stack.desc), _ptr(blob), _ptr(x), _ptr(y),
                          ctypes.c_int32(kind), ctypes.c_float(det), ctypes.c_float(grad_scale),
                          _ptr(terms), _ptr(grads), _ptr(dx), ctypes.c_int64(B), _ptr(ws),
                          ctypes.c_size_t(nws), _stream(dev))
    _lib.check("cnf_loss_vjp", st)
    stats["loss_vjp"] += 1
    return terms, grads, dx


_warned = set()


def _torch_vjp(stack, x, g_out, g_ld, all_grads, need_dx):
    """Reverse modes the ABI reports unsupported (CNF_ERR_UNSUPPORTED: shapes
    past the layer-at-a-time kernels' LDS envelope): autograd through the
    layers' own torch ops, on the same device.  strict_nan stacks have native
    reverse modes for the forward and the inverse."""
    key = (stack.dim, tuple(stack.hidden), stack.strict_nan)
    if stack.options & (_lib.OPT_ALT_MASK | _lib.OPT_S_TANH):
        # _torch_forward restates the maintained (ReLU, data-flip) layer only:
        # a legacy stack must not differentiate through it
        raise _lib.UnsupportedShape("cnf_vjp", -3, _lib.lib())
    from flows.flows import STRICT_NATIVE
    if STRICT_NATIVE:
        raise RuntimeError("native coupling path unavailable: no native VJP for %s" % (key,))
    if key not in _warned:
        _warned.add(key)
        warnings.warn("cnf: no native VJP for %s; using torch autograd" % (key,), RuntimeWarning)
    ps = stack.param_tensors()
    with torch.enable_grad():
        xx = x.detach().requires_grad_(need_dx)
        leaves = [p.detach().requires_grad_(True) for p in ps]
        # re-bind the detached leaves into the layers' math
        zs, ld = _torch_forward(stack, xx, leaves)
        outs, grads_in = [], []
        if g_out is not None:
            outs.append(torch.stack(zs) if all_grads else zs[-1])
            grads_in.append(g_out)
        if g_ld is not None:
            outs.append(ld)
            grads_in.append(g_ld.reshape(ld.shape))
        inputs = leaves + ([xx] if need_dx else [])
        if not outs:
            return (torch.zeros_like(x) if need_dx else None), [torch.zeros_like(p) for p in ps]
        res = torch.autograd.grad(outs, inputs, grads_in, allow_unused=True)
    res = [torch.zeros_like(t) if r is None else r for r, t in zip(res, inputs)]
    dx = res[-1] if need_dx else None
    return dx, list(res[:len(leaves)])


def _torch_forward(stack, x, leaves):
    it = iter(leaves)
    ld = torch.zeros(x.shape[0], device=x.device)
    zs = []
    n_lin = len(stack.hidden) + 1
    for ly in stack.layers:
        nets = []
        for on in (stack.scale, stack.shift):
            nets.append([(next(it), next(it)) for _ in range(n_lin)] if on else None)
        mask = ly.mask
        keep = mask * x
        free = 1 - mask

        def run(net, h):
            if net is None:
                return torch.zeros_like(h)
            for i, (W, b) in enumerate(net):
                h = torch.nn.functional.linear(h, W, b)
                if i < len(net) - 1:
                    h = torch.relu(h)
            return h
        s, t = run(nets[0], keep), run(nets[1], keep)
        z = keep + free * (x * torch.exp(s) + t)
        ld = ld + torch.sum(free * s, dim=1)
        if ly.random_flip:
            z = z[:, ly.perm.reshape(-1)]
        x = z.flip((1,))
        zs.append(x)
    return zs, ld
