"""CPU oracle for the coupling-flow hot path -- TEST INFRASTRUCTURE, NOT PRODUCT.

A plain-numpy restatement of the reference's RealNVP/NICE path, op for op, dense
and un-fused exactly as the reference computes it (including the full-width
MLPs that see the masked input, the `0 * inf = NaN` behaviour at masked
positions and the per-layer flip).  Only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg may import this module, and only as the checker
or the timed CPU baseline -- never as the thing measured on the GPU.

Pinned: every function here is checked against the golden vectors in
`tests/golden/*.npz`, which `tests/golden/gen_golden.py` produced by importing
the reference's own `flows/flows.py` (tests/test_oracle.py).

Reference anchors (paths relative to the reference repo root):
  MLP.forward                     flows/utils.py:26-31
  NvpCouplingLayer.__init__ mask  flows/flows.py:81-86
  NvpCouplingLayer.forward        flows/flows.py:101-112
  NvpCouplingLayer.backward       flows/flows.py:114-126  (the INVERSE transform)
  Flow.forward / Flow.backward    flows/flows.py:17-25 / 27-37
  calibrator loss                 calibrators.py:287-291
  CE - det*mean(ld) loss          run_experiment3D.py:102-107
"""
import numpy as np

EPS_CAL = 1e-7  # calibrators.py:289


# ----------------------------------------------------------------------------
# parameter containers (state_dict keys of the reference modules)
# ----------------------------------------------------------------------------
class OracleLayer:
    """One NvpCouplingLayer's parameters as numpy arrays."""

    def __init__(self, dim, s_net, t_net, perm=None):
        self.dim = dim
        self.s_net = s_net      # list of (W[out,in], b[out]) or None (scale=False)
        self.t_net = t_net      # same, None when shift=False
        self.perm = perm        # int64 [dim] or None (random_flip=False)
        mask = np.zeros((1, dim))
        mask[:, dim // 2:] = 1  # flows/flows.py:81-82
        self.mask = mask
        if perm is not None:
            rev = np.zeros(dim, dtype=np.int64)
            rev[perm] = np.arange(dim)  # flows/flows.py:94-95
            self.rev_perm = rev


def layers_from_state(state, L, dim, n_linear, scale=True, shift=True, prefix="layers."):
    """Build OracleLayers from a reference-style state dict {key: ndarray}."""
    layers = []
    for l in range(L):
        p = "%s%d." % (prefix, l)
        nets = []
        for net, on in (("s", scale), ("t", shift)):
            if not on:
                nets.append(None)
                continue
            nets.append([(np.asarray(state[p + "%s.layers.%d.weight" % (net, i)]),
                          np.asarray(state[p + "%s.layers.%d.bias" % (net, i)]))
                         for i in range(n_linear)])
        perm = state.get(p + "perm")
        if perm is not None:
            perm = np.asarray(perm).reshape(-1).astype(np.int64)
        layers.append(OracleLayer(dim, nets[0], nets[1], perm))
    return layers


def cast_layers(layers, dtype):
    out = []
    for ly in layers:
        c = lambda net: None if net is None else [(W.astype(dtype), b.astype(dtype)) for W, b in net]
        out.append(OracleLayer(ly.dim, c(ly.s_net), c(ly.t_net), ly.perm))
    return out


# ----------------------------------------------------------------------------
# forward / inverse
# ----------------------------------------------------------------------------
def _relu(a):
    # torch relu propagates NaN (clamp_min); np.maximum does too.
    return np.maximum(a, 0)


def mlp_forward(net, x, keep=False):
    """flows/utils.py:26-31: relu(Linear) for hidden layers, plain Linear last."""
    acts = [x]
    h = x
    for i, (W, b) in enumerate(net):
        a = h @ W.T + b
        h = _relu(a) if i < len(net) - 1 else a
        acts.append(h)
    return (h, acts) if keep else h


def _net(net, xb, keep=False):
    if net is None:  # flows/flows.py:76-79: lambda x: x.new_zeros(x.size())
        z = np.zeros_like(xb)
        return (z, None) if keep else z
    return mlp_forward(net, xb, keep)


def coupling_forward(layer, x):
    """flows/flows.py:101-112.  Returns (z_flipped, log_det[B])."""
    dt = x.dtype
    m = layer.mask.astype(dt)
    x_b = m * x
    b_1 = 1 - m
    with np.errstate(over="ignore", invalid="ignore"):
        s, t = _net(layer.s_net, x_b), _net(layer.t_net, x_b)
        z = x_b + b_1 * (x * np.exp(s) + t)
        log_det = np.sum(b_1 * s, axis=1)
    if layer.perm is not None:
        z = z[:, layer.perm]
    return z[:, ::-1].copy(), log_det


def coupling_inverse(layer, z):
    """flows/flows.py:114-126 (`backward` = inverse transform)."""
    dt = z.dtype
    z = z[:, ::-1]
    if layer.perm is not None:
        z = z[:, layer.rev_perm]
    m = layer.mask.astype(dt)
    x_b = m * z
    b_1 = 1 - m
    with np.errstate(over="ignore", invalid="ignore"):
        s, t = _net(layer.s_net, x_b), _net(layer.t_net, x_b)
        x = x_b + b_1 * (z - t) * np.exp(-s)
        log_det = np.sum(b_1 * (-s), axis=1)
    return x, log_det


def flow_forward(layers, x):
    """flows/flows.py:17-25: returns (zs list of every layer output, cum log-det)."""
    cum = np.zeros(x.shape[0], dtype=x.dtype)
    zs = []
    for ly in layers:
        x, ld = coupling_forward(ly, x)
        zs.append(x)
        cum = cum + ld
    return zs, cum


def flow_inverse(layers, z):
    """flows/flows.py:27-37: layers in reverse order; xs[-1] is the input estimate."""
    cum = np.zeros(z.shape[0], dtype=z.dtype)
    xs = []
    for ly in layers[::-1]:
        z, ld = coupling_inverse(ly, z)
        xs.append(z)
        cum = cum + ld
    return xs, cum


# ----------------------------------------------------------------------------
# losses and their gradients (hand-written reverse mode of the above)
# ----------------------------------------------------------------------------
def _log_softmax(z):
    mx = np.max(z, axis=1, keepdims=True)
    e = np.exp(z - mx)
    return z - mx - np.log(np.sum(e, axis=1, keepdims=True))


def loss_and_grads(layers, x, y, kind="cal", det=1.0):
    """Loss and parameter gradients.

    kind="cal": -mean(log(softmax(z_L)[y] + 1e-7) + ld)          calibrators.py:287-291
    kind="ce" : CE(z_L, y) - det * mean(ld)                       run_experiment3D.py:102-107
    Returns (loss, grads) with grads[l] = {"s": [(dW, db)...], "t": [...]}.
    """
    B, D = x.shape
    dt = x.dtype
    tape = []
    h = x
    cum = np.zeros(B, dtype=dt)
    for ly in layers:
        m = ly.mask.astype(dt)
        b_1 = 1 - m
        x_b = m * h
        s, s_acts = _net(ly.s_net, x_b, keep=True)
        t, t_acts = _net(ly.t_net, x_b, keep=True)
        e = np.exp(s)
        z = x_b + b_1 * (h * e + t)
        cum = cum + np.sum(b_1 * s, axis=1)
        tape.append((h, m, b_1, s_acts, t_acts, e))
        if ly.perm is not None:
            z = z[:, ly.perm]
        h = z[:, ::-1].copy()
    zL = h
    lsm = _log_softmax(zL)
    p = np.exp(lsm)
    onehot = np.zeros_like(zL)
    onehot[np.arange(B), y] = 1
    if kind == "cal":
        py = p[np.arange(B), y]
        ce = np.log(py + EPS_CAL)
        loss = -np.mean(ce + cum)
        # d(-mean(log(py+eps)))/dz = -(1/B) * py/(py+eps) * (onehot - p)
        g = -(py / (py + EPS_CAL))[:, None] * (onehot - p) / B
        gld = np.full(B, -1.0 / B, dtype=dt)
    elif kind == "ce":
        loss = -np.mean(lsm[np.arange(B), y]) - det * np.mean(cum)
        g = (p - onehot) / B
        gld = np.full(B, -det / B, dtype=dt)
    else:
        raise ValueError(kind)
    grads = [None] * len(layers)
    for l in range(len(layers) - 1, -1, -1):
        ly = layers[l]
        hin, m, b_1, s_acts, t_acts, e = tape[l]
        gz = g[:, ::-1]
        if ly.perm is not None:
            tmp = np.zeros_like(gz)
            tmp[:, ly.perm] = gz
            gz = tmp
        # z = m*h + b_1*(h*e + t);  ld += sum(b_1*s)
        gh = m * gz + b_1 * gz * e
        gs = b_1 * gz * hin * e + b_1 * gld[:, None]
        gt = b_1 * gz
        gl = {"s": None, "t": None}
        gxb = np.zeros_like(hin)
        for key, net, acts, gout in (("s", ly.s_net, s_acts, gs), ("t", ly.t_net, t_acts, gt)):
            if net is None:
                continue
            gw = []
            ga = gout
            for i in range(len(net) - 1, -1, -1):
                W, b = net[i]
                a_in = acts[i]
                gw.append((ga.T @ a_in, ga.sum(axis=0)))
                gin = ga @ W
                if i > 0:
                    gin = gin * (acts[i] > 0)
                ga = gin
            gl[key] = gw[::-1]
            gxb = gxb + ga
        gh = gh + m * gxb
        grads[l] = gl
        g = gh
    return loss, grads
