"""Op-for-op torch CPU port of the reference forward path -- TEST/BENCH INFRASTRUCTURE.

The CPU baseline `bench.py` times on the GPU box's host cores (the reference
itself never travels there).  It issues the same ATen op sequence as the
reference (mul, rsub, addmm, relu, exp, add, sum, flip), so its cost on a given
set of cores tracks the reference's own flows/flows.py (ratio measured in this
container: DESIGN.md).  Pinned against the golden fixtures in
tests/test_oracle.py.  Never imported by the product.

Reference anchors: flows/flows.py:17-25 (Flow.forward), :101-112
(NvpCouplingLayer.forward), :114-126 (backward = inverse), flows/utils.py:26-31.
"""
import torch


def layers_from_state(state, L, n_linear, scale=True, shift=True, prefix="layers."):
    """[(mask, s_net, t_net, perm)] with torch CPU tensors; nets are lists of (W, b)."""
    out = []
    for l in range(L):
        p = "%s%d." % (prefix, l)
        nets = []
        for net, on in (("s", scale), ("t", shift)):
            nets.append([(torch.as_tensor(state[p + "%s.layers.%d.weight" % (net, i)]),
                          torch.as_tensor(state[p + "%s.layers.%d.bias" % (net, i)]))
                         for i in range(n_linear)] if on else None)
        mask = torch.as_tensor(state[p + "mask"])
        perm = state.get(p + "perm")
        perm = None if perm is None else torch.as_tensor(perm).reshape(-1)
        out.append((mask, nets[0], nets[1], perm))
    return out


def _mlp(net, h):
    for i, (W, b) in enumerate(net):
        h = torch.addmm(b, h, W.t())
        if i < len(net) - 1:
            h = torch.relu(h)
    return h


@torch.no_grad()
def flow_forward(layers, x):
    cum = 0.0
    zs = []
    for mask, s_net, t_net, perm in layers:
        x_b = mask * x
        b_1 = 1 - mask
        s = _mlp(s_net, x_b) if s_net is not None else x_b.new_zeros(x_b.size())
        t = _mlp(t_net, x_b) if t_net is not None else x_b.new_zeros(x_b.size())
        z = x_b + b_1 * (x * torch.exp(s) + t)
        ld = torch.sum(b_1 * s, dim=1).squeeze()
        if perm is not None:
            z = z[:, perm]
        x = z.flip((1,))
        zs.append(x)
        cum = cum + ld
    return zs, cum
