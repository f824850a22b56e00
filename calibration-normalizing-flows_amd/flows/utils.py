"""Conditioner MLP and temperature scaler -- drop-in for the reference's
flows/utils.py (same constructor arguments, same parameter names, same RNG
draws at init, so `torch.manual_seed(s)` yields the reference's weights).

The MLP's forward is executed natively (fused into the coupling kernel) when it
sits inside an NvpCouplingLayer on a ROCm device; called on its own it is an
ordinary module.
"""
import torch
import torch.nn.functional as F
from torch import nn


class MLP(nn.Module):
    """units = [dim] + hidden_size + [dim]; Linear weights and biases scaled by
    `wscale` at init; activation between layers, none after the last
    (reference flows/utils.py:6-31)."""

    def __init__(self, dim, hidden_size=[], activation=F.relu, wscale=1.):
        super().__init__()
        self.activation = activation
        widths = [dim, *hidden_size, dim]
        linears = []
        for n_in, n_out in zip(widths[:-1], widths[1:]):
            lin = nn.Linear(n_in, n_out)
            with torch.no_grad():
                lin.weight = nn.Parameter(lin.weight.detach() * wscale)
                lin.bias = nn.Parameter(lin.bias.detach() * wscale)
            linears.append(lin)
        self.layers = nn.ModuleList(linears)

    def forward(self, x):
        *hidden, last = self.layers
        for lin in hidden:
            x = self.activation(lin(x))
        return last(x)


class TempScaler(nn.Module):
    """z = x / |T| with inverse x = z * |T| (reference flows/utils.py:34-48)."""

    def __init__(self):
        super().__init__()
        self.T = nn.Parameter(torch.ones(1))

    def forward(self, x):
        return x / self.T.abs()

    def backward(self, z):
        return z * self.T.abs()
