"""`from flows.realNVP_torch import RealNvpFlow` -- the factory the reference's
notebooks import (notebooks/simulated-predictions-flows.ipynb) but the
reference repo does not ship.

`RealNvpFlow(dim, layers=4, hidden_size=None, **kw)` builds the maintained
coupling flow (flows/flows.py NvpCouplingLayer stack, data flipped between
layers) and returns (z_final, log_det) from its call, the calibrator's factory
protocol (calibrators.py:251, 287).  Defaults follow code-old/realNVP.py:46-52
(layers=4, hidden_size=[dim]); they are otherwise unpinned.

The TensorFlow-era semantics of code-old/realNVP.py are options:
  mask_mode='alternate_mask'   alternate the mask per layer, never flip data;
  s_activation='tanh'          tanh hidden layers in the s-net;
either returns flows.legacy.LegacyRealNvpFlow (parity unpinned: TensorFlow is
absent).  Unknown keyword arguments (the calibrator passes dev / epochs /
batch_size) are ignored.
"""
from ._factory import CouplingFlow


class RealNvpFlow(CouplingFlow):
    """RealNVP affine coupling stack (s-net and t-net)."""

    scale = True

    def __new__(cls, dim=None, *args, mask_mode="flip_data", s_activation=None, **kwargs):
        if mask_mode not in ("flip_data", "alternate_mask"):
            raise ValueError("mask_mode must be 'flip_data' or 'alternate_mask'")
        if s_activation not in (None, "none", "relu", "tanh"):
            raise ValueError("s_activation must be None, 'relu' or 'tanh'")
        if mask_mode == "alternate_mask" or s_activation == "tanh":
            from .legacy import LegacyRealNvpFlow
            layers = args[0] if args else kwargs.pop("layers", 4)
            hidden = args[1] if len(args) > 1 else kwargs.pop("hidden_size", None)
            act = kwargs.pop("activation", "relu")
            if mask_mode != "alternate_mask":
                raise ValueError("s_activation='tanh' is the legacy flow: "
                                 "use it with mask_mode='alternate_mask'")
            # code-old/realNVP.py:58-64: the s-net is always tanh there
            s_act = "tanh" if s_activation in (None, "tanh") else s_activation
            if s_act == "none":
                raise ValueError("s_activation='none' has no hidden activation to apply; "
                                 "use 'relu' or 'tanh'")
            return LegacyRealNvpFlow(dim, layers=layers, hidden_size=hidden, activation=act,
                                     s_activation=s_act)
        return super().__new__(cls)

    def __init__(self, dim, *args, mask_mode="flip_data", s_activation=None, **kwargs):
        super().__init__(dim, *args, **kwargs)
