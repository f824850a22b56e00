"""`from flows.nice_torch import NiceFlow` -- the additive-coupling factory the
reference's notebooks import (notebooks/simulated-predictions-flows.ipynb,
notebooks/benchmark-nice-calibration.ipynb) but the reference repo does not
ship.

NICE is the maintained coupling layer with scale=False (flows/flows.py:76-79:
s == 0, so the log-det is identically 0): each layer adds t(x_b) to the
transformed half, the data flip between layers.  The call returns
(z_final, log_det) for the calibrator (calibrators.py:251, 287); unknown
keyword arguments are ignored.  Defaults (layers=4, hidden_size=[dim]) follow
code-old/realNVP.py:46-52 and are otherwise unpinned.

The TensorFlow-era NICE flows of code-old/nice.py are the `legacy` option
(parity unpinned, TensorFlow is absent):
  legacy=1   NiceFlow     split coupling, x2 += f(x1) / x1 += f(x2) alternating;
  legacy=2   NiceFlow_v2  x1 += f(x2) then a full reversal per layer;
  legacy=3   NiceFlow_v3  alternating masks, no data permutation (native);
each returns flows.legacy.LegacyNiceFlow.
"""
from ._factory import CouplingFlow


class NiceFlow(CouplingFlow):
    """NICE additive coupling stack (t-net only, log-det = 0)."""

    scale = False

    def __new__(cls, dim=None, *args, legacy=None, **kwargs):
        if legacy is None:
            return super().__new__(cls)
        if legacy not in (1, 2, 3):
            raise ValueError("legacy must be None, 1, 2 or 3")
        from .legacy import LegacyNiceFlow
        layers = args[0] if args else kwargs.pop("layers", 4)
        hidden = args[1] if len(args) > 1 else kwargs.pop("hidden_size", None)
        act = kwargs.pop("activation", "relu")
        return LegacyNiceFlow(dim, layers=layers, hidden_size=hidden, activation=act,
                              version=legacy)

    def __init__(self, dim, *args, legacy=None, **kwargs):
        super().__init__(dim, *args, **kwargs)
