"""`from flows.nice_torch import NiceFlow` -- the additive-coupling factory the
reference's notebooks import (notebooks/simulated-predictions-flows.ipynb,
notebooks/benchmark-nice-calibration.ipynb) but the reference repo does not
ship.

NICE is the maintained coupling layer with scale=False (flows/flows.py:76-79:
s == 0, so the log-det is identically 0): each layer adds t(x_b) to the
transformed half, the data flip between layers.  The call returns
(z_final, log_det) for the calibrator (calibrators.py:251, 287); unknown
keyword arguments are ignored.  Defaults (layers=4, hidden_size=[dim]) follow
code-old/realNVP.py:46-52 and are otherwise unpinned; the reference's NICE
split-coupling v1 (code-old/nice.py:140-155) is not built.
"""
from ._factory import CouplingFlow


class NiceFlow(CouplingFlow):
    """NICE additive coupling stack (t-net only, log-det = 0)."""

    scale = False
