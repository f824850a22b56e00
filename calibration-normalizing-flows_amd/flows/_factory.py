"""Flow factories for TorchFlowCalibrator (calibrators.py:239-353).

The calibrator builds its flow as `Flow(n_classes, **kwargs)` (calibrators.py:251)
with kwargs that also carry `dev`, `epochs`, `batch_size`, and calls it as
`pred, log_det = self.flow(x)` (calibrators.py:287, 304, 339): the FINAL output,
not the reference Flow's list.  The reference notebooks import such factories
from `flows.realNVP_torch` / `flows.nice_torch`, modules absent from the
reference repo; their defaults here follow code-old/realNVP.py:46-52
(layers=4, hidden_size=[dim]) and are otherwise unpinned.
"""
from .flows import Flow, NvpCouplingLayer


class CouplingFlow(Flow):
    """A Flow of NvpCouplingLayers whose call returns (z_final, log_det)."""

    scale = True

    def __init__(self, dim, layers=4, hidden_size=None, random_flip=False, strict_nan=None,
                 **kwargs):
        hidden = [dim] if hidden_size is None else list(hidden_size)
        super().__init__([NvpCouplingLayer(dim, hidden, scale=self.scale, shift=True,
                                           random_flip=random_flip) for _ in range(layers)],
                         strict_nan=strict_nan)
        self.dim = dim

    def forward(self, x):
        return self.transform(x)

    def backward(self, z):
        return self.inverse_transform(z)

    def forward_all(self, x):
        """The reference Flow.forward: (zs list, cum_log_det)."""
        return Flow.forward(self, x)
