"""`from flows.realNVP_torch import RealNvpFlow` (notebooks/simulated-predictions-flows.ipynb)."""
from ._factory import RealNvpFlow  # noqa: F401
