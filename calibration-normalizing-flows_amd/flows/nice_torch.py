"""`from flows.nice_torch import NiceFlow` (notebooks/simulated-predictions-flows.ipynb)."""
from ._factory import NiceFlow  # noqa: F401
