"""Build the drop-in Flow for a golden case and load the fixture's weights."""
import numpy as np
import torch

from flows.flows import Flow, NvpCouplingLayer


def build_flow(meta, state, device="cpu", strict_nan=None):
    torch.manual_seed(0)
    np.random.seed(meta["seed"])  # random_flip perms are overwritten from state below
    flow = Flow([NvpCouplingLayer(meta["D"], list(meta["hidden"]), scale=meta["scale"],
                                  shift=meta["shift"], random_flip=meta["random_flip"])
                 for _ in range(meta["L"])], strict_nan=strict_nan)
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in state.items()}
    missing, unexpected = flow.load_state_dict(sd, strict=True), None
    return flow.to(device)
