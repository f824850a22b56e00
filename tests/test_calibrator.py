"""TorchFlowCalibrator drop-in (calibrators.py:239-353) against the reference's
own calibrator run (golden g7: history, trained weights, predictions)."""
import json
import os

import numpy as np
import pytest
import torch

from _golden import GOLDEN
from flows.realNVP_torch import RealNvpFlow
from flows.nice_torch import NiceFlow
import calibrators as C


def _g7(name="g7_calibrator_d3"):
    f = np.load(os.path.join(GOLDEN, name + ".npz"))
    return json.loads(str(f["meta"])), f


G7B = "g7b_calibrator_d3_mb128"  # batch_size=128: the DataLoader order is pinned too


def _fit(dev, name="g7_calibrator_d3"):
    meta, f = _g7(name)
    torch.manual_seed(meta["seed"])
    np.random.seed(meta["seed"])
    kw = {"batch_size": meta["batch_size"]} if "batch_size" in meta else {}
    return C.TorchFlowCalibrator(RealNvpFlow, f["x"].astype(np.float64), f["y"], layers=5,
                                 hidden_size=[3, 3], epochs=meta["epochs"],
                                 dev=torch.device(dev), **kw), f


def _check(cal, f, tol):
    for k in ("loss", "ce", "log_det"):
        got = np.array([float(v) for v in cal.history[k]])
        ref = f["hist_" + k]
        assert np.max(np.abs(got - ref) / (np.abs(ref) + 1)) <= tol, k
    sd = cal.flow.state_dict()
    for k in sd:
        ref = f["p:" + k]
        assert np.max(np.abs(sd[k].numpy() - ref)) <= tol * (np.max(np.abs(ref)) + 1e-3), k
    pred = cal.predict(f["x_test"].astype(np.float64))
    assert np.max(np.abs(pred - f["pred"])) <= tol


def test_calibrator_cpu_matches_reference():
    cal, f = _fit("cpu")
    assert cal.history["loss"][0].device.type == "cpu"
    _check(cal, f, 1e-5)


@pytest.mark.gpu
def test_calibrator_native_matches_reference():
    from cnf_hip import engine
    n0 = engine.stats["loss_vjp"]
    cal, f = _fit("cuda:0")
    assert engine.stats["loss_vjp"] >= n0 + 25, "fused native training step did not run"
    assert cal.history["loss"][0].device.type == "cuda"     # no host sync per epoch
    assert next(cal.flow.parameters()).device.type == "cpu"  # flow returned to host
    _check(cal, f, 1e-5)


def test_calibrator_minibatch_cpu_matches_reference():
    """g7b: the reference's own minibatch fit (batch_size=128 of N=600)."""
    cal, f = _fit("cpu", G7B)
    _check(cal, f, 1e-5)


@pytest.mark.gpu
def test_calibrator_native_minibatch_matches_reference():
    """The native fit draws each pass's order as DataLoader(shuffle=True)
    does (calibrators._loader_order), so its 5 batches per epoch, weights,
    history (the last eval batch's sums) and predictions match g7b."""
    from cnf_hip import engine
    n0 = engine.stats["loss_vjp"]
    cal, f = _fit("cuda:0", G7B)
    meta, _ = _g7(G7B)
    assert engine.stats["loss_vjp"] >= n0 + meta["epochs"] * 5, "fused native step did not run"
    _check(cal, f, 1e-5)
    # the torch optimizer received the native Adam's state
    st = cal.optimizer.state[cal.flow.layers[0].s.layers[0].weight]
    assert int(st["step"]) == meta["epochs"] * 5


@pytest.mark.parametrize("n,bs", [(600, 128), (7, 3), (5, 5), (1, 4)])
def test_loader_order_is_the_dataloader_order(n, bs):
    """calibrators._loader_order reproduces DataLoader(TensorDataset, bs,
    shuffle=True)'s batches AND leaves torch's global CPU RNG where the loader
    leaves it (two passes in a row)."""
    from torch.utils.data import DataLoader, TensorDataset
    dl = DataLoader(TensorDataset(torch.arange(n)), batch_size=bs, shuffle=True)
    torch.manual_seed(11)
    ref = [torch.cat([b[0] for b in dl]) for _ in range(2)]
    after_ref = torch.rand(3)
    torch.manual_seed(11)
    got = [C._loader_order(n) for _ in range(2)]
    after_got = torch.rand(3)
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
    assert torch.equal(after_got, after_ref)


def test_calibrator_nice_factory_and_minibatches_cpu():
    meta, f = _g7()
    torch.manual_seed(0)
    cal = C.TorchFlowCalibrator(NiceFlow, f["x"].astype(np.float64), f["y"], layers=2,
                                hidden_size=[5, 5], epochs=3, batch_size=128, dev="cpu")
    assert len(cal.history["loss"]) == 3
    p = cal(f["x_test"].astype(np.float64))
    assert p.shape == (200, 3) and np.allclose(p.sum(axis=1), 1, atol=1e-6)
    assert float(cal.history["log_det"][-1]) == 0.0     # NICE is volume preserving
