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


def _g7():
    f = np.load(os.path.join(GOLDEN, "g7_calibrator_d3.npz"))
    return json.loads(str(f["meta"])), f


def _fit(dev):
    meta, f = _g7()
    torch.manual_seed(meta["seed"])
    np.random.seed(meta["seed"])
    return C.TorchFlowCalibrator(RealNvpFlow, f["x"].astype(np.float64), f["y"], layers=5,
                                 hidden_size=[3, 3], epochs=meta["epochs"],
                                 dev=torch.device(dev)), f


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


def test_calibrator_nice_factory_and_minibatches_cpu():
    meta, f = _g7()
    torch.manual_seed(0)
    cal = C.TorchFlowCalibrator(NiceFlow, f["x"].astype(np.float64), f["y"], layers=2,
                                hidden_size=[5, 5], epochs=3, batch_size=128, dev="cpu")
    assert len(cal.history["loss"]) == 3
    p = cal(f["x_test"].astype(np.float64))
    assert p.shape == (200, 3) and np.allclose(p.sum(axis=1), 1, atol=1e-6)
    assert float(cal.history["log_det"][-1]) == 0.0     # NICE is volume preserving
