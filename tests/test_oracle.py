"""Pin the numpy oracle against the reference's own outputs (golden fixtures)."""
import numpy as np
import pytest

from _golden import load, names, rel_err
from oracle import cnf_oracle as O

TOL = 1e-5  # north_star: <= 1e-5 rel fp32 (metric max|d|/(|ref|+1))


def _layers(meta, state, dtype=np.float32):
    ly = O.layers_from_state(state, meta["L"], meta["D"], len(meta["hidden"]) + 1,
                             meta["scale"], meta["shift"])
    return O.cast_layers(ly, dtype)


@pytest.mark.parametrize("name", [n for n in names() if not n.startswith("g5")])
def test_oracle_forward_matches_reference(name):
    meta, state, d = load(name)
    zs, ld = O.flow_forward(_layers(meta, state), d["x"])
    assert rel_err(np.stack(zs), d["zs"]) <= TOL
    assert rel_err(ld.reshape(d["ld"].shape) if d["ld"].ndim else ld[0], d["ld"]) <= TOL


@pytest.mark.parametrize("name", [n for n in names() if not n.startswith("g5")])
def test_oracle_inverse_matches_reference(name):
    meta, state, d = load(name)
    if "inv_xs" not in d:
        pytest.skip("no inverse recorded for this case")
    xs, ld = O.flow_inverse(_layers(meta, state), d["zs"][-1])
    got = np.stack(xs)
    if d["inv_xs"].shape[0] == 1:
        got = got[-1:]
    assert rel_err(got, d["inv_xs"]) <= TOL
    assert rel_err(ld.reshape(d["inv_ld"].shape), d["inv_ld"]) <= TOL


@pytest.mark.parametrize("name", names("g5"))
@pytest.mark.parametrize("kind", ["cal", "ce"])
def test_oracle_grads_match_reference(name, kind):
    meta, state, d = load(name)
    loss, grads = O.loss_and_grads(_layers(meta, state), d["x"], d["y"], kind)
    assert abs(loss - float(d["loss_" + kind])) / (abs(float(d["loss_" + kind])) + 1) <= TOL
    pre = "gcal:" if kind == "cal" else "gce:"
    worst = 0.0
    for l, gl in enumerate(grads):
        for net in ("s", "t"):
            if gl[net] is None:
                continue
            for i, (gw, gb) in enumerate(gl[net]):
                k = "layers.%d.%s.layers.%d." % (l, net, i)
                # gradients: normalise by the tensor's own scale (fp32 sums of B terms)
                for g, r in ((gw, d[pre + k + "weight"]), (gb, d[pre + k + "bias"])):
                    sc = np.max(np.abs(r)) + 1e-3
                    worst = max(worst, float(np.max(np.abs(g - r))) / sc)
    assert worst <= 1e-4, worst


def test_oracle_fp64_floor_g2():
    """fp32 reference vs the fp64 restatement: the noise floor the 1e-5 bar sits on."""
    meta, state, d = load("g2_nvp_d10_n02")
    zs, ld = O.flow_forward(_layers(meta, state, np.float64), d["x"].astype(np.float64))
    assert rel_err(zs[-1], d["zs"][-1]) <= 1e-6
    assert rel_err(ld, d["ld"]) <= 1e-6


def test_oracle_nan_case_reproduces_reference_nan():
    meta, state, d = load("g6_d4_nan")
    assert np.isnan(d["zs"][-1]).any(), "fixture should carry the reference's NaN"
    zs, ld = O.flow_forward(_layers(meta, state), d["x"])
    assert rel_err(np.stack(zs), d["zs"]) <= TOL


@pytest.mark.parametrize("name", ["g1_nice_d3_n02", "g2_nvp_d10_n02", "g3_nvp_d100_n003",
                                  "g6_d10_randflip", "g6_d10_noshift", "g6_d10_b1"])
def test_torch_port_matches_reference(name):
    import torch
    from oracle import cnf_torch_port as P
    meta, state, d = load(name)
    ly = P.layers_from_state(state, meta["L"], len(meta["hidden"]) + 1, meta["scale"],
                             meta["shift"])
    zs, ld = P.flow_forward(ly, torch.from_numpy(d["x"]))
    assert rel_err(torch.stack(zs).numpy(), d["zs"]) <= TOL
    assert rel_err(ld.numpy(), d["ld"]) <= TOL
