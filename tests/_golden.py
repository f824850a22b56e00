"""Loader for the committed golden fixtures (tests/golden/*.npz).

The fixtures were produced by tests/golden/gen_golden.py from the reference's
own flows/flows.py.  This loader reads only the .npz files, so it works on the
GPU box where the reference is absent.
"""
import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _param_keys(meta):
    keys = []
    n_lin = len(meta["hidden"]) + 1
    for l in range(meta["L"]):
        for net, on in (("s", meta["scale"]), ("t", meta["shift"])):
            if not on:
                continue
            for i in range(n_lin):
                keys.append("layers.%d.%s.layers.%d.weight" % (l, net, i))
                keys.append("layers.%d.%s.layers.%d.bias" % (l, net, i))
    return keys


def _param_shapes(meta):
    units = [meta["D"]] + list(meta["hidden"]) + [meta["D"]]
    shapes = []
    for _ in range(meta["L"]):
        for on in (meta["scale"], meta["shift"]):
            if not on:
                continue
            for i in range(len(units) - 1):
                shapes.append((units[i + 1], units[i]))
                shapes.append((units[i + 1],))
    return shapes


def load(name):
    """Returns (meta, state, data): state is a reference-style state dict."""
    f = np.load(os.path.join(GOLDEN, name + ".npz"))
    meta = json.loads(str(f["meta"]))
    state = {k[2:]: f[k] for k in f.files if k.startswith("p:")}
    keys = _param_keys(meta)
    if any(k not in state for k in keys):
        # big cases: regenerate 'normal:sigma' weights (gen_golden.py build())
        sigma = float(meta["init"].split(":")[1])
        rs = np.random.RandomState(meta["seed"] + 1000)
        for k, shp in zip(keys, _param_shapes(meta)):
            state[k] = (rs.standard_normal(shp) * sigma).astype(np.float32)
    h = hashlib.sha256()
    for k in keys:
        h.update(np.ascontiguousarray(state[k]).tobytes())
    assert h.hexdigest() == meta["wsha"], "golden weights do not match the recorded sha256"
    data = {k: f[k] for k in f.files if not k.startswith("p:") and k != "meta"}
    return meta, state, data


def names(prefix=""):
    """Flow-output fixtures (g1-g6); the calibrator fixture g7 only by prefix."""
    return sorted(n[:-4] for n in os.listdir(GOLDEN)
                  if n.endswith(".npz") and n.startswith(prefix)
                  and (prefix.startswith("g7") or not n.startswith("g7")))


def rel_err(a, b):
    """SURVEY.md 8(c) metric: max |a-b| / (|b| + 1); NaNs must coincide."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if a.shape != b.shape:
        raise AssertionError("shape %s vs %s" % (a.shape, b.shape))
    if a.size == 0:
        return 0.0
    na, nb = np.isnan(a), np.isnan(b)
    if (na != nb).any():
        return float("inf")
    fin = ~nb
    ia, ib = np.isinf(a) & fin, np.isinf(b) & fin
    if (ia != ib).any() or (a[ib] != b[ib]).any():
        return float("inf")
    ok = fin & ~ib
    if not ok.any():
        return 0.0
    return float(np.max(np.abs(a[ok] - b[ok]) / (np.abs(b[ok]) + 1.0)))
