"""Legacy semantics (flows/legacy.py, include/cnf.h CNF_OPT_ALT_MASK /
CNF_OPT_S_TANH) on the native kernels (k_valu for the D <= 16 shapes of its
tables, the MFMA-tile family otherwise) against the torch
restatement on the CPU.  Parity UNPINNED against the reference itself
(code-old/realNVP.py needs TensorFlow, absent): the restatement is the check."""
import os
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "calibration-normalizing-flows_amd"))

from cnf_hip import engine  # noqa: E402
from flows.legacy import LegacyRealNvpFlow  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _legacy(D, L, hidden, s_act, seed=0, sigma=0.2):
    torch.manual_seed(seed)
    f = LegacyRealNvpFlow(D, layers=L, hidden_size=hidden, s_activation=s_act)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for p in f.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * sigma)
    return f


def _rel(a, b):
    return ((a - b).abs() / (b.abs() + 1)).max().item()


# legacy shapes k_valu serves (its tables: cnf_valu.hip kTable, and kLTable for
# the tanh s-net); every other legacy shape stays on the MFMA-tile family
_NARROW = {(10, (10,)), (10, (5, 5)), (3, (3,))}


def _kernel(D, hidden):
    return "valu-fused" if (D, tuple(hidden)) in _NARROW else "mfma-tile"


@pytest.mark.parametrize("D,L,hidden,s_act", [
    (10, 4, [10], "tanh"),      # code-old defaults: hidden [dim], layers 4
    (10, 3, [5, 5], "tanh"),    # odd L: one final un-flip
    (3, 5, [3], "tanh"),        # odd D and L, hidden [dim] (k_valu tanh table)
    (7, 5, [6], "relu"),        # odd D
    (100, 2, [100, 100], "tanh"),
    (20, 1, [], "tanh"),
])
def test_legacy_forward_inverse_and_grads(D, L, hidden, s_act):
    f = _legacy(D, L, hidden, s_act, sigma=0.2 if D <= 20 else 0.05)
    x = torch.randn(513, D, generator=torch.Generator().manual_seed(3))
    w = torch.randn(513, D, generator=torch.Generator().manual_seed(4))
    with torch.no_grad():
        y_ref, ld_ref = f(x)
        x_back, ild_ref = f.backward(y_ref)
    xc = x.clone().requires_grad_(True)
    y2, ld2 = f(xc)
    ((y2 * w).sum() + ld2.sum()).backward()
    g_ref = {k: p.grad.clone() for k, p in f.named_parameters()}
    gx_ref = xc.grad.clone()

    fg = f.to(DEV)
    assert fg._native_stack().kernel_name() == _kernel(D, hidden)
    n0 = engine.stats["forward"] + engine.stats["inverse"]
    with torch.no_grad():
        y, ld = fg(x.to(DEV))
        xb, ild = fg.backward(y_ref.to(DEV))
    assert engine.stats["forward"] + engine.stats["inverse"] >= n0 + 2, "native path did not run"
    assert _rel(y.cpu(), y_ref) <= 1e-5 and _rel(ld.cpu(), ld_ref) <= 1e-5
    assert _rel(xb.cpu(), x_back) <= 1e-5 and _rel(ild.cpu(), ild_ref) <= 1e-5
    fg.zero_grad()
    xg = x.to(DEV).requires_grad_(True)
    y3, ld3 = fg(xg)
    ((y3 * w.to(DEV)).sum() + ld3.sum()).backward()
    for k, p in fg.named_parameters():
        sc = g_ref[k].abs().max().item() + 1e-3
        assert (p.grad.cpu() - g_ref[k]).abs().max().item() / sc <= 1e-4, k
    sc = gx_ref.abs().max().item() + 1e-3
    assert (xg.grad.cpu() - gx_ref).abs().max().item() / sc <= 1e-4


@pytest.mark.parametrize("D,L,hidden", [
    (10, 4, [10]),      # code-old/nice.py defaults: hidden [dim], layers 4
    (7, 3, [5, 5]),     # odd D, odd L
    (100, 2, [100]),
])
def test_legacy_nice_v3_native_matches_restatement(D, L, hidden):
    """NiceFlow_v3 (code-old/nice.py:214-263) as CNF_OPT_ALT_MASK on the
    shift-only kernels: forward, inverse and gradients vs the CPU torch
    restatement (parity unpinned: TensorFlow absent)."""
    from flows.legacy import LegacyNiceFlow
    torch.manual_seed(0)
    f = LegacyNiceFlow(D, layers=L, hidden_size=hidden, version=3)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for p in f.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * (0.2 if D <= 20 else 0.05))
    x = torch.randn(257, D, generator=torch.Generator().manual_seed(3))
    w = torch.randn(257, D, generator=torch.Generator().manual_seed(4))
    with torch.no_grad():
        y_ref, _ = f(x)
        x_back, _ = f.backward(y_ref)
    xc = x.clone().requires_grad_(True)
    (f(xc)[0] * w).sum().backward()
    g_ref = {k: p.grad.clone() for k, p in f.named_parameters()}
    gx_ref = xc.grad.clone()

    fg = f.to(DEV)
    assert fg._native_stack().kernel_name() == _kernel(D, hidden)
    n0 = engine.stats["forward"] + engine.stats["inverse"]
    with torch.no_grad():
        y, ld = fg(x.to(DEV))
        xb, ild = fg.backward(y_ref.to(DEV))
    assert engine.stats["forward"] + engine.stats["inverse"] >= n0 + 2, "native path did not run"
    assert _rel(y.cpu(), y_ref) <= 1e-5 and _rel(xb.cpu(), x_back) <= 1e-5
    assert ld.abs().max().item() == 0 and ild.abs().max().item() == 0
    fg.zero_grad()
    xg = x.to(DEV).requires_grad_(True)
    (fg(xg)[0] * w.to(DEV)).sum().backward()
    for k, p in fg.named_parameters():
        sc = g_ref[k].abs().max().item() + 1e-3
        assert (p.grad.cpu() - g_ref[k]).abs().max().item() / sc <= 1e-4, k
    sc = gx_ref.abs().max().item() + 1e-3
    assert (xg.grad.cpu() - gx_ref).abs().max().item() / sc <= 1e-4


@pytest.mark.parametrize("version,D,L,hidden", [
    (1, 10, 4, [10]),     # code-old/nice.py NiceFlow defaults: hidden [dim], layers 4
    (1, 6, 3, [5, 5]),    # odd L: one more reversal
    (1, 4, 2, []),        # one Linear per conditioner
    (1, 7, 3, [5, 5]),    # odd D: 'odd' layers add to the larger half (padded stack)
    (1, 3, 4, [3]),       # odd D, even L, hidden [dim]
    (1, 5, 1, []),        # odd D, one Linear
    (2, 10, 4, [10]),     # NiceFlow_v2
    (2, 7, 3, [5, 5]),    # odd D, odd L
    (2, 3, 2, []),
])
def test_legacy_nice_split_versions_native(version, D, L, hidden):
    """NiceFlow / NiceFlow_v2 (code-old/nice.py:101-212) natively: the
    half-width Keras conditioners zero-embedded into the maintained additive
    layer (flows/legacy.py _EmbeddedNice).  Forward, inverse and every
    gradient vs the CPU torch restatement (parity unpinned: TensorFlow
    absent)."""
    from flows.legacy import LegacyNiceFlow
    torch.manual_seed(0)
    f = LegacyNiceFlow(D, layers=L, hidden_size=hidden, version=version)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for p in f.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.2)
    x = torch.randn(257, D, generator=torch.Generator().manual_seed(3))
    w = torch.randn(257, D, generator=torch.Generator().manual_seed(4))
    with torch.no_grad():
        y_ref, _ = f(x)
        x_back, _ = f.backward(y_ref)
    xc = x.clone().requires_grad_(True)
    (f(xc)[0] * w).sum().backward()
    g_ref = {k: p.grad.clone() for k, p in f.named_parameters()}
    gx_ref = xc.grad.clone()

    fg = f.to(DEV)
    n0 = engine.stats["forward"] + engine.stats["inverse"]
    with torch.no_grad():
        y, ld = fg(x.to(DEV))
        xb, ild = fg.backward(y_ref.to(DEV))
    assert engine.stats["forward"] + engine.stats["inverse"] >= n0 + 2, "native path did not run"
    assert _rel(y.cpu(), y_ref) <= 1e-5 and _rel(xb.cpu(), x_back) <= 1e-5
    assert ld.abs().max().item() == 0 and ild.abs().max().item() == 0
    fg.zero_grad()
    v0 = engine.stats["vjp"]
    xg = x.to(DEV).requires_grad_(True)
    (fg(xg)[0] * w.to(DEV)).sum().backward()
    assert engine.stats["vjp"] > v0, "native reverse mode did not run"
    for k, p in fg.named_parameters():
        sc = g_ref[k].abs().max().item() + 1e-3
        assert (p.grad.cpu() - g_ref[k]).abs().max().item() / sc <= 1e-4, k
    sc = gx_ref.abs().max().item() + 1e-3
    assert (xg.grad.cpu() - gx_ref).abs().max().item() / sc <= 1e-4
    # an optimizer-style in-place update reaches the kernels
    with torch.no_grad():
        for p in fg.parameters():
            p.mul_(0.5)
        y2, _ = fg(x.to(DEV))
    f2 = LegacyNiceFlow(D, layers=L, hidden_size=hidden, version=version)
    f2.load_state_dict({k: v.cpu() for k, v in fg.state_dict().items()})
    with torch.no_grad():
        y2_ref, _ = f2(x)
    assert _rel(y2.cpu(), y2_ref) <= 1e-5


def test_legacy_nice_v1_odd_dim_is_native():
    """NiceFlow (version 1) with odd D transforms the larger half in its 'odd'
    layers (code-old/nice.py:140-155); it runs natively over the D + 1-wide
    padded stack (flows/legacy.py) with no torch-ops warning, and equals the
    CPU restatement (parity unpinned: TensorFlow absent)."""
    import warnings
    from flows.legacy import LegacyNiceFlow
    import flows.flows as FF
    torch.manual_seed(0)
    f = LegacyNiceFlow(7, layers=3, version=1)
    x = torch.randn(64, 7)
    with torch.no_grad():
        y_ref, _ = f(x)
    fg = f.to(DEV)
    FF._warned.clear()
    n0 = engine.stats["forward"]
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)
        with torch.no_grad():
            y, _ = fg(x.to(DEV))
    assert engine.stats["forward"] > n0, "native path did not run"
    assert _rel(y.cpu(), y_ref) <= 1e-5
