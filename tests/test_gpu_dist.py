"""The data-parallel composition on the GPU: ranks (processes) each run the
native fused loss + VJP kernels on their shard, add gradients with one
all-reduce per step and step Adam natively (cnf_hip/dist.py).  The result must
equal single-process full-batch training and the reference's loss
(calibrators.py:284-295) at <= 1e-5.
  * gloo, 2 ranks on one device (always runs: RCCL refuses two ranks per GPU);
  * nccl (RCCL over xGMI), one rank per visible GPU (configs[2]'s collective),
    skipped on a box with fewer than 2 GPUs."""
import os
import socket
import subprocess
import sys
import tempfile

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
DEV = "cuda:0"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _visible_gpus():
    # device_count() does not initialise the GPU in this (parent) process
    return torch.cuda.device_count()


def _run_ranks(world, backend):
    import _dist_gpu_worker as W
    out = os.path.join(tempfile.mkdtemp(), "r0.pt")
    port = str(_free_port())
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_dist_gpu_worker.py"),
                                       out, backend], env=env))
    codes = []
    for p in procs:
        try:
            codes.append(p.wait(timeout=240))
        except subprocess.TimeoutExpired:
            p.kill()
            codes.append(-9)
    assert codes == [0] * world, codes
    got = torch.load(out, weights_only=True)
    assert got["native_steps"] == W.STEPS, "ranks did not run cnf_loss_vjp + cnf_adam_step"
    assert got["world"] == world and got["backend"] == backend
    _check_against_full_batch(got)


def test_two_rank_native_sharded_training_equals_full_batch():
    _run_ranks(2, "gloo")


def test_rccl_all_gpus_sharded_training_equals_full_batch():
    """The RCCL path of configs[2]: one rank per visible GPU (at most 8),
    backend nccl (= RCCL over xGMI on ROCm).  Needs a multi-GPU box."""
    n = min(_visible_gpus(), 8)
    if n < 2:
        pytest.skip("needs >= 2 visible GPUs for an RCCL run (%d visible)" % n)
    _run_ranks(n, "nccl")


def _check_against_full_batch(got):
    import _dist_gpu_worker as W
    from cnf_hip import vjp as V
    # single process, full batch, the same native kernels
    f = W.make_flow().to(DEV)
    stack = f._native_stack()
    opt = torch.optim.Adam(f.parameters(), lr=1e-2)
    x, y = W.data(DEV)
    params = stack.param_tensors()
    sums = []
    for _ in range(W.STEPS):
        terms, grads, _ = V.loss_and_grads(stack, x, y, grad_scale=1.0 / W.N)
        for p, g in zip(params, V._split(stack, grads)):
            p.grad = g.clone()
        opt.step()
        sums.append(terms[0].item())
    for k, v in f.state_dict().items():
        ref = v.detach().cpu()
        assert torch.allclose(got["params"][k], ref, atol=1e-5, rtol=1e-5), k
    for s_got, s_ref in zip(got["terms"][:, 0].tolist(), sums):
        assert abs(s_got - s_ref) / W.N <= 1e-5 * (abs(s_ref) / W.N + 1)
    # and the reference's own loss on the full batch after the last step
    with torch.no_grad():
        z, ld = f.transform(x)
        probs = torch.softmax(z, dim=1)
        ce = torch.log(probs.gather(1, y.view(-1, 1)) + 1e-7)
        full = -torch.mean(ce.squeeze() + ld).item()
    assert abs(got["eval"][0].item() / W.N - full) <= 1e-5 * (abs(full) + 1)
