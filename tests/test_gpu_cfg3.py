"""BASELINE configs[2] itself: the 6-layer RealNVP D=10 eval at 2^20 rows per
rank, sharded over every visible GPU (at most 8) with RCCL (backend nccl), each
rank through bench.py's own step (cnf_forward_loss) and NllAllReduce, and
through cnf_hip.dist.sharded_nll.  The reduced sums must equal ONE rank's
fused eval over the concatenated world * 2^20 rows (<= 1e-5 relative;
reference: the single-device eval of calibrators.py:297-317) and an fp64
restatement of the calibrator NLL over every row, and 4,096 sampled rows of
every shard must match the numpy oracle (flows/flows.py:17-25, <= 1e-5).
Skipped on a box with fewer than 2 GPUs; the CPU wiring is covered by
tests/test_dist_cpu.py::test_cfg3_sharded_eval_wiring_gloo."""
import pytest
import torch

from _cfg3_worker import check_against_single, run_ranks

pytestmark = pytest.mark.gpu
ROWS = 1 << 20


def test_cfg3_rccl_sharded_eval_equals_single_device():
    n = min(torch.cuda.device_count(), 8)  # device_count() does not initialise the GPU
    if n < 2:
        pytest.skip("configs[2] needs >= 2 visible GPUs (%d visible)" % n)
    res = run_ranks(n, "nccl", ROWS)
    check_against_single(res, ROWS, torch.device("cuda:0"))
