"""One rank of tests/test_gpu_dist.py: the data-parallel trainer on device
tensors.  Backend "gloo" (argv[2], the default): every rank on cuda:0 (two
ranks share the one GPU of the test box; RCCL refuses two ranks per device).
Backend "nccl" (RCCL over xGMI): rank r on cuda:LOCAL_RANK, one GPU each.
Runs the native fused loss + VJP kernels (cnf_loss_vjp), the native Adam step
(cnf_adam_step) and the fused eval (cnf_forward_loss)."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "calibration-normalizing-flows_amd"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

N, D, L, STEPS = 1 << 16, 10, 6, 3


def make_flow():
    from flows.realNVP_torch import RealNvpFlow
    torch.manual_seed(3)
    np.random.seed(3)
    f = RealNvpFlow(D, layers=L, hidden_size=[5, 5])
    g = torch.Generator().manual_seed(4)
    with torch.no_grad():
        for p in f.parameters():
            if p.requires_grad:
                p.copy_(torch.randn(p.shape, generator=g) * 0.1)
    return f


def data(dev):
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, D, generator=g)
    y = torch.randint(0, D, (N,), generator=g)
    return x.to(dev), y.to(dev)


def main():
    out = sys.argv[1]
    backend = sys.argv[2] if len(sys.argv) > 2 else "gloo"
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", int(os.environ["LOCAL_RANK"]) if backend == "nccl" else 0)
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", init_method="env://", device_id=dev)
    else:
        dist.init_process_group("gloo", init_method="env://")
    from cnf_hip import engine
    from cnf_hip.dist import ShardedFlowTrainer, shard
    f = make_flow()
    if rank == 1:  # replicas must be re-synchronised by the trainer's broadcast
        with torch.no_grad():
            for p in f.parameters():
                p.add_(0.5)
    f = f.to(dev)
    tr = ShardedFlowTrainer(f, torch.optim.Adam(f.parameters(), lr=1e-2))
    x, y = data(dev)
    a, b = shard(N, rank, world)
    n0 = engine.stats["loss_vjp"]
    a0 = engine.stats.get("adam", 0)
    terms = [tr.step(x[a:b], y[a:b], N) for _ in range(STEPS)]
    ev = tr.evaluate(x[a:b], y[a:b])
    native = min(engine.stats["loss_vjp"] - n0, engine.stats.get("adam", 0) - a0)
    torch.cuda.synchronize()
    if rank == 0:
        torch.save({"params": {k: v.detach().cpu().clone() for k, v in f.state_dict().items()},
                    "terms": torch.stack(terms).cpu(), "eval": ev.cpu(),
                    "native_steps": native, "world": world, "backend": backend}, out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
