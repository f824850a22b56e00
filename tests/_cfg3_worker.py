"""One rank of BASELINE configs[2] (tests/test_gpu_cfg3.py, tests/test_dist_cpu.py):
the 6-layer RealNVP D=10 eval sharded over ranks, each rank's rows through
the fused forward + log-det + NLL sums, then the one real exchange, an
all-reduce of the 3 sums.

  nccl (RCCL over xGMI): rank r on cuda:LOCAL_RANK, its shard through
       bench.py's own step (Runner, cnf_forward_loss) and its NllAllReduce,
       and through cnf_hip.dist.sharded_nll;
  gloo (CPU): cnf_hip.dist.sharded_nll on CPU tensors (the torch path) --
       the same sharding and collective wiring without a GPU.

Rank r's shard is bench.synthetic_logits(rows, 10, dev, SEED + r); the
parent regenerates every shard to check the reduced sums and sampled rows.
argv: out_dir backend rows_per_rank"""
import os
import subprocess
import sys
import tempfile

import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "calibration-normalizing-flows_amd"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

SEED = 5000
NSAMPLE = 4096


def shard_data(rows, rank, dev):
    import bench
    if dev.type == "cuda":
        return bench.synthetic_logits(rows, 10, dev, SEED + rank)
    g = torch.Generator().manual_seed(SEED + rank)
    x = torch.randn(rows, 10, generator=g)
    y = torch.randint(0, 10, (rows,), generator=g)
    x[torch.arange(rows), y] += 2.0
    return x - x.mean(dim=1, keepdim=True), y


def workload(rows):
    import bench
    return dict(bench.WORKLOADS["cfg2"], B=rows)


def run_ranks(world, backend, rows, timeout=240):
    """Start `world` _cfg3_worker.py ranks; returns their saved results."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = str(s.getsockname()[1])
    s.close()
    out = tempfile.mkdtemp()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, os.path.basename(__file__)),
                                       out, backend, str(rows)], env=env))
    codes = []
    for p in procs:
        try:
            codes.append(p.wait(timeout=timeout))
        except subprocess.TimeoutExpired:
            p.kill()
            codes.append(-9)
    assert codes == [0] * world, codes
    return [torch.load(os.path.join(out, "rank%d.pt" % r), weights_only=True)
            for r in range(world)]


def check_against_single(res, rows, dev):
    """The reduced sums vs one eval over every shard; sampled rows vs the oracle."""
    import bench
    from _golden import rel_err
    from oracle import cnf_oracle as O
    world = len(res)
    w = workload(rows * world)
    flow = bench.make_flow(w, dev)
    xs, ys = zip(*[shard_data(rows, r, dev) for r in range(world)])
    x, y = torch.cat(xs), torch.cat(ys)
    from cnf_hip.dist import sharded_nll
    single = sharded_nll(flow, x, y).double().cpu()  # no process group: one device, all rows
    for r in res:
        assert r["world"] == world
        assert torch.equal(r["terms"], res[0]["terms"]), "ranks disagree on the reduced sums"
        if "bench_terms" in r:
            assert torch.equal(r["bench_terms"], r["terms"])
    got = res[0]["terms"]
    # different summation orders (per-rank block sums, then the all-reduce):
    # the sums agree to fp32 accumulation error, far inside 1e-5 relative
    assert ((got - single).abs() / single.abs()).max().item() <= 1e-5, (got, single)
    # and an fp64 restatement of the calibrator NLL (calibrators.py:289, the
    # kind sharded_nll uses) over every row of every shard, from the full
    # batch's forward -- whose rows are checked against the oracle below
    with torch.no_grad():
        zf, ldf = flow.transform(x)
    lpy = torch.log_softmax(zf.double(), dim=1).gather(1, y.view(-1, 1)).squeeze(1)
    ce = -torch.log(torch.exp(lpy) + 1e-7)
    ldd = ldf.double().reshape(-1)
    ref = torch.stack([(ce - ldd).sum(), ce.sum(), ldd.sum()]).cpu()
    n = rows * world
    assert ((got - ref).abs() <= 1e-5 * (ref.abs() + n)).all(), (got, ref)
    st = {k: v.detach().cpu().numpy() for k, v in flow.state_dict().items()}
    ol = O.layers_from_state(st, w["L"], 10, len(w["hidden"]) + 1)
    for rk, r in enumerate(res):
        xr = xs[rk][r["idx"].to(dev)].cpu().numpy()
        ozs, old = O.flow_forward(ol, xr)
        assert rel_err(r["z"].numpy(), ozs[-1]) <= 1e-5
        assert rel_err(r["ld"].numpy(), old) <= 1e-5


def main():
    out_dir, backend, rows = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import bench
    from cnf_hip.dist import sharded_nll
    if backend == "nccl":
        dev = torch.device("cuda", int(os.environ["LOCAL_RANK"]))
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", init_method="env://", device_id=dev)
    else:
        dev = torch.device("cpu")
        dist.init_process_group("gloo", init_method="env://")
    w = workload(rows)
    x, y = shard_data(rows, rank, dev)
    res = {"world": dist.get_world_size(), "backend": backend}
    if backend == "nccl":
        r = bench.Runner(w, dev, 0.0, mode="loss", data=(x, y))
        coll = bench.NllAllReduce(r)
        r.step()
        coll()
        coll.drain()
        torch.cuda.synchronize(dev)
        res["bench_terms"] = r.terms.double().cpu()
        flow = r.flow
        z, ld = r.sets[0][2], r.sets[0][3]
    else:
        flow = bench.make_flow(w, dev)
        with torch.no_grad():
            z, ld = flow.transform(x)
    res["terms"] = sharded_nll(flow, x, y).double().cpu()
    idx = torch.randperm(rows, generator=torch.Generator().manual_seed(rank))[:NSAMPLE]
    res["idx"] = idx
    res["z"] = z[idx.to(dev)].cpu()
    res["ld"] = ld[idx.to(dev)].cpu()
    torch.save(res, os.path.join(out_dir, "rank%d.pt" % rank))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
