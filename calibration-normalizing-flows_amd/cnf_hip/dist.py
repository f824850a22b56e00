"""Data-parallel coupling-flow training and evaluation, one process per GPU.

The reference trains on one device (calibrators.py:253-256); its batch is a
set of independent logit vectors, so the batch axis shards with no data-path
exchange.  Each rank runs the fused kernels on its shard and the ranks add
one flat buffer per step with a single all-reduce (RCCL over xGMI when the
process group is "nccl"; gloo for the CPU tests):

  train step  [grad_scale * d(sum of shard loss)/dW  (P floats) | loss terms (3)]
              -> all_reduce(SUM) -> Adam step on identical replicas
  eval        [loss terms (3)] -> all_reduce(SUM)

On a ROCm device the step is three launches and one collective, no host
sync: cnf_loss_vjp on the shard, the all-reduce of the flat buffer, and
cnf_adam_step (the calibrator's optimizer, calibrators.py:259, 295) reading the
reduced gradient in place.  The torch optimizer handed to the trainer supplies
the hyper-parameters and, through sync_optimizer(), receives the state.

Overlap: the all-reduce cannot run under the next step's forward (that
forward needs the updated weights); overlapping it with the reverse mode
would need per-layer buckets of the layer-at-a-time wide VJP.  At cfg4
(727,200 floats = 2.9 MB per step) a ring all-reduce over 8 ranks moves
2 * 7/8 * 2.9 MB per rank, about 40 us at 7 x 153 GB/s of xGMI even before
latency terms, against a 17-18 ms step (round 3): under 0.3 %, so one bucket
at the end of the step ships.

The native Adam step (cnf_adam_step) serves exactly torch.optim.Adam; any
other optimizer (SGD, AdamW, amsgrad) receives the reduced gradient in .grad
and steps itself.  The learning rate is re-read from the param group at every
step, so LR schedulers apply.

grad_scale = 1 / global batch, so the summed gradient is exactly the gradient
of the reference's -mean over the whole (unsharded) batch.  For cfg2
(D=10, L=6, hidden [5,5]) one step moves 1,743 floats (7 KB) per rank.
"""
import torch
import torch.distributed as dist

from . import _lib


def _native(flow, x):
    if not x.is_cuda:
        return None
    from calibrators import _native_stack
    return _native_stack(flow, x.device)


def local_loss_and_grads(flow, x, y, grad_scale, kind=_lib.LOSS_CAL, det=1.0):
    """(flat grads [P] * grad_scale, terms[3]) of the shard: the fused native
    kernel on a ROCm device, torch autograd of the same loss on CPU."""
    stack = _native(flow, x)
    if stack is not None:
        from .vjp import loss_and_grads
        terms, grads, _ = loss_and_grads(stack, x, y, kind=kind, det=det, grad_scale=grad_scale)
        return grads, terms
    params = [p for p in _coupling_params(flow)]
    with torch.enable_grad():
        z, ld = flow.transform(x) if hasattr(flow, "transform") else flow(x)
        ld = ld.reshape(-1)
        lsm = torch.log_softmax(z, dim=1)
        lpy = lsm.gather(1, y.view(-1, 1)).squeeze(1)
        if kind == _lib.LOSS_CAL:
            ce = -torch.log(torch.exp(lpy) + 1e-7)
            rows = ce - ld
        else:
            ce = -lpy
            rows = ce - det * ld
        total = rows.sum()
        grads = torch.autograd.grad(total * grad_scale, params)
    flat = torch.cat([g.reshape(-1) for g in grads])
    terms = torch.stack([rows.sum(), ce.sum(), ld.sum()]).detach()
    return flat, terms


def _coupling_params(flow):
    """Parameters in the native ABI order (per layer: s-net Linears, t-net Linears)."""
    for ly in flow.layers:
        for net, on in ((ly.s, ly.scale), (ly.t, ly.shift)):
            if on:
                for lin in net.layers:
                    yield lin.weight
                    yield lin.bias


class ShardedFlowTrainer:
    """Data-parallel trainer for a Flow of NvpCouplingLayers."""

    def __init__(self, flow, optimizer, group=None, broadcast=True, nan_guard=False):
        self.flow = flow
        self.optimizer = optimizer
        self.group = group
        # nan_guard: every native step also ORs the non-finite state of the
        # reduced [grads | loss terms] buffer into self.guard.flag (device int,
        # no host sync; the reference aborts its loop on NaN predictions,
        # run_experiment3D.py:129-131 -- read self.guard.tripped() when wanted),
        # and the step's Adam update is skipped on the device when the flag is
        # set, so the weights and moments stay at the last finite step
        self.nan_guard = nan_guard
        self.guard = None
        self.params = list(_coupling_params(flow))
        self._adam = None  # StackAdam of the native path (built on the first step)
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if broadcast and self.world > 1:
            # every replica starts from rank 0's state (weights, masks, permutations)
            with torch.no_grad():
                for t in flow.state_dict().values():
                    dist.broadcast(t, src=0, group=group)
            # collectives write in place without bumping version counters
            if hasattr(flow, "invalidate_native"):
                flow.invalidate_native()

    def step(self, x, y, global_batch, kind=_lib.LOSS_CAL, det=1.0):
        """One synchronous step on this rank's shard; returns the global
        (loss, ce, log-det) sums as a device tensor (no host sync)."""
        stack = _native(self.flow, x)
        if stack is not None:
            from .vjp import loss_and_grads
            from .adam import StackAdam
            # one flat buffer [grads | terms]: the fused kernel writes both, the
            # collective reduces both, Adam reads the gradient part in place
            P = stack.param_count()
            buf = torch.empty(P + 3, dtype=torch.float32, device=x.device)
            loss_and_grads(stack, x, y, kind=kind, det=det, grad_scale=1.0 / global_batch,
                           grads_out=buf[:P], terms_out=buf[P:])
            if self.world > 1:
                dist.all_reduce(buf, group=self.group)
            if self.nan_guard:
                if self.guard is None:
                    from .guard import NonFiniteGuard
                    self.guard = NonFiniteGuard(x.device)
                self.guard.check(buf)
            from .adam import supports, group_hparams
            hp = group_hparams(self.optimizer, stack) if supports(self.optimizer) else None
            if hp is None:
                # any other optimizer (SGD, AdamW, amsgrad ...), or tensor-valued
                # hyper-parameters, steps itself on the reduced gradient, as on
                # the CPU path (the native moments, if any, go back first)
                if self._adam is not None:
                    self._adam.store_into(self.optimizer)
                    self._adam = None
                self._set_grads(buf[:P])
                # a torch optimizer cannot read the device flag: with the guard
                # on, the host checks it (one sync) and skips a tripped step
                if not (self.nan_guard and self.guard.tripped()):
                    self.optimizer.step()
                return buf[P:]
            if self._adam is None or self._adam.stack is not stack:
                if self._adam is not None:
                    # a rebuilt stack (e.g. after invalidate_native): carry the
                    # moments and step count over through the torch state
                    self._adam.store_into(self.optimizer)
                self._adam = StackAdam.like(stack, self.optimizer)
            # schedulers may move lr, betas (OneCycleLR / CyclicLR momentum
            # cycling), eps or weight decay between steps: read all of them
            self._adam.set_hparams(hp)
            # guarded: a step whose reduced gradient or sums are non-finite
            # updates nothing (the reference breaks out before opt.step(),
            # run_experiment3D.py:129-133, keeping the last finite weights)
            self._adam.step(buf[:P], skip=self.guard.flag if self.nan_guard else None)
            return buf[P:]
        grads, terms = local_loss_and_grads(self.flow, x, y, 1.0 / global_batch, kind, det)
        buf = torch.cat([grads, terms])
        if self.world > 1:
            dist.all_reduce(buf, group=self.group)
        off = self._set_grads(buf)
        self.optimizer.step()
        return buf[off:off + 3]

    def _set_grads(self, flat):
        """Scatter the flat (reduced) gradient into the parameters' .grad;
        returns the number of floats consumed."""
        off = 0
        for p in self.params:
            n = p.numel()
            p.grad = flat[off:off + n].view_as(p).clone()
            off += n
        return off

    def sync_optimizer(self):
        """Write the native Adam's step count and moments into the torch
        optimizer's state (no-op on the torch path, which steps it directly)."""
        if self._adam is not None:
            self._adam.store_into(self.optimizer)

    @torch.no_grad()
    def evaluate(self, x, y, kind=_lib.LOSS_CAL, det=1.0):
        """Global (loss, ce, log-det) sums over all shards."""
        stack = _native(self.flow, x)
        if stack is not None:
            terms, _, _ = stack.forward_loss(x, y, kind=kind, det=det)
        else:
            _, terms = local_loss_and_grads(self.flow, x, y, 0.0, kind, det)
        terms = terms.clone()
        if self.world > 1:
            dist.all_reduce(terms, group=self.group)
        return terms


@torch.no_grad()
def sharded_nll(flow, x, y, group=None, kind=_lib.LOSS_CAL, det=1.0):
    """configs[2]'s step: this rank's shard through the fused forward + loss
    (cnf_forward_loss on a ROCm device, the torch path on CPU), then ONE
    all-reduce of the 3 sums.  Returns the global (loss, ce, ld) sums; divide
    by the global row count for the reference's means (calibrators.py:297-317)."""
    stack = _native(flow, x)
    if stack is not None:
        terms, _, _ = stack.forward_loss(x, y, kind=kind, det=det)
    else:
        _, terms = local_loss_and_grads(flow, x, y, 0.0, kind, det)
    terms = terms.clone()
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(terms, group=group)
    return terms


def shard(n, rank, world):
    """Contiguous [start, stop) of rank's shard of n rows."""
    per = (n + world - 1) // world
    start = min(n, rank * per)
    return start, min(n, start + per)
