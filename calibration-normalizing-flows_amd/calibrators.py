"""Drop-in mirror of the reference's calibrators.py for the flow calibrator.

`Calibrator` (base: logit centring, one-hot targets, prior correction) and
`TorchFlowCalibrator` keep the reference's constructor, `fit` schedule, history
format and `predict` path (calibrators.py:13-44, 239-353).  When the flow built
by the factory is a stack of NvpCouplingLayers on a ROCm device, each training
step is ONE fused native launch (forward + calibrator loss + reverse mode,
cnf_loss_vjp) followed by the optimizer step, and the per-epoch evaluation is
ONE fused forward + loss launch (cnf_forward_loss); history entries stay
device tensors, as in the reference, so no step synchronises the host.
Any other flow (or a CPU device) runs the reference's own torch loop.

Out of scope here (host-side, non-flow calibrators of the reference):
TempScaling / Matrix / Vector / MLR / PAV calibrators (calibrators.py:55-236).
"""
import numpy as np
import torch
from scipy.special import softmax
from torch import nn
from torch.utils.data import DataLoader, TensorDataset


def _onehot(target, n_classes=None):
    """utils/ops.py:42-51 (onehot_encode)."""
    target = np.asarray(target).astype(int).reshape(-1)
    n = int(target.max()) + 1 if n_classes is None else n_classes
    out = np.zeros((target.shape[0], n))
    out[np.arange(target.shape[0]), target] = 1
    return out


class Calibrator:
    """Abstract calibrator (calibrators.py:13-44)."""

    def __init__(self, logits, target):
        logits = logits - np.mean(logits, axis=1, keepdims=True)
        self.logits = logits
        if target.shape != logits.shape:
            target = _onehot(target, logits.shape[1])
        self.target = target
        (_, self.n_classes) = target.shape
        self.log_priors = self._get_log_priors(target)

    def __call__(self, logits):
        return self.predict(logits)

    def _get_log_priors(self, target):
        priors = np.sum(target, axis=0)
        priors = priors / np.sum(priors)
        return np.log(priors)

    def predict_post(self, logits):
        raise NotImplementedError

    def predict(self, logits):
        logits = logits - np.mean(logits, axis=1, keepdims=True)
        probs = self.predict_post(logits)
        return softmax(np.log(probs + 1e-7) - self.log_priors, axis=1)


class DummyCalibrator(Calibrator):
    """Uncalibrated model (calibrators.py:47-53)."""

    def predict_post(self, logits):
        return softmax(logits, axis=1)


def _native_stack(flow, dev, need_vjp=True):
    """The fused CouplingStack behind `flow`, or None when the flow is not a
    stack of NvpCouplingLayers or the device is not a ROCm GPU (need_vjp: the
    shape must also have a native reverse mode)."""
    if torch.device(dev).type != "cuda":
        return None
    try:
        from flows.flows import Flow, NvpCouplingLayer
        from cnf_hip import _lib
    except ImportError:
        return None
    if not isinstance(flow, Flow) or not all(isinstance(l, NvpCouplingLayer) for l in flow.layers):
        return None
    if flow._strict():
        return None
    stack = flow._native_stack()
    if not need_vjp:
        return stack
    try:
        import ctypes
        n = ctypes.c_size_t()
        st = _lib.lib().cnf_vjp_workspace_bytes(ctypes.byref(stack.desc), ctypes.c_int64(1),
                                                ctypes.byref(n))
    except Exception:
        return None
    return stack if st == 0 else None


def _loader_order(n):
    """The row order of one pass of DataLoader(TensorDataset(...), batch_size,
    shuffle=True) (calibrators.py:274-275) with torch's global CPU RNG in the
    same state: creating the loader iterator draws its base seed
    (torch.utils.data._BaseDataLoaderIter), then the RandomSampler draws the
    seed of a fresh CPU generator and takes randperm(n) from it.  Both draws
    are reproduced, so the global RNG advances exactly as in the reference.
    Returns a pinned int64 CPU tensor (one async H2D per pass)."""
    torch.empty((), dtype=torch.int64).random_()  # the iterator's _base_seed
    seed = int(torch.empty((), dtype=torch.int64).random_().item())
    g = torch.Generator()
    g.manual_seed(seed)
    order = torch.randperm(n, generator=g)
    return order.pin_memory() if torch.cuda.is_available() else order


class _EpochRunner:
    """One training epoch of TorchFlowCalibrator.fit on the fused kernels
    (calibrators.py:284-317): gather the pass's rows in loader order, per
    batch cnf_loss_vjp + Adam, then the eval pass's cnf_forward_loss per batch,
    whose LAST batch's sums are the epoch's history terms."""

    def __init__(self, stack, adam, logits, target, bs):
        self.stack, self.adam, self.x, self.y, self.bs = stack, adam, logits, target, bs
        self.N = logits.shape[0]
        self.nb = (self.N + bs - 1) // bs

    def body(self, order_tr, order_ev, terms_out, sched=None):
        from cnf_hip import vjp as V
        N, bs = self.N, self.bs
        xs, ys = self.x.index_select(0, order_tr), self.y.index_select(0, order_tr)
        for b, s in enumerate(range(0, N, bs)):
            xb, yb = xs[s:s + bs], ys[s:s + bs]
            _, grads, _ = V.loss_and_grads(self.stack, xb, yb, grad_scale=1.0 / xb.shape[0])
            if sched is None:
                self.adam.step(grads)
            else:
                self.adam.step_sched(grads, sched[b])
        xe, ye = self.x.index_select(0, order_ev), self.y.index_select(0, order_ev)
        for s in range(0, N, bs):
            last = s + bs >= N
            self.stack.forward_loss(xe[s:s + bs], ye[s:s + bs],
                                    terms_out=terms_out if last else None)

    def eager_epoch(self, terms_out):
        dev = self.x.device
        o_tr = _loader_order(self.N).to(dev, non_blocking=True)
        o_ev = _loader_order(self.N).to(dev, non_blocking=True)
        self.body(o_tr, o_ev, terms_out)


class _EpochGraph:
    """K epochs of _EpochRunner captured once as a HIP graph (torch.cuda.graph;
    every launch of the C ABI goes to the capturing stream).  Per replay the
    host draws the K epochs' loader orders (the global CPU RNG advances as the
    reference's DataLoader would) and the Adam scalars of the K * nb steps,
    stages both with ONE host-to-device copy into the graph's static buffers,
    replays, and copies the K per-epoch terms out."""

    CHUNK = 50

    def __init__(self, run, K):
        self.run, self.K = run, K
        N, nb, dev = run.N, run.nb, run.x.device
        self.ord = torch.empty(K, 2, N, dtype=torch.int64, device=dev)
        self.sched = torch.empty(K, nb, 2, dtype=torch.float32, device=dev)
        self.terms = torch.empty(K, 3, dtype=torch.float32, device=dev)
        run.stack.invalidate()  # the graph's first launch re-prepares the weights
        t0 = run.adam.t
        torch.cuda.synchronize(dev)
        self.g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g):
            for k in range(K):
                run.body(self.ord[k, 0], self.ord[k, 1], self.terms[k], sched=self.sched[k])
        run.adam.t = t0  # capture recorded the steps; replays perform them

    def replay(self, terms_dst):
        run, K, N, nb = self.run, self.K, self.run.N, self.run.nb
        orders = torch.empty(K, 2, N, dtype=torch.int64)
        for k in range(K):
            orders[k, 0] = _loader_order(N)
            orders[k, 1] = _loader_order(N)
        t = run.adam.t
        sched = torch.tensor([run.adam.sched_values(t + 1 + i) for i in range(K * nb)],
                             dtype=torch.float32).reshape(K, nb, 2)
        self.ord.copy_(orders.pin_memory(), non_blocking=True)
        self.sched.copy_(sched.pin_memory(), non_blocking=True)
        self.g.replay()
        run.adam.t = t + K * nb
        terms_dst.copy_(self.terms)


class TorchFlowCalibrator(Calibrator):
    """Trains a normalizing flow on (logits, target) by minimising
    -mean(log(softmax(f(x))[y] + 1e-7) + log|det J_f(x)|)  (calibrators.py:239-353)."""

    def __init__(self, Flow, logits, target, **kwargs):
        super().__init__(logits, target)
        self.target = np.argmax(self.target, axis=1)
        self.logits = torch.as_tensor(self.logits, dtype=torch.float)
        self.target = torch.as_tensor(self.target, dtype=torch.long)
        self.flow = Flow(self.n_classes, **kwargs)
        self.dev = kwargs.get('dev', torch.device("cuda") if torch.cuda.is_available()
                              else torch.device("cpu"))
        self.CE = nn.CrossEntropyLoss()
        self.optimizer = torch.optim.Adam(self.flow.parameters())
        self._replica = None
        self._lp_dev = None
        # native fit: replay chunks of epochs as HIP graphs (False: eager epochs)
        self._graph_ok = bool(kwargs.get('cnf_graph', True))
        self.history = self.fit(self.logits, self.target,
                                epochs=kwargs.get('epochs', 1000),
                                batch_size=kwargs.get('batch_size', logits.shape[0]))

    # ------------------------------------------------------------------ fit
    def fit(self, logits, target, epochs, batch_size):
        logits = logits.to(self.dev)
        target = target.to(self.dev)
        self.flow.to(self.dev)
        stack = _native_stack(self.flow, self.dev)
        if stack is not None:
            # the captured epochs launch on the CURRENT device's stream: make
            # that the calibrator's `dev`, which need not be the current GPU
            with torch.cuda.device(logits.device):
                history = self._fit_native(stack, logits, target, epochs, batch_size)
        else:
            history = self._fit_torch(logits, target, epochs, batch_size)
        self.flow.cpu()
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
        return history

    def _fit_torch(self, logits, target, epochs, batch_size):
        """The reference's loop (calibrators.py:273-317), unchanged semantics."""
        train_dl = DataLoader(TensorDataset(logits, target), batch_size=batch_size, shuffle=True)
        history = {'loss': [], 'ce': [], 'log_det': []}
        softmx = nn.Softmax(dim=1)
        for epoch in range(epochs):
            self.flow.train()
            for xb, yb in train_dl:
                pred, log_det = self.flow(xb)
                probs = softmx(pred)
                ce = torch.log(probs.gather(1, yb.view(-1, 1)) + 1e-7)
                loss = -torch.mean(ce.squeeze() + log_det)
                self.flow.zero_grad()
                loss.backward()
                self.optimizer.step()
            self.flow.eval()
            _loss = _ce = _log_det = 0
            num = 0
            with torch.no_grad():
                for xb, yb in train_dl:
                    pred, log_det = self.flow(xb)
                    probs = softmx(pred)
                    ce = torch.log(probs.gather(1, yb.view(-1, 1)) + 1e-7)
                    log_prob = ce.squeeze() + log_det
                    # the reference ASSIGNS per batch (calibrators.py:308-313): the
                    # history keeps the last batch's sums over the total count
                    _loss = -torch.mean(log_prob) * len(xb)
                    _ce = -torch.mean(ce.squeeze()) * len(xb)
                    _log_det = torch.mean(log_det) * len(xb)
                    num += len(xb)
                history['loss'].append(_loss / num)
                history['ce'].append(_ce / num)
                history['log_det'].append(_log_det / num)
        return history

    def _fit_native(self, stack, logits, target, epochs, batch_size):
        """Same schedule on the fused kernels: one cnf_loss_vjp launch plus one
        cnf_adam_step launch per training batch, one cnf_forward_loss launch per
        evaluation batch.  Each pass over the data draws its order exactly as
        the reference's DataLoader(shuffle=True) does (_loader_order), so
        minibatch runs see the reference's batches and the eval history keeps
        the reference's last-batch value (calibrators.py:274-317).

        After one eager epoch, chunks of epochs run as ONE captured HIP graph
        each (_EpochGraph): the chunk's orders and Adam step scalars are staged
        with one host-to-device copy, so the host issues three operations per
        chunk instead of ~10 launches per epoch.  kwargs cnf_graph=False keeps
        every epoch eager."""
        from cnf_hip.adam import StackAdam
        adam = StackAdam.like(stack, self.optimizer)
        N = logits.shape[0]
        bs = max(1, int(batch_size))
        terms_all = torch.empty(max(epochs, 1), 3, dtype=torch.float32, device=logits.device)
        run = _EpochRunner(stack, adam, logits, target, bs)
        e = 0
        if epochs > 0:  # the eager first epoch also builds every cached buffer
            run.eager_epoch(terms_all[0])
            e = 1
        if self._graph_ok and epochs - e >= 2:
            g = _EpochGraph(run, min(epochs - e, _EpochGraph.CHUNK))
            while epochs - e >= g.K:
                g.replay(terms_all[e:e + g.K])
                e += g.K
        while e < epochs:
            run.eager_epoch(terms_all[e])
            e += 1
        adam.store_into(self.optimizer)
        stack.invalidate()  # drop blobs / workspaces captured into a graph pool
        hist = terms_all[:epochs] / N
        return {'loss': list(hist[:, 0].unbind(0)), 'ce': list(hist[:, 1].unbind(0)),
                'log_det': list(hist[:, 2].unbind(0))}

    # -------------------------------------------------------------- predict
    def _device_flow(self):
        """A device-resident replica of the (CPU) flow, refreshed only when a
        parameter changed -- the reference moves the flow to the device and
        back on every call (calibrators.py:335-343)."""
        import copy
        key = tuple((p.data_ptr(), p._version) for p in self.flow.parameters())
        if self._replica is None or self._replica[0] != key:
            rep = copy.deepcopy(self.flow).to(self.dev)
            rep.eval()
            self._replica = (key, rep)
        return self._replica[1]

    def predict(self, logits):
        """Calibrator.predict (calibrators.py:40-44 with predict_post, :330-353):
        centring, the flow, softmax and the prior correction
        softmax(log(p + 1e-7) - log_priors).  On a ROCm device this is ONE fused
        launch (cnf_predict) on a resident replica of the flow, with one H2D
        copy of the logits and one D2H copy of the probabilities."""
        if torch.device(self.dev).type == "cuda":
            flow = self._device_flow()
            stack = _native_stack(flow, self.dev, need_vjp=False)
            if stack is not None:
                x = torch.as_tensor(np.asarray(logits), dtype=torch.float).to(self.dev)
                if self._lp_dev is None:
                    self._lp_dev = torch.as_tensor(self.log_priors, dtype=torch.float,
                                                   device=self.dev)
                with torch.no_grad():
                    probs = stack.predict(x, self._lp_dev)
                return probs.cpu().numpy().astype(np.float64)
        return super().predict(logits)

    def predict_logits(self, logits):
        logits = torch.as_tensor(logits, dtype=torch.float)
        if torch.device(self.dev).type == "cuda":
            flow = self._device_flow()
            with torch.no_grad():
                preds, _ = flow(logits.to(self.dev))
            return preds.cpu().numpy()
        self.flow.to(self.dev)
        preds, _ = self.flow(logits.to(self.dev))
        return preds.cpu().detach().numpy()

    def predict_post(self, logits):
        logits = self.predict_logits(logits)
        return softmax(logits, axis=1)
