"""The timed training step of the reference (``trainer.py:109-162``) on the HIP path.

One ``Trainer.step(X, y)`` = ``sess.run([train_op, update_range_op])`` of ``trainer.py:157``:
forward, loss, manual backward, ``MomentumOptimizer.apply_gradients`` (``acc = mu*acc + g;
w -= lr*acc``, ``trainer.py:79-84``) and the ``'update_range'`` collection.

MI355X-native execution:
* all trainable variables live in ONE flat fp32 buffer (and their gradients / momentum in two
  more), so the optimiser is a single kernel and the data-parallel exchange is one all-reduce;
* after a warm-up step the whole step is captured into a HIP graph (``torch.cuda.CUDAGraph``)
  and replayed: ~300 kernel launches become one graph launch;
* data parallelism (``torch.distributed``, backend ``nccl`` = RCCL over xGMI): each rank runs
  the step on its own batch shard, with the loss a mean over the GLOBAL batch; between the
  backward graph and the update graph ONE all-reduce sums the step's gradients and the
  quantisers' overflow counters, so every rank applies identical updates and identical DFXP
  exponents. Noise keys (seed, step, quantiser) do not depend on the rank.
  - fused plans (FusedResNet): the gradients travel as their exact int64 numerators (the
    quantised-gradient exchange, lbt_step_reduce_x -> all-reduce -> lbt_step_finish): exact and
    order-independent, so the update is the single-process formula applied to the global sums;
    with ``FusedResNet(sync_bn=True)`` (global BatchNorm statistics) a step on N ranks of b
    samples is bit-identical to one process on the N*b batch.
  - layer-wise models: dequantised fp32 gradients + counters folded into exact fp32 pairs, one
    fp32 all-reduce (gscale = 1/world).
"""
import os
import sys

import torch
import torch.distributed as dist

from . import _lib
from . import distributed as D
from .dfxp import ops


class FlatParams:
    """Bind every (var, grad) of a model into contiguous flat buffers (grads_and_vars order)."""

    def __init__(self, model, grad_buffer=None):
        slots = model.param_slots()
        dev = model.ctx.device
        sizes = [getattr(o, v).numel() for o, v, _ in slots]
        n = sum(sizes)
        self.n = n
        self.w = torch.zeros(n, dtype=torch.float32, device=dev)
        self.g = grad_buffer[:n] if grad_buffer is not None else torch.zeros(n, dtype=torch.float32, device=dev)
        self.a = torch.zeros(n, dtype=torch.float32, device=dev)
        off = 0
        self.offsets = []
        for (o, v, gname), sz in zip(slots, sizes):
            t = getattr(o, v)
            wv = self.w[off:off + sz].view(t.shape)
            wv.copy_(t)
            setattr(o, v, wv)
            setattr(o, gname, self.g[off:off + sz].view(t.shape))
            self.offsets.append((o, v, off, sz))
            off += sz


class Trainer:
    def __init__(self, model, dataset=None, logger=None, logdir=None, lr=1e-2, lr_decay_factor=0.5,
                 lr_decay_epoch=50, momentum=0.95, n_epoch=5, batch_size=128, use_graph=True,
                 process_group=None, exchange=None, capture_comm=None):
        """exchange: run the data-parallel exchange (default: when the process group has > 1 rank;
        True at world 1 exercises the same path -- an all-reduce over one rank is the identity).
        capture_comm: put the step's collectives (the exchange, SyncBN's statistics) INSIDE the
        captured HIP graph, so a step is one graph launch (default: on for the nccl = RCCL backend,
        LBT_CAPTURE_COMM=0 turns it off; gloo collectives cannot be captured and run from the host
        between graph segments / eagerly)."""
        self.model = model
        self.dataset = dataset
        self.logger = logger
        self.lr, self.momentum = lr, momentum
        self.lr_decay_factor, self.lr_decay_epoch = lr_decay_factor, lr_decay_epoch
        self.n_epoch, self.batch_size = n_epoch, batch_size
        self.use_graph = use_graph
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if (dist.is_available() and dist.is_initialized()) else 1
        self.ctx = model.ctx
        if self.world != self.ctx.world_size:
            raise ValueError("DfxpContext.world_size (%d) must equal the process-group size (%d)"
                             % (self.ctx.world_size, self.world))
        # data-parallel exchange: int64 [numerators | counters | loss] (fused plans) or fp32
        # [grads | folded overflow counters] (layer-wise models) -> ONE in-place all-reduce per step
        self.comm = self.xbuf = None
        dist_on = dist.is_available() and dist.is_initialized()
        self.dp = (self.world > 1) if exchange is None else (bool(exchange) and dist_on)
        if capture_comm is None:
            capture_comm = (dist_on and dist.get_backend(process_group) == "nccl"
                            and os.environ.get("LBT_CAPTURE_COMM", "1") == "1")
        self.capture_comm = bool(capture_comm) and dist_on
        exact = self.dp and hasattr(model, "set_exchange")
        # layer-wise models (ResNet-50, configs[3]): the same exact int64 exchange when every gradient
        # is an integer numerator (integer-coded W / gamma / beta only; LBT_EXACT_LAYERWISE=0: fp32)
        self._lw_exact = (self.dp and not exact and D.exact_layerwise_ok(model)
                          and os.environ.get("LBT_EXACT_LAYERWISE", "1") == "1")
        if self.dp and not exact and not self._lw_exact:
            n = sum(getattr(o, v).numel() for o, v, _ in model.param_slots())
            self.comm = D.make_comm_buffer(n, len(self.ctx.quantizers), self.ctx.device)
        self.flat = FlatParams(model, self.comm)
        self._loss_n = 0
        if exact:
            self._setup_exchange()
        elif self._lw_exact:
            self._setup_exchange_layerwise()
        self.ctx.sums_managed = True
        # single process, fused plan: the optimiser + range update run inside the step's last launch
        # (FusedResNet.set_optimizer / lbt_step_reduce_update) instead of one more launch after it
        self._fused_update = hasattr(model, "set_optimizer") and not self.dp
        self._sync_optimizer()
        self.global_step = 0
        self._graphs = None
        self._static = None
        self._gcache = {}  # (X ptr, y ptr, shape) -> captured graphs (models that bind inputs)
        self._eval = {}
        self._plans = {}
        self._active = model
        self._aug = None
        if logger is not None:
            logger.info("Model info:\n" + model.info())

    def _setup_exchange(self):
        """The exact exchange of a fused plan: buffer, descriptor, and the finish kernel's segments."""
        m, ctx, flat = self.model, self.ctx, self.flat
        Q = len(ctx.quantizers)
        self.xbuf, x = D.make_exchange(flat.n, Q, ctx.device)
        x.gbase = flat.g.data_ptr()
        rank = dist.get_rank(self.pg)
        # SyncBN: the gamma / beta numerators come from pass-A sums that are already global
        x.pjob_scale = 1 if (not getattr(m, "sync_bn", False) or rank == 0) else 0
        x.counts = ctx.counts.data_ptr()
        self._xchg = x
        m.set_exchange(x)
        self._segs, self._seg_blocks = D.finish_segments(flat, ctx.device)

    def _setup_exchange_layerwise(self):
        """The exact exchange of a layer-wise model: every gradient reduction writes its integer
        numerator into the exchange buffer (ops.set_exchange_sink during the step), the counters are
        folded in by lbt_step_reduce_x's fold blocks; all-reduce, lbt_step_finish, range update."""
        ctx, flat = self.ctx, self.flat
        self.xbuf, x = D.make_exchange(flat.n, len(ctx.quantizers), ctx.device)
        x.gbase = flat.g.data_ptr()
        x.counts = ctx.counts.data_ptr()
        x.pjob_scale = 1
        self._xchg = x
        self._segs, self._seg_blocks = D.finish_segments(flat, ctx.device)

    def _sync_optimizer(self):
        """Hand the current lr / momentum and the flat buffers to every fused plan that applies the
        update itself (read when a step is captured or run eagerly)."""
        if self._fused_update:
            for p in [self.model] + list(getattr(self, "_plans", {}).values()):
                p.set_optimizer(self.flat, self.lr, self.momentum)

    # -- the reference's API ---------------------------------------------------------------
    def init_model(self):
        self.flat.a.zero_()

    def get_train_op(self):
        """Rebuilding MomentumOptimizer resets its accumulators (trainer.py:79-84)."""
        self.flat.a.zero_()
        self._graphs = None  # lr is baked into the captured optimiser kernel
        self._gcache = {}
        self._sync_optimizer()
        return self.step

    # -- the step ----------------------------------------------------------------------------
    def _plan(self, N):
        """The execution plan for a batch of N: a fused plan is built for one batch shape, so another
        N (the epoch's final partial batch, trainer.py:98) gets a plan of its own over the same
        layers, parameters and quantisers."""
        m = self.model
        if not hasattr(m, "set_exchange") or m._shape is None or m._shape[0] == N:
            return m
        p = self._plans.get(N)
        if p is None:
            from .fused import FusedResNet
            p = FusedResNet(m.model, sync_bn=m.sync_bn, process_group=m.pg, force_sync_bn=m.sync_bn)
            if self.xbuf is not None:
                p.set_exchange(self._xchg)
            if self._fused_update:
                p.set_optimizer(self.flat, self.lr, self.momentum)
            self._plans[N] = p
            # graphs captured while this was the only plan hold no per-step element-count copy
            # (_fwd_bwd adds one only once several plans exist): re-capture them with it, or they
            # would replay with the new plan's overflow-rate denominators
            self._gcache = {}
            self._graphs = None
        return p

    def _fwd_bwd(self, X, y, update=False):
        """The step's forward + backward; update=True lets a fused plan apply the optimiser and the range
        update in its last launch. Returns whether it did (then _update must not run)."""
        m = self._active = self._plan(X.shape[0])
        did = False
        nel = getattr(m, "_nelem", None)
        if nel is not None and self._plans:  # several plans: this one's per-step element counts
            self.ctx.nelem.copy_(nel)
        if not getattr(m, "zeroes_own_sums", False):
            self.ctx.zero_sums()
        if hasattr(m, "train_fwd_bwd"):
            did = bool(m.train_fwd_bwd(X, y, update=update and self._fused_update))
        elif self._lw_exact:
            x = self._xchg
            self._loss_n = int(X.shape[0]) * self.world
            ops.set_exchange_sink(self.flat.g, self.flat.n, self.xbuf, x.loss_off, self.world)
            try:
                m.forward(X)
                m.compute_loss(y)
                m.backward()
            finally:
                ops.set_exchange_sink()
            # the overflow counters into the buffer (lbt_step_reduce_x with its fold blocks only)
            _lib.call("lbt_step_reduce_x", None, 0, 0, None, 0, 0, None, _lib.ctypes.byref(x), _lib.stream())
        else:
            m.forward(X)
            m.compute_loss(y)
            with ops.deferred_reductions():  # the backward's wgrad reduces / BN parameter grads: two launches at the end
                m.backward()
        if nel is None and hasattr(m, "set_exchange"):
            m._nelem = self.ctx.nelem.clone()  # what its build declared (Quantizer.observe)
        if self.comm is not None:
            self.ctx.fold_counts(self.comm[self.flat.n:])
        return did

    def _exchange(self):
        """Sum the step's gradients + overflow counters across ranks (one RCCL all-reduce;
        lbt_amd/distributed.py)."""
        D.allreduce_comm(self.xbuf if self.xbuf is not None else self.comm, self.pg)

    def _update(self):
        if self.xbuf is not None:  # exact exchange: dequantise the global sums, SGD, range update
            ctx, f = self.ctx, self.flat
            x = self._xchg
            _lib.call("lbt_step_finish", _lib.ptr(self._segs), len(self._segs) // _lib.ctypes.sizeof(_lib.FSeg),
                      self._seg_blocks, _lib.ptr(self.xbuf), _lib.ptr(f.w), _lib.ptr(f.a), _lib.ptr(f.g),
                      float(self.lr), float(self.momentum), _lib.ptr(self._active.loss), x.loss_off,
                      self._loss_n if self._lw_exact else int(self._active._head.loss_n), _lib.stream())
            _lib.call("lbt_dfxp_range_update_x", _lib.ptr(ctx.exps), _lib.ptr(self.xbuf), x.cnt_off,
                      _lib.ptr(ctx.bits), _lib.ptr(ctx.target), _lib.ptr(ctx.nelem), len(ctx.quantizers),
                      _lib.ptr(ctx.step), _lib.stream())
        elif self.comm is not None:
            ops.sgd_momentum(self.flat.w, self.flat.a, self.flat.g, self.lr, self.momentum, 1.0 / self.world)
            self.ctx.update_range_folded_op(self.comm[self.flat.n:])
        else:  # optimiser + range update in one launch
            self.ctx.update_range_op(sgd=(self.flat.w, self.flat.a, self.flat.g, self.lr, self.momentum, 1.0))

    def _eager(self, X, y):
        self._sync_optimizer()  # an assignment to self.lr / self.momentum takes effect on the fused update too
        did = self._fwd_bwd(X, y, update=not self.dp)
        if self.dp:
            self._exchange()
        if not did:
            self._update()

    def _warmup(self, X, y):
        """One un-captured forward + backward that allocates every per-layer buffer before a capture.
        Its side effects are undone: the overflow counters (no update is applied) and the BN running
        statistics (the reference moves them once per step, dynamic_fixed_point.py:601-612)."""
        saved = [(bn.X_mean_running.clone(), bn.X_var_running.clone()) for bn in self._bn_layers()]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._fwd_bwd(X, y)
            if self.dp and self.capture_comm:
                # a collective must have run once (communicator set up) before one is captured; the
                # exchange buffer is rewritten by the next step's backward
                self._exchange()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.ctx.counts.zero_()
        for bn, (m, v) in zip(self._bn_layers(), saved):
            bn.X_mean_running.copy_(m)
            bn.X_var_running.copy_(v)

    def _capture(self, X, y):
        m = self.model
        if hasattr(m, "input_buffer") and hasattr(m, "label_buffer"):
            # capture on the model's own buffers: no copies inside the graph
            self._static = (m.input_buffer(X.shape), m.label_buffer(y.shape[0]))
        else:
            self._static = (torch.empty_like(X), torch.empty_like(y))
        sX, sy = self._static
        sX.copy_(X)
        sy.copy_(y)
        self._warmup(sX, sy)
        self._graphs = self._capture_step(sX, sy)

    def _comm_capturable(self):
        """Capture the exchange ALONE into a throwaway graph (never replayed) once: whether this RCCL /
        runtime supports the collective inside a HIP graph. Only this probe may fail over to the
        host-issued exchange; any error while capturing the step itself is raised as it is."""
        if getattr(self, "_comm_probe", None) is None:
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    self._exchange()
                self._comm_probe = True
            except RuntimeError:
                import traceback
                print("trainer: the collective cannot be captured in a HIP graph; the exchange runs from the "
                      "host between two graphs. The capture failed with:\n" + traceback.format_exc(),
                      file=sys.stderr)
                self._comm_probe = False
            del g
            torch.cuda.synchronize()
        return self._comm_probe

    def _capture_step(self, X, y):
        """(g1, g2): the step as one graph (no exchange, or captured collectives), else the forward +
        backward and the update as two graphs with the host-issued exchange between them. When the
        exchange cannot be captured (``_comm_capturable``) it runs from the host, loudly (not for SyncBN
        plans, whose statistics collectives sit inside the forward)."""
        if self.dp and self.capture_comm and not getattr(self.model, "sync_bn", False):
            if not self._comm_capturable():
                self.capture_comm = False
        return self._capture_step_once(X, y)

    def _capture_step_once(self, X, y):
        one = not self.dp or self.capture_comm
        # thread-local capture: the process group's watchdog thread queries events meanwhile
        mode = "thread_local" if self.capture_comm else "global"
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1, capture_error_mode=mode):
            did = self._fwd_bwd(X, y, update=not self.dp)
            if one:
                if self.dp:
                    self._exchange()
                if not did:
                    self._update()
        g2 = None
        if not one:
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2):
                self._update()
        return g1, g2

    def _capture_bound(self, X, y):
        """Capture the step reading (X, y) in place (models with binds_inputs): one graph per batch
        buffer pair, the first capture after a warm-up that allocates every per-layer buffer."""
        if getattr(self._plan(X.shape[0]), "_shape", 0) is None or not self._gcache:
            self._warmup(X, y)  # every plan's first run allocates its buffers outside a capture
        return self._capture_step(X, y)

    def prepare(self, X, y):
        """Build (capture) the step's graph for this batch buffer pair without running a step -- setup
        before a timed loop, so that no capture lands inside it whatever the warm-up count (a loader's
        ring of batch buffers gets one graph per buffer, on its first step otherwise)."""
        self._active = self._plan(X.shape[0])
        if not self.use_graph or (getattr(self.model, "sync_bn", False) and not self.capture_comm):
            return
        key = (X.data_ptr(), y.data_ptr(), tuple(X.shape))
        if getattr(self.model, "binds_inputs", False):
            if key not in self._gcache and len(self._gcache) < 8:
                self._gcache[key] = self._capture_bound(X, y)
        elif self._graphs is None or self._static is None or self._static[0].shape != X.shape:
            self._capture(X, y)

    def step(self, X, y):
        """One training step on batch (X [B,32,32,3] fp32 NHWC, y [B] int32), device tensors.
        A SyncBN plan holds collectives inside the step: captured with them (RCCL), else eager."""
        self._active = self._plan(X.shape[0])
        if not self.use_graph or (getattr(self.model, "sync_bn", False) and not self.capture_comm):
            self._eager(X, y)
        else:
            key = (X.data_ptr(), y.data_ptr(), tuple(X.shape))
            if getattr(self.model, "binds_inputs", False) and (key in self._gcache or len(self._gcache) < 8):
                # the batch is read where it lies: a graph per buffer pair (a loader's ring of
                # batch buffers), no copy into static inputs inside the timed step
                if key not in self._gcache:
                    self._gcache[key] = self._capture_bound(X, y)
                self._graphs = self._gcache[key]
            elif self._graphs is None or self._static is None or self._static[0].shape != X.shape:
                self._capture(X, y)
            else:
                self._static[0].copy_(X)
                self._static[1].copy_(y)
            g1, g2 = self._graphs
            g1.replay()
            if g2 is not None:
                self._exchange()
                g2.replay()
        self.global_step += 1
        return self._active.loss

    def train(self, augment=True):
        """Epoch loop of trainer.py:117-192 over an in-memory dataset ((Xtr, ytr), (Xte, yte)):
        shuffled batches, preprocess_image on device (random flip + pad-4 random crop,
        lbt_augment_flip_crop), the lr schedule of :122-140, and the test loop after every epoch.
        Returns the per-epoch test accuracies."""
        (Xtr, ytr), (Xte, yte) = self.dataset
        dev = self.ctx.device
        history = []
        for epoch in range(self.n_epoch):
            if epoch == 0:
                self.get_train_op()
            elif epoch in (80, 120, 140):
                self.lr *= self.lr_decay_factor
                self.get_train_op()
            perm = torch.randperm(len(Xtr))
            self.batch_sizes = []
            for b in range(0, len(Xtr), self.batch_size):  # the final partial batch too (trainer.py:98)
                idx = perm[b:b + self.batch_size]
                X = torch.as_tensor(Xtr[idx.numpy()], dtype=torch.float32).to(dev).contiguous()
                y = torch.as_tensor(ytr[idx.numpy()], dtype=torch.int32).to(dev)
                if augment:
                    if self._aug is None or self._aug.shape != X.shape:
                        self._aug = torch.empty_like(X)
                    X = ops.augment_flip_crop(X, 4, self.ctx.seed, self.global_step, out=self._aug)
                loss = self.step(X, y)
                self.batch_sizes.append(len(idx))
                if self.logger is not None and (b // self.batch_size + 1) % 100 == 0:
                    self.logger.info("Batch %d loss %f" % (b // self.batch_size + 1, loss.item()))
            if Xte is not None and len(Xte):
                acc, _ = self.evaluate(Xte, yte)
                history.append(acc)
                if self.logger is not None:
                    self.logger.info("Epoch %d test accuracy %f" % (epoch + 1, acc))
        return history

    # -- test loop and checkpoint (trainer.py:164-197) ----------------------------------------
    def _eval_model(self, n):
        """The model the test loop runs for a batch of n: a FusedResNet gets a plan of its own per
        test-batch size (its own buffers, so the captured training graph stays valid); a
        layer-wise model is shared (its per-layer buffers are re-sized by the test batch, so the
        training graph is re-captured afterwards)."""
        from .fused import FusedResNet
        m = self.model
        if isinstance(m, FusedResNet):
            if n not in self._eval:
                self._eval[n] = FusedResNet(m.model)
            return self._eval[n], False
        return m, True

    def evaluate(self, X, y, batch_size=1000):
        """The reference's test loop (trainer.py:166-190): per batch of 1000 the forward pass in
        training mode (batch-statistic BN, stochastic quantisers -- the reference never runs
        set_testing, :164-165), loss and accuracy; returns (mean accuracy, mean loss) over the
        batches. The overflow counters these forwards accumulate are discarded (the loop does not
        fetch update_range_op); BN running statistics are updated, as the reference's are."""
        dev = self.ctx.device
        saved = self.ctx.counts.clone()
        saved_nelem = self.ctx.nelem.clone()  # an eval plan's build declares its own element counts
        acc_sum, loss_sum, nb, shared = 0.0, 0.0, 0, False
        for b in range(0, len(X), batch_size):
            Xb = torch.as_tensor(X[b:b + batch_size], dtype=torch.float32).to(dev).contiguous()
            yb = torch.as_tensor(y[b:b + batch_size], dtype=torch.int32).to(dev)
            m, shared = self._eval_model(len(Xb))
            logits = m.forward(Xb)
            loss = m.compute_loss(yb)
            acc = (logits.argmax(dim=1).to(torch.int32) == yb).float().mean()
            acc_sum += float(acc.item())
            loss_sum += float(loss.item())
            nb += 1
        self.ctx.counts.copy_(saved)
        self.ctx.nelem.copy_(saved_nelem)
        # the quantisers' cached counts now describe the eval plan, not ctx.nelem: forget them so
        # the next plan build writes its own (Quantizer.observe skips a write that matches its cache)
        for q in self.ctx.quantizers:
            q._nelem = None
        if shared:
            self._graphs = None
        return acc_sum / max(nb, 1), loss_sum / max(nb, 1)

    def _bn_layers(self):
        out = []

        def walk(layers):
            for layer in layers:
                if hasattr(layer, "X_mean_running"):
                    out.append(layer)
                for attr in ("layers", "residual", "shortcut"):
                    sub = getattr(layer, attr, None)
                    if sub is None:
                        continue
                    walk(sub.layers if hasattr(sub, "layers") and not isinstance(sub, (list, tuple)) else sub)
        root = getattr(self.model, "model", self.model)
        walk(root.layers)
        return out

    def save_model(self, exp_path):
        """Checkpoint (trainer.py:189-192, tf.train.Saver): parameters, momentum accumulators, DFXP
        exponents + noise step, BN running statistics and the trainer's step / lr, as one
        safetensors file exp_path/model.safetensors (no pickled objects)."""
        import json
        import os

        from safetensors.torch import save_file
        os.makedirs(exp_path, exist_ok=True)
        t = {"w": self.flat.w, "a": self.flat.a, "exps": self.ctx.exps, "step": self.ctx.step}
        for i, bn in enumerate(self._bn_layers()):
            t["bn%d/mean" % i] = bn.X_mean_running
            t["bn%d/var" % i] = bn.X_var_running
        meta = {"global_step": str(self.global_step), "lr": repr(self.lr), "momentum": repr(self.momentum),
                "quantizers": json.dumps([q.name for q in self.ctx.quantizers]),
                "params": json.dumps([[o.name if hasattr(o, "name") else "", v, off, sz]
                                      for o, v, off, sz in self.flat.offsets])}
        path = os.path.join(exp_path, "model.safetensors")
        save_file({k: v.detach().contiguous().cpu() for k, v in t.items()}, path, metadata=meta)
        return path

    def load_model(self, path):
        """Restore a save_model checkpoint into this trainer (same model layout)."""
        import json

        from safetensors import safe_open
        with safe_open(path, framework="pt") as f:
            meta = f.metadata()
            if json.loads(meta["quantizers"]) != [q.name for q in self.ctx.quantizers]:
                raise ValueError("checkpoint quantiser layout differs from this model's")
            self.flat.w.copy_(f.get_tensor("w"))
            self.flat.a.copy_(f.get_tensor("a"))
            self.ctx.exps.copy_(f.get_tensor("exps"))
            self.ctx.step.copy_(f.get_tensor("step"))
            for i, bn in enumerate(self._bn_layers()):
                bn.X_mean_running.copy_(f.get_tensor("bn%d/mean" % i))
                bn.X_var_running.copy_(f.get_tensor("bn%d/var" % i))
        self.global_step = int(meta["global_step"])
        self.lr = float(meta["lr"])
        self.momentum = float(meta["momentum"])
        self._graphs = None  # lr is baked into the captured optimiser
        self._gcache = {}
        self._sync_optimizer()
