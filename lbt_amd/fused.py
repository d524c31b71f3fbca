"""Fused execution plan of a ``CIFAR10_Resnet`` -- the MI355X-native hot path.

Same parameters, quantisers (names, noise streams, exponents) and arithmetic as executing the
model layer by layer through the Layer_q API, so the results are BIT-IDENTICAL (tested); only
the kernel schedule changes. Per residual block the reference's 13 layer calls
(conv, BN-norm, BN-rescale, ReLU, conv, BN-norm, BN-rescale, [conv, BN-norm, BN-rescale], add,
ReLU) become 4-5 kernels forward and 8-11 backward:

forward   conv-1 (int8 MFMA, epilogue = bn1-norm quantiser + exact channel sums)
          chain  (bn1 moments -> normalise -> rescale quantiser -> affine -> ReLU -> conv-2 input quantiser)
          conv-2 (epilogue = bn2-norm quantiser + sums)            [+ 1x1 shortcut conv, same epilogue]
          chain  (bn2 [+ shortcut BN] + residual -> ReLU -> block output + next block's input quantisers)
backward  chain A (ReLU mask, bn2-rescale grad quantiser, dgamma/dbeta sums, bn2-norm grad quantiser)
          chain B (bn2-norm backward -> conv-2 grad quantiser + column sums)     [+ shortcut BN]
          conv-2 dgrad, conv-2 wgrad, chain A/B for bn1, [shortcut dgrad], conv-1 dgrad (+ residual
          gradient), conv-1 wgrad [+ shortcut wgrad]
and all weight / gamma / beta quantisers, all split wgrad reductions and all dgamma / dbeta are one
batched launch each. Every launch is prebuilt (ctypes arguments fixed) on the first call, so a
step is a flat list of C calls -- and one HIP graph once captured by the Trainer.
"""
import ctypes
import math
import os

import torch

from . import _lib
from ._lib import NO_Q, OUT_I8, OUT_I16, OUT_U8OFF, BnNorm, BwdBranch, ChainBwdA, ChainBwdB, ChainFwd, ConvBwd, \
    ConvFwd, NJob, PJob, QJob, RJob, WgradJob, WJob, call, ptr
from .dfxp import ops
from .dfxp.layers import _Cache


def _desc(q):
    return q.desc


def _dev_array(jobs, device):
    """Upload an array of ctypes job structs to device memory (kept alive by the returned tensor)."""
    n = len(jobs)
    T = type(jobs[0])
    buf = (T * n)(*jobs)
    host = torch.frombuffer(bytearray(bytes(buf)), dtype=torch.uint8)
    return host.to(device)


class _Block:
    def __init__(self, blk):
        r = blk.residual.layers
        self.c1, self.n1, self.r1 = r[0], r[1].layers[0], r[1].layers[1]
        self.c2, self.n2, self.r2 = r[3], r[4].layers[0], r[4].layers[1]
        sc = blk.shortcut.layers
        if sc:
            self.cs, self.ns, self.rs = sc[0], sc[1].layers[0], sc[1].layers[1]
        else:
            self.cs = self.ns = self.rs = None
        self.blk = blk


class FusedResNet:
    """Drop-in for the Trainer (forward / compute_loss / backward / param_slots / ctx / loss)."""

    def __init__(self, model, sync_bn=False, process_group=None, force_sync_bn=False):
        """sync_bn: data-parallel parity mode -- every BatchNorm takes its moments (forward) and its
        pass-A sums (backward) over the GLOBAL batch: the per-rank integer sums are all-reduced
        (exact) before the kernel that consumes them, so N ranks of b samples compute what one
        process computes on the N*b batch (tf.nn.moments over the whole batch,
        dynamic_fixed_point.py:588). The step then holds collectives: the Trainer captures them into
        its HIP graph (RCCL) or runs the step eagerly (gloo).
        force_sync_bn: keep the collectives at world size 1 (tests of the captured path: a sum over
        one rank is the identity, so the step must equal the plain plan bit for bit)."""
        self.model = model
        self.ctx = model.ctx
        self.sync_bn = bool(sync_bn) and (self.ctx.world_size > 1 or bool(force_sync_bn))
        self.pg = process_group
        self.xchg = None  # data-parallel exchange descriptor (Trainer.set_exchange)
        L = model.layers
        self.conv1, bn0 = L[0], L[1]
        self.n0, self.r0 = bn0.layers[0], bn0.layers[1]
        self.blocks = [_Block(b) for b in L[3:-3]]
        self.dense = L[-1]
        self.convs = [self.conv1] + [c for b in self.blocks for c in (b.c1, b.c2, b.cs) if c is not None]
        self.rescales = [self.r0] + [r for b in self.blocks for r in (b.r1, b.r2, b.rs) if r is not None]
        self._c = _Cache()
        self._shape = None
        self.loss = None
        self.dlogits = None
        self.overlap_wgrad = os.environ.get("LBT_OVERLAP_WGRAD", "0") == "1"  # measured: a loss here (60K vs 67K samples/s)
        # run each BN backward pass A inside the dgrad that produces its input (1 = default)
        self.fuse_dgrad_chain = os.environ.get("LBT_FUSE_DGRAD_CHAIN", "1") == "1"
        # a conv's wgrad launched together with its dgrad (+ pass A): one launch per conv, not two
        self.fuse_wgrad = os.environ.get("LBT_FUSE_WGRAD", "1") == "1" and not self.overlap_wgrad
        # stride-1 3x3 convs: pass B + dgrad + pass A in one launch (lbt_conv_bwd_fused_i8), each
        # conv's wgrad deferred into the next such launch (1 = default)
        self.fuse_bwd = (os.environ.get("LBT_FUSE_BWD", "1") == "1" and self.fuse_dgrad_chain and self.fuse_wgrad)
        self._pending = None  # the deferred wgrad job (lbt_wgrad_job) of the last fused backward launch
        # stride-1 3x3 convs: the BN chain producing the input runs in the conv launch (lbt_conv_fwd_fused_i8)
        self.fuse_fwd = os.environ.get("LBT_FUSE_FWD", "1") == "1"
        self._chain_pending = None  # a forward chain not launched yet (the next conv may absorb it)
        # fused backward: each conv's wgrad on the side stream (a parallel graph branch) instead of
        # deferred into the next conv's launch
        # (measured a loss: 0.78 -> 1.02 ms per step -- graph branches do not overlap here)
        self.side_wgrad = os.environ.get("LBT_SIDE_WGRAD", "0") == "1"
        # the end-of-backward batched wgrad launch as a parallel graph branch beside the stem's pass B
        # and weight gradient (independent until the final reduction). Measured a loss: 0.65 -> 0.71
        # ms/step (a forked HIP graph pays more in inter-stream synchronisation than the overlap wins)
        self.tail_fork = os.environ.get("LBT_TAIL_FORK", "0") == "1"
        # a projection block's two strided convs (3x3/2 + 1x1/2 shortcut) as ONE launch forward, and
        # its two pass-B chains (shortcut BN, first BN) as ONE launch backward
        self.pair_launch = os.environ.get("LBT_PAIR", "1") == "1"
        # the last block's output BN pass A inside the fused head launch (lbt_head.pa)
        self.head_pass_a = os.environ.get("LBT_HEAD_PASS_A", "1") == "1"
        # ... and that block's end chain (BN + Rescale_q + residual + ReLU) too (lbt_head.chain): the head
        # pools the block output from registers, one launch fewer per training step
        self.head_chain = os.environ.get("LBT_HEAD_CHAIN", "1") == "1"
        # the step prologue in two launches: noise tables + sums + input + conv1's weights ahead of the
        # stem, the other weight / gamma / beta quantisers on the side stream underneath it. Measured a
        # loss: 0.4288 -> 0.5060 ms/step (profiles/r10_prologue_split.txt; the forked graph again)
        self.prologue_split = os.environ.get("LBT_PROLOGUE_SPLIT", "0") == "1"
        self._side = None
        # every conv's weight gradient of the step in ONE launch at the end of the backward
        # (lbt_conv_wgrad_many_i8) instead of inside the dgrad launches: a dgrad launch's tiles fill
        # every workgroup slot of the chip, so wgrad workgroups in the same grid ran as extra rounds
        # ahead of them (measured per-workgroup: +6..10 us on each of 14 launches)
        self.batch_wgrad = (os.environ.get("LBT_BATCH_WGRAD", "1") == "1" and not self.overlap_wgrad
                            and not self.side_wgrad)
        self._wbatch = []  # the batched launch's jobs (lbt_wgrad_job), in backward order
        # with the batch on: a fused conv backward launch whose own tiles leave CU slots empty (fewer
        # than two workgroups per CU: the 64-channel stage at B = 128, every stage at small batches)
        # carries the previous such launch's wgrad job in those slots, as the unbatched plan does (the
        # job keeps the batched split, so a job no launch carries still joins the batch)
        self.defer_underfilled = os.environ.get("LBT_DEFER_UNDERFILLED", "0") == "1"
        # the optimiser and the range update inside the step's last launch (lbt_step_reduce_update;
        # single process): one launch fewer per step. Off until the Trainer hands over its flat
        # buffers and hyper-parameters (set_optimizer)
        self.fused_update = os.environ.get("LBT_FUSED_UPDATE", "1") == "1"
        self._upd = _lib.Update()
        self._upd_set = False

    # ------------------------------------------------------------------ Trainer interface
    def param_slots(self):
        return self.model.param_slots()

    def grads_and_vars(self):
        return self.model.grads_and_vars()

    def info(self):
        return "fused " + self.model.info()

    zeroes_own_sums = True  # the plan's first launch clears the sums arena

    def input_buffer(self, shape):
        """The plan's own input buffer (a caller may write batches straight into it)."""
        return self._c.get("X", tuple(shape), torch.float32, self.ctx.device)

    def label_buffer(self, n):
        return self._c.get("labels", (int(n),), torch.int32, self.ctx.device)

    binds_inputs = True  # the step reads the caller's batch buffers in place (Trainer caches a graph per pair)

    def _bind(self, X, labels=None):
        """Point the step's input launches at the caller's batch (no copy into the plan's own
        buffers): the prologue's image quantiser job and the fused head's labels. Buffers of
        another dtype / layout are copied into the plan's own first."""
        if X.dtype != torch.float32 or not X.is_contiguous() or X.device != self._X_own.device:
            self._X_own.copy_(X)
            X = self._X_own
        self._X = X
        self._input_job.x = X.data_ptr()
        if labels is not None:
            if labels.dtype != torch.int32 or not labels.is_contiguous():
                self._labels_own.copy_(labels)
                labels = self._labels_own
            self._head.labels = labels.data_ptr()

    def forward(self, X):
        self._ensure(X)
        self._bind(X)
        for f in self._fwd + self._hfwd:  # the first launch also zeroes the step's sums
            f()
        return self.logits

    def compute_loss(self, labels):
        if labels.data_ptr() != self._labels.data_ptr():  # the separate softmax-CE reads the own buffer
            self._labels.copy_(labels)
        for f in self._hloss:
            f()
        return self.loss

    def backward(self):
        if self.xchg is not None:
            raise NotImplementedError("the data-parallel exchange runs with the fused head (train_fwd_bwd)")
        for f in self._hbwd + self._bwd + self._tail_sep:
            f()

    def set_exchange(self, xchg):
        """Write the step's gradient numerators / counters / loss into the exchange buffer instead of
        dequantising them (lbt_step_reduce_x); set before the first step."""
        if self._shape is not None:
            raise RuntimeError("set_exchange after the plan was built")
        self.xchg = xchg

    def _allreduce(self, t):
        """A SyncBN collective inside the launch list: the exact int64 sum of t over the ranks."""
        import torch.distributed as dist
        pg = self.pg

        def run():
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=pg)
        run.kname = "allreduce"
        return run

    def set_optimizer(self, flat, lr, momentum):
        """MomentumOptimizer's flat buffers and hyper-parameters (trainer.py:79-84) for the fused update
        (train_fwd_bwd(update=True)); call again when lr changes, before the step is re-captured."""
        ctx = self.ctx
        u = self._upd
        u.w, u.a, u.g = flat.w.data_ptr(), flat.a.data_ptr(), flat.g.data_ptr()
        u.lr, u.mu = float(lr), float(momentum)
        u.exps, u.counts, u.bits = ctx.exps.data_ptr(), ctx.counts.data_ptr(), ctx.bits.data_ptr()
        u.target, u.nelem, u.step = ctx.target.data_ptr(), ctx.nelem.data_ptr(), ctx.step.data_ptr()
        u.nslots = len(ctx.quantizers)
        self._upd_set = True

    def updates_in_step(self):
        """Whether train_fwd_bwd(update=True) applies the optimiser and the range update itself."""
        return self.fused_update and self._upd_set and self.xchg is None

    def _flat_params(self):
        return [getattr(o, v) for o, v, _ in self.model.param_slots()]

    def step_tail(self, update):
        """The step's last launch: the reductions (+ the optimiser and the range update)."""
        return self._tail_upd if update and self.updates_in_step() else self._tail_fused

    def train_fwd_bwd(self, X, labels, update=False):
        """forward + compute_loss + backward of one training step, the head as one launch
        (lbt_head_fwd_bwd): same results bit for bit as the three calls. update=True (and
        updates_in_step()): the last launch also applies SGD-momentum and update_range (the Trainer's
        optimiser step, bit-identical). Returns whether it did."""
        self._ensure(X)
        self._bind(X, labels)
        tail = self.step_tail(update)
        for f in self._fwd + self._hfused + self._bwd + tail:
            f()
        return tail is not self._tail_fused

    # ------------------------------------------------------------------ streams
    def _on_side(self, run, force=False):
        """Run a launch on the side stream after everything already queued on the main stream
        (the weight-gradient GEMMs only feed the final reduction, so they overlap the serial
        dgrad -> BN-backward chain; under graph capture this becomes a parallel branch)."""
        if not (self.overlap_wgrad or force):
            return run

        def f():
            main = torch.cuda.current_stream()
            ev = torch.cuda.Event()
            ev.record(main)
            self._side.wait_event(ev)
            with torch.cuda.stream(self._side):
                run()
        f.kname, f.nbytes, f.inner = getattr(run, "kname", "side"), getattr(run, "nbytes", 0), run
        return f

    def _join_side(self):
        def f():
            ev = torch.cuda.Event()
            ev.record(self._side)
            torch.cuda.current_stream().wait_event(ev)
        f.kname = "join"
        return f

    # ------------------------------------------------------------------ plan
    def _buf(self, key, shape, dtype):
        return self._c.get(key, shape, dtype, self.ctx.device)

    def _sums(self, key, n):
        return self._c.sums(key, n, self.ctx)

    def _ensure(self, X):
        if self._shape == tuple(X.shape):
            return
        if self._shape is not None:
            raise RuntimeError("FusedResNet plan is built for one batch shape; got %s after %s"
                               % (tuple(X.shape), self._shape))
        self._shape = tuple(X.shape)
        self._build(X)

    def _build(self, X):
        if not getattr(self.model, "training", True):
            raise NotImplementedError("FusedResNet runs training-mode BatchNorm; use the layer-wise model after "
                                      "set_testing()")
        ctx = self.ctx
        st = _lib.stream
        N, H, W, Cin0 = X.shape
        self._X = self._X_own = self.input_buffer(X.shape)
        self._labels = self._labels_own = self.label_buffer(N)
        fwd, bwd = [], []
        lib = _lib.load()
        if self._side is None:
            self._side = torch.cuda.Stream(device=ctx.device)

        def L(name, *args, k=None, nb=0):
            """A prebuilt launch; `k` / `nb` = kernel name and algorithmic bytes for the roofline hook."""
            fn = getattr(lib, name)
            kname = k or name

            def run(fn=fn, args=args, name=name):
                with ops._Timed(kname, nb):
                    rc = fn(*args, st())
                if rc:
                    raise _lib.LbtError("%s failed with status %d" % (name, rc))
            run.kname = kname
            run.nbytes = nb
            return run

        self._nd, njobs = {}, []
        self._exps_snap = self._buf("exps_snap", tuple(ctx.exps.shape), torch.int32)

        def obs(q, n, table=True):
            """Declare an activation / gradient quantiser's per-step element count and give it a
            noise table (its inner = n / N noise values, refreshed by the step's first launch)."""
            q.observe(n)
            if table and q.stochastic and q not in self._nd:
                inner = n // N
                tab = self._buf("noise:" + q.name, ((inner + 3) // 4 * 4,), torch.float32)
                d = _lib.QDesc.from_buffer_copy(q.desc)
                d.noise = tab.data_ptr()
                self._nd[q] = d
                njobs.append(NJob(ctx.step.data_ptr(), ctx.seed, q.qid, 0, inner, tab.data_ptr()))

        # ---- 4-bit weights (config 5): every MFMA conv's int8 operand images live in ONE arena so a
        # single lbt_pack_int4 launch packs them all (two codes per byte) after quantisation
        w4 = [c for c in self.convs if c.mfma and c.w4]
        if w4:
            sizes = [(c.wf.numel(), c.wd.numel()) for c in w4]
            total = sum(a + b for a, b in sizes)
            self._w8 = torch.zeros(total, dtype=torch.int8, device=ctx.device)
            self._w4 = torch.zeros(total // 2, dtype=torch.uint8, device=ctx.device)
            off = 0
            for c, (a, b) in zip(w4, sizes):
                c.wf = self._w8[off:off + a].view(c.wf.shape)
                c.wf4 = self._w4[off // 2:(off + a) // 2].view(c.wf4.shape)
                off += a
                c.wd = self._w8[off:off + b].view(c.wd.shape)
                c.wd4 = self._w4[off // 2:(off + b) // 2].view(c.wd4.shape)
                off += b

        # ---- batched weight + gamma/beta quantisation (all layers, one launch each)
        wjobs = []
        for c in self.convs:
            kh, kw, ci, co = c.ksize
            c.W_range.observe(c.W.numel())
            wjobs.append(WJob(c.W.data_ptr(), kh, kw, ci, co, c.W_range.desc, c.w_hwio.data_ptr(),
                              c.wf.data_ptr() if c.mfma else None, c.ksf, c.wd.data_ptr() if c.mfma else None,
                              c.ksd, c.wcolsum.data_ptr() if c.mfma else None))
        d = self.dense
        d.W_range.observe(d.W.numel())
        wjobs.append(WJob(d.W.data_ptr(), d.in_units, 1, 1, d.units, d.W_range.desc, d.w_hwio.data_ptr(),
                          None, 0, None, 0, None))
        self._wjobs = _dev_array(wjobs, ctx.device)
        max_cout = max(j.Cout for j in wjobs)
        if w4:
            self._w4_pack = L("lbt_pack_int4", ptr(self._w8), ptr(self._w4), self._w8.numel(), k="pack_int4_kernel",
                              nb=self._w8.numel() + self._w4.numel())
        qjobs = []
        for r in self.rescales:
            C = r.C
            r.g_range.observe(C)
            r.b_range.observe(C)
            qjobs.append(QJob(r.gamma.data_ptr(), r.gb.data_ptr(), _lib.OUT_F32, C, 1, r.g_range.desc))
            qjobs.append(QJob(r.beta.data_ptr(), r.gb.data_ptr() + 4 * C, _lib.OUT_F32, C, 1, r.b_range.desc))
        self._qjobs = _dev_array(qjobs, ctx.device)

        # ---- stem: conv1 on the signed 9-bit image (VALU), BN, ReLU
        c = self.conv1
        kh, kw, _, C0 = c.ksize
        dc = ops.conv_desc(N, H, W, Cin0, C0, kh, kw, c.strides[1], c.strides[2], c.padding)
        c.d = dc
        ximg = self._buf("ximg", (N, H, W, Cin0), torch.int16)
        obs(c.X_range, X.numel(), table=False)  # quantised inside the step prologue (Philox inline)
        self._input_job = QJob(self._X.data_ptr(), ximg.data_ptr(), OUT_I16, X.numel(), H * W * Cin0, c.X_range.desc)
        n0, r0 = self.n0, self.r0
        shp0 = (N, dc.Ho, dc.Wo, C0)
        numel0 = math.prod(shp0)
        qn0 = self._buf("qn0", shp0, torch.int8)
        chs0 = self._sums("chs0", ops.NSHARD * 2 * C0)
        obs(n0.X_range, numel0)
        self._stem = c.stem(dc)
        if self._stem:
            # fp16-MFMA stem with the bn0-norm quantiser + channel sums in its epilogue
            fwd.append(L("lbt_conv_stem_fwd", ptr(ximg), ptr(c.w_hwio), dc, self._qd(c.X_range), c.W_range.desc, None,
                         ptr(qn0), self._qd(n0.X_range), ptr(chs0), k="stem_fwd_kernel",
                         nb=ximg.numel() * 2 + c.w_hwio.numel() + numel0))
        else:
            y0 = self._buf("y0", shp0, torch.float32)
            fwd.append(L("lbt_conv_fwd_generic", ptr(ximg), 1, ptr(c.w_hwio), dc, self._qd(c.X_range), c.W_range.desc,
                         ptr(y0), k="conv_fwd_generic_kernel", nb=ximg.numel() * 2 + numel0 * 4))
            fwd.append(L("lbt_dfxp_quantize", ptr(y0), ptr(qn0), OUT_I8, N, numel0 // N, self._qd(n0.X_range), ptr(chs0),
                         C0, k="quantize_rows_kernel", nb=numel0 * 5))
        R0 = self._buf("R0", shp0, torch.int8)
        X0 = self._buf("X0", shp0, torch.float32)
        b0 = self.blocks[0]
        xa = self._buf("xa0", shp0, torch.int8)
        xs = self._buf("xs0", shp0, torch.int8) if b0.cs is not None else None
        obs(r0.X_range, numel0)
        obs(b0.c1.X_range, numel0)
        if xs is not None:
            obs(b0.cs.X_range, numel0)
        a = self._chain_fwd(n0, qn0, chs0, r0, R0, None, None, None, None, None, relu=True, y=X0,
                            o1=xa, q1=b0.c1.X_range, o2=xs, q2=b0.cs.X_range if xs is not None else None)
        if self.sync_bn:
            fwd.append(self._allreduce(chs0))
        self._keep = [a]
        self._chain_pending = a

        # ---- residual blocks
        Xin = X0
        saved = []
        for i, b in enumerate(self.blocks):
            nxt = self.blocks[i + 1] if i + 1 < len(self.blocks) else None
            Xin, xa, xs, info = self._block_fwd(i, b, nxt, Xin, xa, xs, fwd, L, obs)
            saved.append(info)
        Ylast = Xin
        # the last block's end chain: launched here, or (the training step's fused head) evaluated inside
        # the head launch; the separate head launches (forward / compute_loss / backward) run it first
        last = self._chain_pending
        self._chain_pending = None
        last_launch = None
        if last is not None:
            last_launch = L("lbt_bn_chain_fwd", ctypes.byref(last), k="chain_fwd_kernel", nb=ops._chain_fwd_bytes(last))

        # ---- head: avg pool, dense, loss -- as separate launches (forward / compute_loss /
        # backward called one by one) and as ONE fused launch (train_fwd_bwd, the training step)
        Nb, Hh, Wh, Ch = Ylast.shape
        pooled = self._buf("pool", (Nb, Ch), torch.float32)
        hfwd, hloss, hbwd = [], [], []  # (the end chain joins hfwd or fwd once head_chain is decided, below)
        hfwd.append(L("lbt_avgpool_fwd", ptr(Ylast), ptr(pooled), Nb, Hh * Wh, Ch))
        dd = _lib.ConvDesc(Nb, 1, 1, d.in_units, d.units, 1, 1, 1, 1, 0, 0, 0, 0, 1, 1)
        d.d = dd
        pq = self._buf("pq", (Nb, Ch), torch.int8)
        obs(d.X_range, pooled.numel())
        hfwd.append(L("lbt_dfxp_quantize", ptr(pooled), ptr(pq), OUT_I8, Nb, Ch, self._qd(d.X_range), None, 0))
        self.logits = self._buf("logits", (Nb, d.units), torch.float32)
        hfwd.append(L("lbt_conv_fwd_generic", ptr(pq), 0, ptr(d.w_hwio), dd, self._qd(d.X_range), d.W_range.desc,
                      ptr(self.logits)))
        self.loss = self._buf("loss", (1,), torch.float32)
        self.dlogits = self._buf("dz", (Nb, d.units), torch.float32)
        hloss.append(L("lbt_softmax_xent", ptr(self.logits), ptr(self._labels), Nb, d.units, ptr(self.loss),
                       ptr(self.dlogits)))

        # ================================================================ backward
        rjobs, pjobs = [], []
        gqd = self._buf("gqd", (Nb, d.units), torch.int8)
        obs(d.grad_range, self.dlogits.numel())
        hbwd.append(L("lbt_dfxp_quantize", ptr(self.dlogits), ptr(gqd), OUT_I8, Nb, d.units, self._qd(d.grad_range), None,
                      0))
        nsd = ops.wgrad_nsplit(dd, generic=True)
        slabd = self._buf("slabd", (nsd, d.in_units, d.units), torch.int32)
        hbwd.append(L("lbt_conv_wgrad_generic", ptr(pq), 0, ptr(gqd), dd, ptr(slabd), nsd,
                      k="conv_wgrad_generic_kernel", nb=pq.numel() + gqd.numel() + 4 * slabd.numel()))
        hbwd.append(L("lbt_conv_wgrad_reduce", ptr(slabd), nsd, d.in_units, d.units, 0, None, self._qd(d.X_range),
                      self._qd(d.grad_range), ptr(d.W), ops.f32(2 * d.weight_decay), ptr(d.dW)))
        dpool = self._buf("dpool", (Nb, Ch), torch.float32)
        hbwd.append(L("lbt_conv_dgrad_generic", ptr(gqd), ptr(d.w_hwio), dd, self._qd(d.grad_range), d.W_range.desc,
                      ptr(dpool), None))
        gY = self._buf("gYlast", Ylast.shape, torch.float32)
        hbwd.append(L("lbt_avgpool_bwd", ptr(dpool), ptr(gY), Nb, Hh * Wh, Ch))
        scratch = self._buf("head_scratch", (lib.lbt_head_scratch_bytes(Nb, Ch, d.units),), torch.uint8)
        hd = _lib.Head(Ylast.data_ptr(), Nb, Hh * Wh, Ch, d.units, pooled.data_ptr(), pq.data_ptr(), self._qd(d.X_range),
                       d.w_hwio.data_ptr(), d.W_range.desc, self._labels.data_ptr(), self.logits.data_ptr(),
                       self.loss.data_ptr(), self.dlogits.data_ptr(), gqd.data_ptr(), self._qd(d.grad_range),
                       d.W.data_ptr(), ops.f32(2 * d.weight_decay), d.dW.data_ptr(), gY.data_ptr(),
                       scratch.data_ptr(), Nb * ctx.world_size)  # mean over the global batch
        self._head = hd
        hfused = [L("lbt_head_fwd_bwd", ctypes.byref(hd), k="head_kernel",
                    nb=4 * Ylast.numel() * 2 + d.w_hwio.numel())]
        self._hfwd, self._hloss, self._hbwd, self._hfused = hfwd, hloss, hbwd, hfused
        # Pass-A descriptors of every block-end BN chain and of the stem's, built first: each runs
        # as the epilogue of the dgrad that produces its input gradient (lbt_conv_dgrad_chain_i8),
        # except the last block's, which follows the avgpool backward.
        ends = [self._block_end_chain(i, b, saved[i], obs) for i, b in enumerate(self.blocks)]
        # the last block's output pass A runs inside the fused head (per sample, on the un-pooled
        # gradient it would have written); the separate head launches run it after avgpool_bwd
        aL = ends[-1]["a"]
        head_a = self.head_pass_a and not aL.has_b2 and bool(aL.y_mask) and (1024 % Ch == 0)
        if head_a:
            aL.g = gY.data_ptr()
            hd.pa = ctypes.addressof(aL)
            hbwd.append(L("lbt_bn_chain_bwd_a", ctypes.byref(aL), k="chain_bwd_a_kernel", nb=ops._chain_bwd_a_bytes(aL)))
            # head bytes: x in, weights, and pass A's operands / outputs instead of the fp32 gx
            hfused[0].nbytes = 4 * Ylast.numel() + d.w_hwio.numel() + ops._chain_bwd_a_bytes(aL) - 4 * Ylast.numel()
            gY = None
        qr_last = last.b1.qr if last is not None else None
        head_chain = (self.head_chain and head_a and last is not None and not last.has_b2 and bool(last.b1.nrm.q)
                      and bool(last.res) and bool(last.relu) and not last.o1 and not last.o2 and last.C == Ch
                      and Hh * Wh * Ch == 4096 and qr_last.bits > 0 and qr_last.stochastic and bool(qr_last.noise))
        if head_chain:
            hd.chain = ctypes.addressof(last)
            # the training step's fused head evaluates the chain itself; the separate head launches
            # (forward / compute_loss / backward) run it first -- in exactly one of the two lists, since
            # forward() runs _fwd + _hfwd
            hfwd.insert(0, last_launch)
            # per element the chain's operands (q codes 1 B, residual 4 B) replace the block output (4 B) and
            # pass A's y mask / R / qn reads (6 B), which come from registers; y and R are not written
            hfused[0].nbytes += (5 - 4 - 6) * Ylast.numel()
        elif last_launch is not None:
            fwd.append(last_launch)
        gq0 = self._buf("gq0", shp0, torch.int8)
        Gn0 = self._buf("Gn0", shp0, torch.int8)
        sums0 = self._sums("sums0", ops.NSHARD * 4 * C0)
        obs(r0.grad_range, numel0)
        obs(n0.grad_range, numel0)
        obs(c.grad_range, numel0)
        aA = self._chain_bwd_a(None, X0, False, None, (r0, R0, n0, qn0, Gn0, sums0), None, shp0, C0)
        stem_end = dict(a=aA)
        for i in reversed(range(len(self.blocks))):
            consumer = ends[i - 1] if i > 0 else stem_end
            gY = self._block_bwd(i, self.blocks[i], saved[i], gY, ends[i], consumer, bwd, L, obs, rjobs, pjobs)

        # ---- stem backward (d loss / d image is never needed)
        self._flush_pending(bwd, L)
        tail_fork = self.tail_fork and self.batch_wgrad and not (self.overlap_wgrad or self.side_wgrad)
        # the stem's pass B evaluated inside its weight-gradient launch (lbt_conv_stem_bwd): one launch,
        # and the gradient codes (read by nothing else: d loss / d image is not needed) stay in LDS
        stem_bwd = (self._stem and os.environ.get("LBT_STEM_BWD", "1") == "1" and C0 == 16 and Cin0 <= 4
                    and (dc.KH, dc.KW, dc.SH, dc.SW, dc.PT, dc.PL) == (3, 3, 1, 1, 1, 1) and dc.Ho == H and dc.Wo == W
                    and W in (8, 16, 32, 64) and (H * W) % 256 == 0)
        # ... and that launch's row blocks as workgroups of the batched weight-gradient launch
        # (lbt_conv_wgrad_many_stem_i8; its first workgroups by default, its last with LBT_STEM_FIRST=0):
        # both read only block 0's dgrad output
        stem_merge = (stem_bwd and not tail_fork and os.environ.get("LBT_STEM_MERGE", "1") == "1"
                      and len(self._wbatch) > 0)
        if not stem_merge:
            self._flush_wbatch(bwd, L, side=tail_fork)
        if gY is not None:  # pass A not fused into block 0's dgrad
            aA.g = gY.data_ptr()
            bwd.append(L("lbt_bn_chain_bwd_a", ctypes.byref(aA), k="chain_bwd_a_kernel", nb=ops._chain_bwd_a_bytes(aA)))
        aB = self._chain_bwd_b(n0, Gn0, qn0, sums0, shp0, C0, gq0, c.grad_range, None)
        if self.sync_bn:
            bwd.append(self._allreduce(sums0))
        self._keep += [aA, aB]
        if stem_merge:
            aB.gq = None
            ns0, slab0 = ops.stem_slab(self._c, "slab0", dc, ctx)
            jobs, self._wbatch = self._wbatch, []
            arr = (WgradJob * len(jobs))(*jobs)
            self._keep.append(arr)
            bwd.append(L("lbt_conv_wgrad_many_stem_i8", arr, len(jobs), ctypes.byref(aB), ptr(ximg), dc, ptr(slab0),
                         ns0, k="conv_wgrad_many_stem_kernel",
                         nb=sum(w._nb for w in jobs) + ops._chain_bwd_b_bytes(aB) + 2 * ximg.numel() + 4 * slab0.numel()))
        elif stem_bwd:
            aB.gq = None
            ns0, slab0 = ops.stem_slab(self._c, "slab0", dc, ctx)
            bwd.append(L("lbt_conv_stem_bwd", ctypes.byref(aB), ptr(ximg), dc, ptr(slab0), ns0, k="stem_bwd_kernel",
                         nb=ops._chain_bwd_b_bytes(aB) + 2 * ximg.numel() + 4 * slab0.numel()))
        else:
            bwd.append(L("lbt_bn_chain_bwd_b", ctypes.byref(aB), k="chain_bwd_b_kernel", nb=ops._chain_bwd_b_bytes(aB)))
        if stem_bwd:
            pass  # (the weight gradient ran above)
        elif self._stem:
            ns0, slab0 = ops.stem_slab(self._c, "slab0", dc, ctx)
            bwd.append(L("lbt_conv_stem_wgrad", ptr(ximg), ptr(gq0), dc, ptr(slab0), ns0, k="stem_wgrad_kernel",
                         nb=2 * ximg.numel() + gq0.numel() + 4 * slab0.numel()))
        else:
            ns0 = ops.wgrad_nsplit(dc, generic=True)
            slab0 = self._buf("slab0", (ns0, kh * kw * Cin0, C0), torch.int32)
            bwd.append(L("lbt_conv_wgrad_generic", ptr(ximg), 1, ptr(gq0), dc, ptr(slab0), ns0,
                         k="conv_wgrad_generic_kernel", nb=2 * ximg.numel() + gq0.numel() + 4 * slab0.numel()))
        rjobs.append(RJob(slab0.data_ptr(), ns0, kh * kw * Cin0, C0, 0, None, self._qd(c.X_range), self._qd(c.grad_range),
                          c.W.data_ptr(), ops.f32(2 * c.weight_decay), c.dW.data_ptr()))
        pjobs.append(PJob(sums0.data_ptr(), C0, self._qd(r0.grad_range), self._qd(r0.X_range), r0.gamma.data_ptr(),
                          ops.f32(2 * r0.weight_decay), r0.dgamma.data_ptr(), r0.dbeta.data_ptr()))

        # ---- batched reductions (after the side-stream weight gradients have landed): every
        # split wgrad, every dgamma / dbeta and -- in the training step -- the head's Dense_q dW
        # and loss, one launch (lbt_step_reduce)
        if self.overlap_wgrad or (self.side_wgrad and self.fuse_bwd) or tail_fork:
            bwd.append(self._join_side())
        # the tail's dequantisations read the step's exponent snapshot (identical values: taken by the
        # prologue, and no exponent changes before the tail), so the fused update's range-update blocks
        # may rewrite the live exponents in the same launch
        snap = self._exps_snap.data_ptr()
        for j in rjobs:
            j.qx.exps = j.qg.exps = snap
        for j in pjobs:
            j.qrg.exps = j.qr.exps = snap
        hd.qx.exps = hd.qg.exps = snap
        self._rjobs = _dev_array(rjobs, ctx.device)
        total_blocks = sum(lib.lbt_rjob_blocks(j.K * j.Cout) for j in rjobs)
        self._pjobs = _dev_array(pjobs, ctx.device)
        max_c = max(j.C for j in pjobs)
        nb_red = sum(4 * j.nsplit * j.K * j.Cout + 8 * j.K * j.Cout for j in rjobs)
        self._tail_sep = [L("lbt_step_reduce", ptr(self._rjobs), len(rjobs), total_blocks, ptr(self._pjobs), len(pjobs),
                            max_c, None, k="step_reduce_kernel", nb=nb_red)]
        if self.xchg is not None:  # data parallel: the numerators go to the exchange buffer
            self._tail_fused = [L("lbt_step_reduce_x", ptr(self._rjobs), len(rjobs), total_blocks, ptr(self._pjobs),
                                  len(pjobs), max_c, ctypes.byref(hd), ctypes.byref(self.xchg), k="step_reduce_kernel",
                                  nb=nb_red + scratch.numel() + 8 * d.W.numel())]
        else:
            self._tail_fused = [L("lbt_step_reduce", ptr(self._rjobs), len(rjobs), total_blocks, ptr(self._pjobs),
                                  len(pjobs), max_c, ctypes.byref(hd), k="step_reduce_kernel",
                                  nb=nb_red + scratch.numel() + 8 * d.W.numel())]
        # ... + SGD-momentum on every parameter (w, a read and written, g written) + update_range
        nflat = sum(p.numel() for p in self._flat_params())
        self._tail_upd = [L("lbt_step_reduce_update", ptr(self._rjobs), len(rjobs), total_blocks, ptr(self._pjobs),
                            len(pjobs), max_c, ctypes.byref(hd), ctypes.byref(self._upd), k="step_reduce_kernel",
                            nb=nb_red + scratch.numel() + 8 * d.W.numel() + 16 * nflat)]
        # ---- this step's noise tables: one launch ahead of everything else
        self._njobs = _dev_array(njobs, ctx.device)
        max_n = max(j.n for j in njobs)
        # ... which also clears the step's integer sums (everything this plan carved from the arena)
        nz = ctx._sums_used
        if ctx._extra_arenas:  # the prologue clears the first arena only
            raise RuntimeError("FusedResNet: the sums arena overflowed (raise DfxpContext sums_capacity)")
        # (together with every weight / gamma / beta quantiser and the input image: one launch)
        split = self._stem and not w4 and self.convs[0] is self.conv1 and self.prologue_split
        if split:
            # the stem needs only the noise tables, the cleared sums, the input image and conv1's
            # weights: the other layers' weight / gamma / beta quantisers run on the side stream
            # underneath it and join before the first block's conv
            self._wjobs_rest = _dev_array(wjobs[1:], ctx.device)
            fwd.insert(0, L("lbt_step_prologue", ptr(self._njobs), len(njobs), max_n, ptr(ctx.sums_arena), nz,
                            ptr(self._wjobs), 1, wjobs[0].Cout, None, 0,
                            ctypes.byref(self._input_job), ptr(ctx.exps), ptr(self._exps_snap), len(ctx.quantizers),
                            k="step_prologue_kernel",
                            nb=4 * sum(j.n for j in njobs) + 8 * nz + 6 * X.numel()))
            fwd.insert(1, self._on_side(L("lbt_step_prologue", None, 0, 0, None, 0,
                                          ptr(self._wjobs_rest), len(wjobs) - 1, max(j.Cout for j in wjobs[1:]),
                                          ptr(self._qjobs), len(qjobs), None, None, None, 0,
                                          k="step_prologue_kernel"), force=True))
            fwd.insert(3, self._join_side())  # [P1, P2 (side), stem, join, ...]
        else:
            fwd.insert(0, L("lbt_step_prologue", ptr(self._njobs), len(njobs), max_n, ptr(ctx.sums_arena), nz,
                            ptr(self._wjobs), len(wjobs), max_cout, ptr(self._qjobs), len(qjobs),
                            ctypes.byref(self._input_job), ptr(ctx.exps), ptr(self._exps_snap), len(ctx.quantizers),
                            k="step_prologue_kernel",
                            nb=4 * sum(j.n for j in njobs) + 8 * nz + 6 * X.numel()))
        if w4:  # the packed weight images need the quantised ones
            fwd.insert(1, self._w4_pack)
        self._fwd, self._bwd = fwd, bwd

    # W4: the packed weight image and the *_w4 entry point of a conv's GEMM
    @staticmethod
    def _fn(c, name):
        return name + "w4" if getattr(c, "w4", False) else name

    @staticmethod
    def _wf(c):
        return ptr(c.wf4 if getattr(c, "w4", False) else c.wf)

    @staticmethod
    def _wd(c):
        return ptr(c.wd4 if getattr(c, "w4", False) else c.wd)

    def _qd(self, q):
        """The plan's descriptor of quantiser q: with its noise table when it has one."""
        return self._nd.get(q, q.desc)

    def _qs(self, q):
        """_qd(q) reading its exponent from the step's snapshot (lbt_step_prologue copies the exponents
        at the start of the step): for the step's last launch, whose range-update blocks rewrite the
        live exponents while its reductions dequantise (lbt_step_reduce_update)."""
        d = _lib.QDesc.from_buffer_copy(self._qd(q))
        d.exps = self._exps_snap.data_ptr()
        return d

    # ------------------------------------------------------------------ descriptor builders
    def _gn(self, n):
        """Elements per channel a BatchNorm's statistics are over: global under SyncBN."""
        return n * self.ctx.world_size if self.sync_bn else n

    def _bn_norm(self, n, q, chsum, numel, C):
        return BnNorm(q.data_ptr(), self._qd(n.X_range), chsum.data_ptr(), self._gn(numel // C), ops.f32(n.eps),
                      ops.f32(n.momentum), ops.f32(1 - n.momentum), n.ms.data_ptr(), n.X_mean_running.data_ptr(),
                      n.X_var_running.data_ptr())

    def _chain_fwd(self, n, qn, chs, r, R, n2, qn2, chs2, r2, R2, relu, y, o1=None, q1=None, o2=None, q2=None,
                   res=None):
        C = qn.shape[-1]
        a = ChainFwd()
        a.b1.nrm = self._bn_norm(n, qn, chs, qn.numel(), C)
        a.b1.qr = self._qd(r.X_range)
        a.b1.rout = R.data_ptr()
        a.b1.gb = r.gb.data_ptr()
        if n2 is not None:
            a.has_b2 = 1
            a.b2.nrm = self._bn_norm(n2, qn2, chs2, qn2.numel(), C)
            a.b2.qr = self._qd(r2.X_range)
            a.b2.rout = R2.data_ptr()
            a.b2.gb = r2.gb.data_ptr()
        a.res = res.data_ptr() if res is not None else None
        a.relu = 1 if relu else 0
        a.y = y.data_ptr() if y is not None else None
        if o1 is not None:
            a.o1, a.o1_kind, a.qo1 = o1.data_ptr(), OUT_U8OFF, self._qd(q1)
        if o2 is not None:
            a.o2, a.o2_kind, a.qo2 = o2.data_ptr(), OUT_U8OFF, self._qd(q2)
        a.rows, a.inner, a.C = qn.shape[0], qn.numel() // qn.shape[0], C
        return a

    def _chain_bwd_a(self, g, y_mask, mask_from_r, gmask, br1, br2, shape, C):
        a = ChainBwdA()
        a.g = g.data_ptr() if g is not None else None
        a.y_mask = y_mask.data_ptr() if y_mask is not None else None
        a.mask_from_r = 1 if mask_from_r else 0
        a.gmask_out = gmask.data_ptr() if gmask is not None else None
        for slot, br in ((0, br1), (1, br2)):
            if br is None:
                continue
            r, R, n, qn, G, sums = br
            bb = BwdBranch(self._qd(r.grad_range), R.data_ptr(), self._qd(r.X_range), r.gb.data_ptr(), self._qd(n.grad_range),
                           qn.data_ptr(), G.data_ptr(), None, sums.data_ptr())
            if slot == 0:
                a.b1 = bb
            else:
                a.b2 = bb
                a.has_b2 = 1
        a.rows, a.inner, a.C = shape[0], math.prod(shape[1:]), C
        return a

    def _chain_bwd_b(self, n, G, qn, sums, shape, C, gq, qo, gcol):
        rows = shape[0]
        inner = math.prod(shape[1:])
        return ChainBwdB(G.data_ptr(), self._qd(n.grad_range), qn.data_ptr(), self._qd(n.X_range), n.ms.data_ptr(),
                         sums.data_ptr(), self._gn(rows * inner // C), None, gq.data_ptr(), self._qd(qo),
                         gcol.data_ptr() if gcol is not None else None, rows, inner, C)

    # ------------------------------------------------------------------ one residual block
    def _block_fwd(self, i, b, nxt, Xin, xa, xs, fwd, L, obs):
        N, H, W, Cin = Xin.shape
        c1, c2, cs = b.c1, b.c2, b.cs
        C = c1.ksize[3]
        s = c1.strides[1]
        d1 = ops.conv_desc(N, H, W, Cin, C, 3, 3, s, s, c1.padding)
        d2 = ops.conv_desc(N, d1.Ho, d1.Wo, C, C, 3, 3, 1, 1, c2.padding)
        c1.d, c2.d = d1, d2
        shp = (N, d1.Ho, d1.Wo, C)
        numel = N * d1.Ho * d1.Wo * C
        k = "b%d_" % i
        qn1 = self._buf(k + "qn1", shp, torch.int8)
        chs1 = self._sums(k + "chs1", ops.NSHARD * 2 * C)
        obs(b.n1.X_range, numel)
        ds = qns = chss = Rs = None
        if cs is not None:
            ds = ops.conv_desc(N, H, W, Cin, C, 1, 1, s, s, cs.padding)
            cs.d = ds
            qns = self._buf(k + "qns", shp, torch.int8)
            chss = self._sums(k + "chss", ops.NSHARD * 2 * C)
            obs(b.ns.X_range, numel)
        pair = (self.pair_launch and cs is not None and not self._fusable_bwd(c1, d1, flag=True)
                and (Cin, C) in ((16, 32), (32, 64)))
        a = self._chain_pending
        # the whole transition (the pending end chain of the previous block + both strided convs and their
        # quantising epilogues) as ONE launch (lbt_conv_fwd2_fused_i8)
        fwd2 = (pair and a is not None and os.environ.get("LBT_FUSE_FWD2", "1") == "1" and not a.has_b2
                and a.o1 == xa.data_ptr() and a.o2 == xs.data_ptr() and bool(a.res) and bool(a.y)
                and W * Cin == 512 and d1.Ho % 4 == 0 and (d1.PT, d1.PL, ds.PT, ds.PL) == (0, 0, 0, 0)
                and getattr(c1, "w4", False) == getattr(cs, "w4", False))
        if fwd2:
            cf2 = _lib.ConvFwd2()
            cf2.c = a
            cf2.wf1, cf2.ksf1, cf2.wcolsum1 = self._wf(c1).value, c1.ksf, c1.wcolsum.data_ptr()
            cf2.wfs, cf2.ksfs, cf2.wcolsums = self._wf(cs).value, cs.ksf, cs.wcolsum.data_ptr()
            cf2.w4 = 1 if getattr(c1, "w4", False) else 0
            cf2.d1, cf2.ds, cf2.qw1, cf2.qws = d1, ds, c1.W_range.desc, cs.W_range.desc
            cf2.yq1, cf2.qout1, cf2.ychsum1 = qn1.data_ptr(), self._qd(b.n1.X_range), chs1.data_ptr()
            cf2.yqs, cf2.qouts, cf2.ychsums = qns.data_ptr(), self._qd(b.ns.X_range), chss.data_ptr()
            self._keep.append(cf2)
            self._chain_pending = None
            nb = (ops._chain_fwd_bytes(a) + c1.wf.numel() + cs.wf.numel() + 2 * qn1.numel()
                  + 4 * (3 * a.inner + 2 * qn1.numel() // N))
            fwd.append(L("lbt_conv_fwd2_fused_i8", ctypes.byref(cf2), k="conv_fwd2_kernel", nb=nb))
        elif pair:  # conv-1 and the shortcut conv read the same input codes: one launch
            self._flush_chain(fwd, L)
            j0 = self._fwd_job(c1, d1, xa, qn1, b.n1.X_range, chs1)
            j1 = self._fwd_job(cs, ds, xs, qns, b.ns.X_range, chss)
            self._keep += [j0, j1]
            fwd.append(L("lbt_conv_fwd_pair_i8", ctypes.byref(j0), ctypes.byref(j1), k="conv_gemm2_kernel (fwd pair)",
                         nb=xa.numel() + xs.numel() + c1.wf.numel() + cs.wf.numel() + 2 * qn1.numel()))
        else:
            self._conv_fwd(fwd, L, c1, d1, xa, qn1, b.n1.X_range, chs1)
        R1 = self._buf(k + "R1", shp, torch.int8)
        xb = self._buf(k + "xb", shp, torch.int8)
        obs(b.r1.X_range, numel)
        obs(c2.X_range, numel)
        a1 = self._chain_fwd(b.n1, qn1, chs1, b.r1, R1, None, None, None, None, None, relu=True, y=None, o1=xb,
                             q1=c2.X_range)
        if self.sync_bn:
            fwd.append(self._allreduce(chs1))
        self._flush_chain(fwd, L)
        self._chain_pending = a1
        qn2 = self._buf(k + "qn2", shp, torch.int8)
        chs2 = self._sums(k + "chs2", ops.NSHARD * 2 * C)
        obs(b.n2.X_range, numel)
        self._conv_fwd(fwd, L, c2, d2, xb, qn2, b.n2.X_range, chs2)
        if cs is not None:
            if not pair:
                self._conv_fwd(fwd, L, cs, ds, xs, qns, b.ns.X_range, chss)
            Rs = self._buf(k + "Rs", shp, torch.int8)
            obs(b.rs.X_range, numel)
        R2 = self._buf(k + "R2", shp, torch.int8)
        obs(b.r2.X_range, numel)
        Y = self._buf(k + "Y", shp, torch.float32)
        xa_n = xs_n = None
        if nxt is not None:
            xa_n = self._buf("xa%d" % (i + 1), shp, torch.int8)
            obs(nxt.c1.X_range, numel)
            if nxt.cs is not None:
                xs_n = self._buf("xs%d" % (i + 1), shp, torch.int8)
                obs(nxt.cs.X_range, numel)
        a2 = self._chain_fwd(b.n2, qn2, chs2, b.r2, R2, b.ns, qns, chss, b.rs, Rs, relu=True, y=Y,
                             o1=xa_n, q1=nxt.c1.X_range if nxt is not None else None,
                             o2=xs_n, q2=nxt.cs.X_range if xs_n is not None else None,
                             res=None if cs is not None else Xin)
        if self.sync_bn:
            fwd.append(self._allreduce(chs2))
            if chss is not None:
                fwd.append(self._allreduce(chss))
        self._flush_chain(fwd, L)
        self._chain_pending = a2
        self._keep += [a1, a2]
        info = dict(Xin=Xin, xa=xa, xs=xs, d1=d1, d2=d2, ds=ds, qn1=qn1, R1=R1, xb=xb, qn2=qn2, R2=R2, qns=qns,
                    Rs=Rs, Y=Y, shp=shp, C=C, Cin=Cin)
        return Y, xa_n, xs_n, info

    def _block_end_chain(self, i, b, f, obs):
        """Pass A of block i's output BN(s): ReLU mask from Y, bn2 (and shortcut-BN) gradient
        quantisers and sums. Its input gradient is set later (fused dgrad or explicit g)."""
        k = "b%d_" % i
        shp, C = f["shp"], f["C"]
        numel = math.prod(shp)
        c2, cs = b.c2, b.cs
        Gn2 = self._buf(k + "Gn2", shp, torch.int8)
        sums2 = self._sums(k + "sums2", ops.NSHARD * 4 * C)
        for q in (b.r2.grad_range, b.n2.grad_range):
            obs(q, numel)
        gm = br2 = Gns = sumss = None
        if cs is not None:
            Gns = self._buf(k + "Gns", shp, torch.int8)
            sumss = self._sums(k + "sumss", ops.NSHARD * 4 * C)
            br2 = (b.rs, f["Rs"], b.ns, f["qns"], Gns, sumss)
            for q in (b.rs.grad_range, b.ns.grad_range):
                obs(q, numel)
        else:
            gm = self._buf(k + "gm", shp, torch.float32)
        a = self._chain_bwd_a(None, f["Y"], False, gm, (b.r2, f["R2"], b.n2, f["qn2"], Gn2, sums2), br2, shp, C)
        self._keep.append(a)
        return dict(a=a, Gn2=Gn2, sums2=sums2, gm=gm, Gns=Gns, sumss=sumss)

    def _flush_chain(self, fwd, L):
        """Launch the pending forward chain on its own (the next launch does not absorb it)."""
        a = self._chain_pending
        if a is None:
            return
        self._chain_pending = None
        fwd.append(L("lbt_bn_chain_fwd", ctypes.byref(a), k="chain_fwd_kernel", nb=ops._chain_fwd_bytes(a)))

    def _fwd_job(self, c, d, xq, yq, qout, chs):
        """One lbt_conv_fwd_job: the arguments of conv c's lbt_conv_fwd_i8 (quantising epilogue)."""
        return _lib.ConvFwdJob(xq.data_ptr(), 1, 1 if getattr(c, "w4", False) else 0, self._wf(c).value, c.ksf,
                               c.wcolsum.data_ptr(), d, self._qd(c.X_range), c.W_range.desc, None, yq.data_ptr(),
                               self._qd(qout), chs.data_ptr())

    def _conv_fwd(self, fwd, L, c, d, xq, yq, qout, chs):
        """Append conv c's forward (quantising epilogue yq / qout / chs): one lbt_conv_fwd_fused_i8 with
        the pending chain when that chain produces exactly this conv's input, else the chain's own
        launch (if any) and lbt_conv_fwd_i8."""
        a = self._chain_pending
        if (a is not None and self.fuse_fwd and self._fusable_bwd(c, d, flag=True) and a.o1 == xq.data_ptr()
                and not a.o2):
            cf = ConvFwd()
            cf.c = a
            cf.wf = self._wf(c).value
            cf.ksf = c.ksf
            cf.w4 = 1 if getattr(c, "w4", False) else 0
            cf.wcolsum = c.wcolsum.data_ptr()
            cf.d = d
            cf.qw = c.W_range.desc
            cf.yq = yq.data_ptr()
            cf.qout = self._qd(qout)
            cf.ychsum = chs.data_ptr()
            nq = (2 if a.has_b2 else 1) + 2  # noise tables: R quantiser(s), X, output
            nb = ops._chain_fwd_bytes(a) + c.wf.numel() + yq.numel() + 4 * nq * a.inner
            fwd.append(L("lbt_conv_fwd_fused_i8", ctypes.byref(cf), k="conv_fwd_fused_kernel", nb=nb))
            self._keep.append(cf)
            self._chain_pending = None
            return
        self._flush_chain(fwd, L)
        fwd.append(L(self._fn(c, "lbt_conv_fwd_i8"), ptr(xq), 1, self._wf(c), c.ksf, ptr(c.wcolsum), d, self._qd(c.X_range),
                     c.W_range.desc, None, ptr(yq), self._qd(qout), ptr(chs), k="conv_gemm_kernel<0> (fwd)",
                     nb=xq.numel() + c.wf.numel() + yq.numel()))

    def _fusable_bwd(self, c, d, flag=None):
        """lbt_conv_bwd_fused_i8 / lbt_conv_fwd_fused_i8 take this conv: stride-1 3x3 SAME, Cin = Cout,
        W*C = 512 (flag: the switch to honour, default fuse_bwd)."""
        return ((self.fuse_bwd if flag is None else flag) and c.mfma and d.KH == 3 and d.KW == 3 and d.SH == 1 and d.SW == 1 and d.PT == 1
                and d.PB == 1 and d.PL == 1 and d.PR == 1 and d.Cin == d.Cout and d.Cin in (16, 32, 64)
                and d.H % (8 if d.Cin == 16 else 4) == 0 and d.W * d.Cin == 512)

    @staticmethod
    def _bwd_tiles(d):
        """lbt_conv_bwd_fused_i8's workgroup tiles for conv d (conv_mfma.hip tile_rows_for)."""
        cs = d.Cin // 16
        if cs != 1:
            f23 = os.environ.get("LBT_TILE_ROWS23")
            th = 2 if d.H % 4 == 0 and f23 != "4" and (f23 == "2" or d.N * d.H // 4 < 256) else 4
        elif d.N * (d.H // 8) >= 256:
            th = 8
        else:
            th = 2 if d.N * d.H // 4 < 256 else 4
        return d.N * (d.H // th)

    def _defers(self, d, fusable):
        """This conv's fused backward launch takes a deferred wgrad job (and defers its own)."""
        return bool(self.batch_wgrad and self.defer_underfilled and fusable and self._bwd_tiles(d) < 2 * 256)

    def _wgrad(self, bwd, L, xq, gq, d, slab, nsplit, nshard, nb):
        """One conv's weight gradient (pass 1 into its slab): a job of the end-of-backward batched
        launch, or its own lbt_conv_wgrad_i8 launch (on the side stream in overlap mode)."""
        if self.batch_wgrad:
            w = self._wjob(xq, gq, d, slab, nsplit, nshard)
            w._nb = nb
            self._wbatch.append(w)
            return
        bwd.append(self._on_side(L("lbt_conv_wgrad_i8", ptr(xq), 1, ptr(gq), d, ptr(slab), nsplit, nshard,
                                   k="conv_wgrad_kernel", nb=nb)))

    def _flush_wbatch(self, bwd, L, side=False):
        """The batched weight-gradient launch of every job collected so far (side: on the side stream,
        joined before the final reduction)."""
        jobs, self._wbatch = self._wbatch, []
        if not jobs:
            return
        arr = (WgradJob * len(jobs))(*jobs)
        self._keep.append(arr)
        run = L("lbt_conv_wgrad_many_i8", arr, len(jobs), k="conv_wgrad_many_kernel", nb=sum(w._nb for w in jobs))
        bwd.append(self._on_side(run, force=True) if side else run)

    def _flush_pending(self, bwd, L):
        """Run the deferred wgrad job on its own (the next launch is not a fused conv backward), or
        hand it to the end-of-backward batch."""
        w = self._pending
        if w is None:
            return
        self._pending = None
        if self.batch_wgrad:
            self._wbatch.append(w)
            return
        bwd.append(L("lbt_conv_wgrad_i8", w.xq, w.x_u8off, w.gq, w.d, w.slab, w.nsplit, w.nshard,
                     k="conv_wgrad_kernel", nb=w._nb))

    def _conv_bwd(self, aB, c, d, add, aA, bwd, L, wjob):
        """Append one lbt_conv_bwd_fused_i8 launch (pass B aB -> dgrad of conv c -> pass A aA), carrying
        the pending wgrad job; wjob (this conv's own wgrad) becomes the pending one."""
        cb = ConvBwd()
        cb.b = aB
        cb.wd = self._wd(c).value
        cb.ksd = c.ksd
        cb.w4 = 1 if getattr(c, "w4", False) else 0
        cb.d = d
        cb.qw = c.W_range.desc
        cb.add_src = add.data_ptr() if add is not None else None
        cb.a = aA
        nbw = 0
        if self.batch_wgrad and self._defers(d, True):  # carry the pending job, defer this conv's
            if self._pending is not None and self._pending.d.Cin == d.Cin:
                cb.w = self._pending
                nbw = self._pending._nb
                self._pending = None
            self._flush_pending(bwd, L)  # (a job of another width: to the batch)
            nb = (ops._chain_bwd_b_bytes(aB) + 4 * aB.inner
                  + ops._dgrad_chain_bytes(0, c.wd.numel(), aA, add is not None) + nbw)
            bwd.append(L("lbt_conv_bwd_fused_i8", ctypes.byref(cb), k="conv_bwd_kernel", nb=nb))
            self._keep.append(cb)
            self._pending = wjob
            return
        if self.batch_wgrad:  # this conv's wgrad joins the end-of-backward batch
            self._flush_pending(bwd, L)
            nb = (ops._chain_bwd_b_bytes(aB) + 4 * aB.inner
                  + ops._dgrad_chain_bytes(0, c.wd.numel(), aA, add is not None))
            bwd.append(L("lbt_conv_bwd_fused_i8", ctypes.byref(cb), k="conv_bwd_kernel", nb=nb))
            self._keep.append(cb)
            self._wbatch.append(wjob)
            return
        if self.side_wgrad:  # this conv's wgrad as a parallel branch: nothing deferred
            nb = (ops._chain_bwd_b_bytes(aB) + 4 * aB.inner
                  + ops._dgrad_chain_bytes(0, c.wd.numel(), aA, add is not None))
            bwd.append(L("lbt_conv_bwd_fused_i8", ctypes.byref(cb), k="conv_bwd_kernel", nb=nb))
            self._keep.append(cb)
            w = wjob
            bwd.append(self._on_side(L("lbt_conv_wgrad_i8", w.xq, w.x_u8off, w.gq, w.d, w.slab, w.nsplit, w.nshard,
                                       k="conv_wgrad_kernel", nb=w._nb), force=True))
            return
        if self._pending is not None:
            cb.w = self._pending
            nbw = self._pending._nb
        inner = aB.inner
        nb = (ops._chain_bwd_b_bytes(aB) + 4 * inner
              + ops._dgrad_chain_bytes(0, c.wd.numel(), aA, add is not None) + nbw)
        bwd.append(L("lbt_conv_bwd_fused_i8", ctypes.byref(cb), k="conv_bwd_kernel", nb=nb))
        self._keep.append(cb)
        self._pending = wjob

    @staticmethod
    def _wjob(xq, gq, d, slab, nsplit, nshard):
        w = WgradJob(xq.data_ptr(), 1, gq.data_ptr(), d, slab.data_ptr(), nsplit, nshard)
        w._nb = xq.numel() + gq.numel() + 4 * slab.numel()
        return w

    def _block_bwd(self, i, b, f, gY, end, consumer, bwd, L, obs, rjobs, pjobs):
        """Block i's backward. gY: materialised d loss / d Y (or None: pass A already ran inside
        the next block's dgrad). consumer: the pass A fed by this block's input gradient.
        Returns the materialised input gradient, or None when it was fused into `consumer`."""
        k = "b%d_" % i
        shp, C, Cin = f["shp"], f["C"], f["Cin"]
        numel = math.prod(shp)
        c1, c2, cs = b.c1, b.c2, b.cs
        d1, d2, ds = f["d1"], f["d2"], f["ds"]
        fuse = self.fuse_dgrad_chain
        for q in (c2.grad_range, b.r1.grad_range, b.n1.grad_range, c1.grad_range):
            obs(q, numel)
        if cs is not None:
            obs(cs.grad_range, numel)
        Gn2, sums2, gm, Gns, sumss = end["Gn2"], end["sums2"], end["gm"], end["Gns"], end["sumss"]
        if gY is not None:
            aA2 = end["a"]
            aA2.g = gY.data_ptr()
            bwd.append(L("lbt_bn_chain_bwd_a", ctypes.byref(aA2), k="chain_bwd_a_kernel",
                         nb=ops._chain_bwd_a_bytes(aA2)))
        gq2 = self._buf(k + "gq2", shp, torch.int8)
        gcol2 = self._sums(k + "gcol2", ops.NSHARD * 2 * C)
        aB2 = self._chain_bwd_b(b.n2, Gn2, f["qn2"], sums2, shp, C, gq2, c2.grad_range, gcol2)
        if self.sync_bn:
            bwd.append(self._allreduce(sums2))
            if sumss is not None:
                bwd.append(self._allreduce(sumss))
        fb2 = self._fusable_bwd(c2, d2)
        fb1 = self._fusable_bwd(c1, d1)
        if not fb2:
            bwd.append(L("lbt_bn_chain_bwd_b", ctypes.byref(aB2), k="chain_bwd_b_kernel",
                         nb=ops._chain_bwd_b_bytes(aB2)))
        keep = [aB2]
        gqs = gcols = aBs = None
        if cs is not None:
            gqs = self._buf(k + "gqs", shp, torch.int8)
            gcols = self._sums(k + "gcols", ops.NSHARD * 2 * C)
            aBs = self._chain_bwd_b(b.ns, Gns, f["qns"], sumss, shp, C, gqs, cs.grad_range, gcols)
            if not fb2:
                bwd.append(L("lbt_bn_chain_bwd_b", ctypes.byref(aBs), k="chain_bwd_b_kernel",
                             nb=ops._chain_bwd_b_bytes(aBs)))
            keep.append(aBs)
        # conv-2 dgrad, fused with pass A of bn1 (ReLU mask recomputed from R1)
        Gn1 = self._buf(k + "Gn1", shp, torch.int8)
        sums1 = self._sums(k + "sums1", ops.NSHARD * 4 * C)
        nb_dg2 = gq2.numel() + c2.wd.numel()
        sp2, ns2, slab2 = ops.wgrad_slab(self._c, k + "slab2", d2, self.ctx, batched=self.batch_wgrad)
        nb_wg2 = f["xb"].numel() + gq2.numel() + 4 * slab2.numel()
        # the shortcut BN's pass B shares one launch with bn1's when conv-1 is not fused either
        bpair = self.pair_launch and cs is not None and fb2 and not fb1
        if fb2:  # pass B (bn2) + dgrad + pass A (bn1) in one launch, conv-2 wgrad deferred
            if cs is not None and not bpair:  # the shortcut BN's pass B (its conv is not fused) goes first
                bwd.append(L("lbt_bn_chain_bwd_b", ctypes.byref(aBs), k="chain_bwd_b_kernel",
                             nb=ops._chain_bwd_b_bytes(aBs)))
            aA1 = self._chain_bwd_a(None, None, True, None, (b.r1, f["R1"], b.n1, f["qn1"], Gn1, sums1), None, shp, C)
            self._conv_bwd(aB2, c2, d2, None, aA1, bwd, L, self._wjob(f["xb"], gq2, d2, slab2, sp2, ns2))
        elif fuse:
            aA1 = self._chain_bwd_a(None, None, True, None, (b.r1, f["R1"], b.n1, f["qn1"], Gn1, sums1), None, shp, C)
            nb = ops._dgrad_chain_bytes(gq2.numel(), c2.wd.numel(), aA1, False)
            if self.fuse_wgrad and not self.batch_wgrad:  # conv-2 wgrad in the same launch
                bwd.append(L(self._fn(c2, "lbt_conv_dgrad_chain_wgrad_i8"), ptr(gq2), self._wd(c2), c2.ksd, d2,
                             self._qd(c2.grad_range), c2.W_range.desc, None, ctypes.byref(aA1), ptr(f["xb"]), 1,
                             ptr(slab2), sp2, ns2, k="dgrad_wgrad_kernel", nb=nb + nb_wg2 - gq2.numel()))
            else:
                bwd.append(L(self._fn(c2, "lbt_conv_dgrad_chain_i8"), ptr(gq2), self._wd(c2), c2.ksd, d2,
                             self._qd(c2.grad_range), c2.W_range.desc, None, ctypes.byref(aA1),
                             k="conv_gemm_kernel<1> (dgrad+A)", nb=nb))
        else:
            d1g = self._buf(k + "d1", shp, torch.float32)
            bwd.append(L(self._fn(c2, "lbt_conv_dgrad_i8"), ptr(gq2), self._wd(c2), c2.ksd, d2, self._qd(c2.grad_range),
                         c2.W_range.desc, ptr(d1g), None, k="conv_gemm_kernel<1> (dgrad)", nb=nb_dg2 + 4 * numel))
            aA1 = self._chain_bwd_a(d1g, None, True, None, (b.r1, f["R1"], b.n1, f["qn1"], Gn1, sums1), None, shp, C)
        keep.append(aA1)
        if not (fuse and self.fuse_wgrad and not self.batch_wgrad) and not fb2:
            self._wgrad(bwd, L, f["xb"], gq2, d2, slab2, sp2, ns2, nb_wg2)
        rjobs.append(RJob(slab2.data_ptr(), ns2, 9 * C, C, 1, gcol2.data_ptr(), self._qd(c2.X_range),
                          self._qd(c2.grad_range), c2.W.data_ptr(), ops.f32(2 * c2.weight_decay), c2.dW.data_ptr()))
        if not fuse:
            bwd.append(L("lbt_bn_chain_bwd_a", ctypes.byref(aA1), k="chain_bwd_a_kernel", nb=ops._chain_bwd_a_bytes(aA1)))
        gq1 = self._buf(k + "gq1", shp, torch.int8)
        gcol1 = self._sums(k + "gcol1", ops.NSHARD * 2 * C)
        aB1 = self._chain_bwd_b(b.n1, Gn1, f["qn1"], sums1, shp, C, gq1, c1.grad_range, gcol1)
        if self.sync_bn:
            bwd.append(self._allreduce(sums1))
        # conv-1's and the shortcut's dgrads (+ the consumer's pass A) as ONE launch
        dual = (self.pair_launch and cs is not None and not fb1 and fuse and not (self.fuse_wgrad and not self.batch_wgrad)
                and (Cin, C) in ((16, 32), (32, 64)) and getattr(c1, "w4", False) == getattr(cs, "w4", False))
        # ... and with both pass-B chains in the same launch (lbt_conv_bwd2_fused_i8): the whole transition
        bwd2 = (bpair and dual and os.environ.get("LBT_FUSE_BWD2", "1") == "1" and Cin * f["Xin"].shape[2] == 512
                and f["Xin"].shape[1] % (8 if Cin == 16 else 4) == 0 and (d1.PT, d1.PL, ds.PT, ds.PL) == (0, 0, 0, 0))
        if bpair:
            if not bwd2:  # (else both pass-B chains run inside the transition launch below)
                bwd.append(L("lbt_bn_chain_bwd_b_pair", ctypes.byref(aBs), ctypes.byref(aB1), k="chain_bwd_b2_kernel",
                             nb=ops._chain_bwd_b_bytes(aBs) + ops._chain_bwd_b_bytes(aB1)))
        elif not fb1:  # (a pending wgrad stays pending: the next fused launch carries it)
            bwd.append(L("lbt_bn_chain_bwd_b", ctypes.byref(aB1), k="chain_bwd_b_kernel",
                         nb=ops._chain_bwd_b_bytes(aB1)))
        keep.append(aB1)
        add = gm
        if cs is not None and not dual:
            dsg = self._buf(k + "dsc", f["Xin"].shape, torch.float32)
            bwd.append(L(self._fn(cs, "lbt_conv_dgrad_i8"), ptr(gqs), self._wd(cs), cs.ksd, ds, self._qd(cs.grad_range),
                         cs.W_range.desc, ptr(dsg), None, k="conv_gemm_kernel<1> (dgrad)",
                         nb=gqs.numel() + cs.wd.numel() + 4 * dsg.numel()))
            add = dsg
        # conv-1 dgrad (+ shortcut gradient), fused with the consumer's pass A
        nin = math.prod(f["Xin"].shape)
        nb_dg1 = gq1.numel() + c1.wd.numel() + 8 * nin
        gin = None
        sp1, ns1, slab1 = ops.wgrad_slab(self._c, k + "slab1", d1, self.ctx, batched=self.batch_wgrad)
        nb_wg1 = f["xa"].numel() + gq1.numel() + 4 * slab1.numel()
        if fb1:  # pass B (bn1) + dgrad (+ residual gradient) + the consumer's pass A, wgrad deferred
            self._conv_bwd(aB1, c1, d1, add, consumer["a"], bwd, L, self._wjob(f["xa"], gq1, d1, slab1, sp1, ns1))
        elif fuse:
            nb = ops._dgrad_chain_bytes(gq1.numel(), c1.wd.numel(), consumer["a"], add is not None)
            if self.fuse_wgrad and not self.batch_wgrad:  # conv-1 wgrad in the same launch
                bwd.append(L(self._fn(c1, "lbt_conv_dgrad_chain_wgrad_i8"), ptr(gq1), self._wd(c1), c1.ksd, d1,
                             self._qd(c1.grad_range), c1.W_range.desc, ptr(add), ctypes.byref(consumer["a"]),
                             ptr(f["xa"]), 1, ptr(slab1), sp1, ns1, k="dgrad_wgrad_kernel",
                             nb=nb + nb_wg1 - gq1.numel()))
            elif bwd2:
                cb2 = _lib.ConvBwd2()
                cb2.b1, cb2.bs = aB1, aBs
                cb2.wd1, cb2.ksd1, cb2.wds, cb2.ksds = self._wd(c1).value, c1.ksd, self._wd(cs).value, cs.ksd
                cb2.w4 = 1 if getattr(c1, "w4", False) else 0
                cb2.d1, cb2.ds, cb2.qw1, cb2.qws = d1, ds, c1.W_range.desc, cs.W_range.desc
                cb2.a = consumer["a"]
                self._keep.append(cb2)
                nb = (ops._chain_bwd_b_bytes(aBs) + ops._chain_bwd_b_bytes(aB1) + 4 * (aBs.inner + aB1.inner)
                      + ops._dgrad_chain_bytes(0, c1.wd.numel(), consumer["a"], False) + cs.wd.numel())
                bwd.append(L("lbt_conv_bwd2_fused_i8", ctypes.byref(cb2), k="conv_bwd2_kernel", nb=nb))
            elif dual:
                nb = (ops._dgrad_chain_bytes(gq1.numel(), c1.wd.numel(), consumer["a"], False)
                      + gqs.numel() + cs.wd.numel())
                bwd.append(L("lbt_conv_dgrad2_chain_i8", ptr(gq1), self._wd(c1), c1.ksd, d1, self._qd(c1.grad_range),
                             c1.W_range.desc, ptr(gqs), self._wd(cs), cs.ksd, ds, self._qd(cs.grad_range),
                             cs.W_range.desc, 1 if getattr(c1, "w4", False) else 0, ctypes.byref(consumer["a"]),
                             k="conv_dgrad2_kernel (dgrad x2 + A)", nb=nb))
            else:
                bwd.append(L(self._fn(c1, "lbt_conv_dgrad_chain_i8"), ptr(gq1), self._wd(c1), c1.ksd, d1,
                             self._qd(c1.grad_range), c1.W_range.desc, ptr(add), ctypes.byref(consumer["a"]),
                             k="conv_gemm_kernel<1> (dgrad+A)", nb=nb))
        else:
            gin = self._buf(k + "gin", f["Xin"].shape, torch.float32)
            bwd.append(L(self._fn(c1, "lbt_conv_dgrad_i8"), ptr(gq1), self._wd(c1), c1.ksd, d1, self._qd(c1.grad_range),
                         c1.W_range.desc, ptr(gin), ptr(add), k="conv_gemm_kernel<1> (dgrad)", nb=nb_dg1))
        if not (fuse and self.fuse_wgrad and not self.batch_wgrad) and not fb1:
            self._wgrad(bwd, L, f["xa"], gq1, d1, slab1, sp1, ns1, nb_wg1)
        rjobs.append(RJob(slab1.data_ptr(), ns1, 9 * Cin, C, 1, gcol1.data_ptr(), self._qd(c1.X_range),
                          self._qd(c1.grad_range), c1.W.data_ptr(), ops.f32(2 * c1.weight_decay), c1.dW.data_ptr()))
        if cs is not None:
            sps, nss, slabs = ops.wgrad_slab(self._c, k + "slabs", ds, self.ctx, batched=self.batch_wgrad)
            self._wgrad(bwd, L, f["xs"], gqs, ds, slabs, sps, nss, f["xs"].numel() + gqs.numel() + 4 * slabs.numel())
            rjobs.append(RJob(slabs.data_ptr(), nss, Cin, C, 1, gcols.data_ptr(), self._qd(cs.X_range),
                              self._qd(cs.grad_range), cs.W.data_ptr(), ops.f32(2 * cs.weight_decay), cs.dW.data_ptr()))
        for r in (b.r1, b.r2) + ((b.rs,) if cs is not None else ()):
            sm = {id(b.r1): sums1, id(b.r2): sums2}.get(id(r), sumss)
            pjobs.append(PJob(sm.data_ptr(), C, self._qd(r.grad_range), self._qd(r.X_range), r.gamma.data_ptr(),
                              ops.f32(2 * r.weight_decay), r.dgamma.data_ptr(), r.dbeta.data_ptr()))
        self._keep += keep
        return gin
