"""The reference's fp32 arithmetic beside the build's exact arithmetic (oracle; test infrastructure).

The build computes every integer GEMM and every BN / Rescale reduction EXACTLY (integer sums,
finished in double, rounded once) -- what the HIP kernels reproduce bit for bit and what
``oracle.nn`` restates in its default ``ARITH = "exact"`` mode. The reference instead hands the
same fake-quantised fp32 values to TensorFlow, which sums them in fp32 (``tf.nn.conv2d`` and its
backprops, ``tf.matmul``, ``tf.nn.moments``, the autodiff of the BN normalisation, Rescale's
reduce_sums, the overflow-rate reduce_means; ``dynamic_fixed_point.py:63-67,291,302-305,388,
457-460,588,616,623,689-691``). ``oracle.nn`` with ``ARITH = "tf32"`` is a model of that
arithmetic: fp32 GEMMs (BLAS sgemm, fp32 accumulation) and pairwise fp32 reductions (the class of
Eigen's tree reductions; TF's exact summation order is an implementation detail of its kernels and
cannot be reproduced without TensorFlow). Everything else -- the quantisers, the noise, the ReLU /
residual / pooling / softmax glue, the optimiser -- is shared.

``compare_step`` runs one training step both ways from the same state and measures how far the
reference's arithmetic lands from the build's: loss, every gradient, the BN running statistics,
the integer codes of every quantiser and the exponent updates. ``tools/tf_tolerance.py`` runs it
along the bench workload's trajectory; DESIGN.md section 4 quotes the result and
``tests/test_tf_tolerance.py`` pins the bounds.
"""
import contextlib

import numpy as np

from . import nn
from . import resnet as oresnet

F32 = np.float32


@contextlib.contextmanager
def arith(mode):
    old = nn.ARITH
    nn.ARITH = mode
    try:
        yield
    finally:
        nn.ARITH = old


def tf32_arith():
    return arith("tf32")


def _norms(model):
    return [l for l in oresnet._walk(model) if isinstance(l, nn.NormQ)]


def _bn_state(model):
    return [(n.mean_running.copy(), n.var_running.copy()) for n in _norms(model)]


def _set_bn_state(model, st):
    for n, (m, v) in zip(_norms(model), st):
        n.mean_running, n.var_running = m.copy(), v.copy()


def _rel(a, b):
    """max |a - b| / max |b| (0 when both are 0)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = np.max(np.abs(b)) if b.size else 0.0
    num = np.max(np.abs(a - b)) if b.size else 0.0
    return float(num / den) if den > 0 else float(num)


def _step_in(mode, model, state, x, y, seed, target, lr, momentum, bn0):
    _set_bn_state(model, bn0)
    with arith(mode):
        l, st, c = oresnet.train_step(model, state, x, y, lr, momentum, seed, target)
        g = oresnet.get_grads(model)
    return dict(loss=float(l), state=st, ctx=c, grads=g, bn=_bn_state(model))


def _diff(a, b):
    """Step-level distance of run a from run b (both from the same state)."""
    ga, gb = a["grads"], b["grads"]
    gnum = sum(float(np.sum((np.asarray(ga[k], np.float64) - gb[k]) ** 2)) for k in gb)
    gden = sum(float(np.sum(np.asarray(gb[k], np.float64) ** 2)) for k in gb)
    ca, cb = a["ctx"], b["ctx"]
    flips = {k: int(np.count_nonzero(ca.record[k] != cb.record[k])) for k in cb.record
             if k in ca.record and ca.record[k].shape == cb.record[k].shape}
    mism = sorted(k for k in b["state"]["ranges"] if b["state"]["ranges"][k] != a["state"]["ranges"][k])
    return dict(
        loss_rel=abs(a["loss"] - b["loss"]) / abs(b["loss"]),
        logits_rel=_rel(ca.logits, cb.logits),
        grad_rel_max=max(_rel(ga[k], gb[k]) for k in gb),
        grad_rel_l2=float(np.sqrt(gnum / gden)) if gden > 0 else 0.0,
        weights_rel_max=max(_rel(a["state"]["params"][k], b["state"]["params"][k]) for k in b["state"]["params"]),
        bn_mean_rel_max=max(_rel(p[0], q[0]) for p, q in zip(a["bn"], b["bn"])),
        bn_var_rel_max=max(_rel(p[1], q[1]) for p, q in zip(a["bn"], b["bn"])),
        code_flips=int(sum(flips.values())), code_elems=int(sum(ca.record[k].size for k in flips)),
        code_flip_tensors=int(sum(1 for v in flips.values() if v)),
        exponent_mismatches=len(mism), exponent_mismatch_names=mism)


def compare_step(model, state, x, y, seed=0, target=0.0, lr=1e-2, momentum=0.9, control=True):
    """One step from ``state`` (params, accum, ranges, step; BN running stats live in ``model``) in the
    exact arithmetic (the build's), in the reference's fp32 arithmetic ("tf32") and -- control -- in
    fp32 with another summation order ("tf32seq"). Returns (exact new state, metrics): "tf32" vs
    "exact" at step level and op level, and "tf32seq" vs "tf32" (how far two fp32 orders of the
    reference itself land apart). The model keeps the EXACT step's running statistics."""
    bn0 = _bn_state(model)
    runs = {m: _step_in(m, model, state, x, y, seed, target, lr, momentum, bn0)
            for m in (("tf32", "tf32seq") if control else ("tf32",))}
    ex = _step_in("exact", model, state, x, y, seed, target, lr, momentum, bn0)
    c_tf = runs["tf32"]["ctx"]
    rate_eq = all(np.float32(c) / np.float32(n) == c_tf.rates[k][0] and np.float32(c2) / np.float32(n) == c_tf.rates[k][1]
                  for k, (c, c2, n, _) in c_tf.counts.items() if k in c_tf.rates)
    m = _diff(runs["tf32"], ex)
    m.update(loss_exact=ex["loss"], loss_tf32=runs["tf32"]["loss"], rates_equal_counts=bool(rate_eq),
             op_level=op_level(model, ex["ctx"]))
    if control:
        m["control_tf32seq_vs_tf32"] = _diff(runs["tf32seq"], runs["tf32"])
    return ex["state"], m


class _ReplayCtx(nn.Ctx):
    """Hands a layer the integer codes a finished step recorded (its inputs are ignored), so one op
    can be re-evaluated in either arithmetic on IDENTICAL operands."""

    def __init__(self, ctx):
        super().__init__(dict(ctx.I), ctx.step, ctx.seed, ctx.target)
        self.src = ctx.record

    def q(self, name, x, bits, stochastic=True):
        q = self.src[name]
        self.record[name] = q
        return q, nn.dfxp.frac_bits(bits, self.I[name])


def _layer_both(layer, ctx, run):
    """run(copy) in exact and in tf32 arithmetic on copies of ``layer``."""
    import copy
    outs = []
    for mode in ("exact", "tf32"):
        lc = copy.deepcopy(layer)
        old = nn.ARITH
        nn.ARITH = mode
        try:
            outs.append(run(lc, _ReplayCtx(ctx)))
        finally:
            nn.ARITH = old
    return outs


def op_level(model, ctx):
    """After an EXACT step: every conv / dense / BN-norm / BN-rescale of ``model`` re-evaluated on the
    step's recorded integer codes in both arithmetics. Returns {op: max over layers of
    max|tf32 - exact| / max|exact|} -- the arithmetic difference alone, no code flips involved."""
    res = {}

    def put(k, v):
        res[k] = max(res.get(k, 0.0), v)
    for L in oresnet._walk(model):
        if isinstance(L, (nn.Conv2dQ, nn.DenseQ)) and not L.fmode:
            xs = ctx.record[L.name + "/X_range"].shape
            gs = ctx.record[L.name + "/grad_range"].shape

            def run(lc, rc, xs=xs, gs=gs):
                y = lc.forward(np.empty(xs, F32), rc)
                dx = lc.backward(np.empty(gs, F32), rc)
                return y, dx, lc.dW
            (y0, d0, w0), (y1, d1, w1) = _layer_both(L, ctx, run)
            kind = "conv" if isinstance(L, nn.Conv2dQ) else "dense"
            put(kind + "_fwd", _rel(y1, y0))
            if not (kind == "conv" and L.name == "conv1"):  # conv1's dX is not consumed (TF prunes it)
                put(kind + "_dgrad", _rel(d1, d0))
            put(kind + "_wgrad", _rel(w1, w0))
        elif isinstance(L, nn.NormQ) and not L.fmode and L.train:
            xs = ctx.record[L.name + "/X_range"].shape
            gs = ctx.record[L.name + "/grad_range"].shape

            def run(lc, rc, xs=xs, gs=gs):
                y = lc.forward(np.empty(xs, F32), rc)
                mu, sig = lc.mu.copy(), lc.sigma.copy()
                return y, mu, sig, lc.backward(np.empty(gs, F32), rc)
            (y0, m0, s0, d0), (y1, m1, s1, d1) = _layer_both(L, ctx, run)
            put("bn_mean", _rel(m1, m0))
            put("bn_sigma", _rel(s1, s0))
            put("bn_fwd", _rel(y1, y0))
            put("bn_bwd", _rel(d1, d0))
        elif isinstance(L, nn.RescaleQ) and not L.fmode:
            xs = ctx.record[L.name + "/X_range"].shape
            gs = ctx.record[L.name + "/grad_range"].shape

            def run(lc, rc, xs=xs, gs=gs):
                y = lc.forward(np.empty(xs, F32), rc)
                dx = lc.backward(np.empty(gs, F32), rc)
                return y, dx, lc.dgamma, lc.dbeta
            (y0, d0, g0, b0), (y1, d1, g1, b1) = _layer_both(L, ctx, run)
            put("rescale_fwd", _rel(y1, y0))
            put("rescale_dgamma", _rel(g1, g0))
            put("rescale_dbeta", _rel(b1, b0))
    return res


def init_state(model, seed=0, grad_range=None):
    """The bench CPU baseline's initialisation (U(+-sqrt(3/fan_in)) weights, gamma 1, beta 0, every
    range 2; grad_range: start the gradient quantisers there instead)."""
    rng = np.random.default_rng(seed)
    params = {}
    for name, owner in model.params():
        if name.endswith("/W"):
            shp = owner.ksize if hasattr(owner, "ksize") else (owner.in_units, owner.units)
            fan = float(np.prod(shp[:-1]))
            params[name] = rng.uniform(-np.sqrt(3 / fan), np.sqrt(3 / fan), size=shp).astype(F32)
        elif name.endswith("/g"):
            params[name] = np.ones(owner.C, F32)
        else:
            params[name] = np.zeros(owner.C, F32)
    ranges = oresnet.init_ranges(model)
    if grad_range is not None:
        ranges = {k: (grad_range if k.endswith("/grad_range") else v) for k, v in ranges.items()}
    return dict(params=params, accum={k: np.zeros_like(v) for k, v in params.items()}, ranges=ranges, step=0)


def run(batches, steps, seed=0, grad_range=None, log=None):
    """Teacher-forced comparison along the exact trajectory: every step starts both arithmetics from
    the exact state. Returns the per-step metrics."""
    model = oresnet.build_resnet((3, 3, 3), 8, 2e-4)
    state = init_state(model, seed, grad_range)
    out = []
    for i in range(steps):
        x, y = batches[i % len(batches)]
        state, m = compare_step(model, state, x, y, seed=seed)
        m["step"] = i
        out.append(m)
        if log is not None:
            log(m)
    return out
