"""Quantised layers of the DFXP path in numpy (oracle; test infrastructure only).

Each class restates one reference layer (``dynamic_fixed_point.py``) with the
Layer_q protocol ``forward(X) / backward(grad) / grads_and_vars()``:

* Conv2dQ    -- ``Conv2d_q`` / ``Conv2d_pq`` ``:129-316`` (X at bits+1, W at bits,
                grad at bits; dW = wgrad(Xq, gq) + 2*wd*W; dX = dgrad(gq, Wq)).
* DenseQ     -- ``Dense_q`` ``:319-470`` (X, W, grad all at bits).
* NormQ      -- ``Normalization_q`` ``:539-623`` (biased batch moments of Xq,
                eps 1e-5, running averages momentum 0.999; full BN backward).
* RescaleQ   -- ``Rescale_q`` ``:626-694`` (y = Xq*gq + bq; dgamma = sum gq*Xq + 2wd*gamma).
* BatchNormQ -- ``BatchNorm_q`` ``:697-743`` (Sequential(Norm, Rescale)).
* ReluQ / AvgPoolQ / FlattenQ / SequentialQ / ResidualBlockQ -- ``:983-1053``,
                ``:512-536``, ``:746-875``.

Integer arithmetic: integer GEMMs (conv fwd/dgrad/wgrad, dense) are computed
exactly (float64 BLAS on integer-valued operands, all partial sums < 2**53) and
dequantised once: ``float32(acc) * 2**-(e_a+e_b)``. TF sums the same integer
products in fp32; the two agree whenever the partial sums stay below 2**24 LSB.
BN moments and BN/Rescale backward reductions are taken from exact integer sums
of the quantised codes (see DESIGN.md "Numerics"): they are the same quantities
the reference computes with ``tf.nn.moments`` / ``tf.gradients``, without
order-dependent fp32 summation.
"""
import numpy as np

from . import dfxp

F32 = np.float32

# Arithmetic mode of the restatement (see oracle/tfarith.py):
#   "exact" -- the build's contract: integer GEMMs and BN / Rescale reductions summed exactly, finished
#              in double, rounded once to fp32 (what the HIP kernels compute bit for bit);
#   "tf32"  -- a model of the REFERENCE's own arithmetic: TF sums the same fake-quantised fp32 values
#              in fp32 -- tf.nn.conv2d / conv2d_backprop_* / tf.matmul as fp32 GEMMs
#              (dynamic_fixed_point.py:291,302-305,388,457-460), tf.nn.moments as fp32 reduce_means
#              (:588), the BN backward as TF's autodiff of (Xq - mean) / (var + eps) ** 0.5 (:616,623),
#              Rescale's dgamma / dbeta as fp32 reduce_sums (:689-690), overflow rates as fp32
#              reduce_means of fp32 masks (:63-67).
ARITH = "exact"


# SyncBN (data-parallel parity mode): when set, a callable SYNC(a, b, n) -> (a, b, n) that sums
# a Normalization_q's exact integer statistics over the ranks -- forward (S1 = sum q, S2 = sum q^2, the
# per-channel element count n) and backward (SG = sum G, SGQ = sum G*q) -- so every shard takes the
# WHOLE-batch moments of tf.nn.moments (dynamic_fixed_point.py:588) and their gradient (:616-623): what
# the build's FusedResNet(sync_bn=True) all-reduces inside its step. None: per-shard statistics.
SYNC = None


#   "tf32seq" -- the same fp32 arithmetic in another legitimate order (sequential reductions, per-tap
#              conv GEMMs): a control for how far two fp32 implementations of the reference land
#              from EACH OTHER (TF's CPU and GPU kernels sum in different orders).


def _tf32():
    return ARITH in ("tf32", "tf32seq")


def _seq():
    return ARITH == "tf32seq"


def f32_colsum(a):
    """fp32 sum over the rows of a 2-D array (one value per column): pairwise (numpy's float32
    reduction along a contiguous axis, the class of Eigen's tree reductions), or row after row
    (ARITH "tf32seq")."""
    a = np.asarray(a, F32)
    if _seq():
        return np.add.reduce(a, axis=0, dtype=F32)
    return np.add.reduce(np.ascontiguousarray(a.T), axis=-1, dtype=F32)


def _im2col(x, kh, kw, sh, sw, Ho, Wo, pt, pl, dtype):
    """[N*Ho*Wo, kh*kw*C] patches of x (zero padding), tap-major then channel."""
    N, H, W, C = x.shape
    xp = _windows(x.astype(dtype), kh, kw, sh, sw, Ho, Wo, pt, pl).astype(dtype)
    cols = np.empty((N, Ho, Wo, kh, kw, C), dtype)
    for i in range(kh):
        for j in range(kw):
            cols[:, :, :, i, j, :] = xp[:, i:i + (Ho - 1) * sh + 1:sh, j:j + (Wo - 1) * sw + 1:sw, :]
    return cols.reshape(N * Ho * Wo, kh * kw * C)


def tf_same_pads(in_size, k, s):
    """TF 'SAME' padding (before, after) and output size."""
    out = -(-in_size // s)
    total = max((out - 1) * s + k - in_size, 0)
    return out, total // 2, total - total // 2


def conv_geometry(H, W, kh, kw, sh, sw, padding):
    """(Ho, Wo, pt, pb, pl, pr) for TF 'SAME' / 'VALID' or an explicit symmetric int padding (the torch
    face, ``custom.py:11-12`` ``padding=1``)."""
    if not isinstance(padding, str):
        ph, pw = (padding, padding) if isinstance(padding, int) else padding
        return (H + 2 * ph - kh) // sh + 1, (W + 2 * pw - kw) // sw + 1, ph, ph, pw, pw
    if padding == "SAME":
        Ho, pt, pb = tf_same_pads(H, kh, sh)
        Wo, pl, pr = tf_same_pads(W, kw, sw)
    elif padding == "VALID":
        Ho = -(-(H - kh + 1) // sh)
        Wo = -(-(W - kw + 1) // sw)
        pt = pb = pl = pr = 0
    else:
        raise ValueError(padding)
    return Ho, Wo, pt, pb, pl, pr


def _windows(x, kh, kw, sh, sw, Ho, Wo, pt, pl):
    """x: [N,H,W,C] -> padded input and a function giving the [N,Ho,Wo,C] slice for tap (i,j)."""
    N, H, W, C = x.shape
    Hp = max(H + pt, (Ho - 1) * sh + kh)
    Wp = max(W + pl, (Wo - 1) * sw + kw)
    xp = np.zeros((N, Hp, Wp, C), dtype=np.float64)
    xp[:, pt:pt + H, pl:pl + W, :] = x
    return xp


def conv_fwd_int(xq, wq, strides, padding):
    """Exact integer conv (NHWC x HWIO). Returns int64 [N,Ho,Wo,Cout]."""
    N, H, W, Cin = xq.shape
    kh, kw, _, Cout = wq.shape
    sh, sw = strides
    Ho, Wo, pt, pb, pl, pr = conv_geometry(H, W, kh, kw, sh, sw, padding)
    if _seq():  # per-tap fp32 GEMMs accumulated in fp32
        xp = _windows(xq.astype(F32), kh, kw, sh, sw, Ho, Wo, pt, pl).astype(F32)
        acc = np.zeros((N * Ho * Wo, Cout), dtype=F32)
        for i in range(kh):
            for j in range(kw):
                xs = xp[:, i:i + (Ho - 1) * sh + 1:sh, j:j + (Wo - 1) * sw + 1:sw, :]
                acc += xs.reshape(-1, Cin) @ wq[i, j].astype(F32)
        return acc.astype(np.int64).reshape(N, Ho, Wo, Cout)
    if _tf32():  # tf.nn.conv2d: one fp32 GEMM over K = kh*kw*Cin (sums of integers stay integers)
        cols = _im2col(xq, kh, kw, sh, sw, Ho, Wo, pt, pl, F32)
        acc = cols @ wq.astype(F32).reshape(kh * kw * Cin, Cout)
        return acc.astype(np.int64).reshape(N, Ho, Wo, Cout)
    xp = _windows(xq.astype(np.float64), kh, kw, sh, sw, Ho, Wo, pt, pl)
    acc = np.zeros((N * Ho * Wo, Cout), dtype=np.float64)
    wf = wq.astype(np.float64)
    for i in range(kh):
        for j in range(kw):
            xs = xp[:, i:i + (Ho - 1) * sh + 1:sh, j:j + (Wo - 1) * sw + 1:sw, :]
            acc += xs.reshape(-1, Cin) @ wf[i, j]
    return np.rint(acc).astype(np.int64).reshape(N, Ho, Wo, Cout)


def conv_dgrad_int(gq, wq, strides, padding, in_shape):
    """Exact integer input-gradient of conv_fwd_int. Returns int64 [N,H,W,Cin]."""
    N, H, W, Cin = in_shape
    kh, kw, _, Cout = wq.shape
    sh, sw = strides
    Ho, Wo, pt, pb, pl, pr = conv_geometry(H, W, kh, kw, sh, sw, padding)
    Hp = max(H + pt, (Ho - 1) * sh + kh)
    Wp = max(W + pl, (Wo - 1) * sw + kw)
    dt = F32 if _tf32() else np.float64  # tf32: per-tap fp32 GEMMs over Cout, fp32 col2im adds
    dxp = np.zeros((N, Hp, Wp, Cin), dtype=dt)
    g = gq.astype(dt).reshape(-1, Cout)
    wf = wq.astype(dt)
    for i in range(kh):
        for j in range(kw):
            contrib = (g @ wf[i, j].T).reshape(N, Ho, Wo, Cin)
            dxp[:, i:i + (Ho - 1) * sh + 1:sh, j:j + (Wo - 1) * sw + 1:sw, :] += contrib
    return np.rint(dxp[:, pt:pt + H, pl:pl + W, :]).astype(np.int64)


def conv_wgrad_int(xq, gq, strides, padding, kshape):
    """Exact integer weight-gradient. Returns int64 [kh,kw,Cin,Cout]."""
    N, H, W, Cin = xq.shape
    kh, kw = kshape
    Cout = gq.shape[-1]
    sh, sw = strides
    Ho, Wo, pt, pb, pl, pr = conv_geometry(H, W, kh, kw, sh, sw, padding)
    if _tf32():  # conv2d_backprop_filter: one fp32 GEMM contracting the N*Ho*Wo pixels
        cols = _im2col(xq, kh, kw, sh, sw, Ho, Wo, pt, pl, F32)
        g2 = gq.astype(F32).reshape(-1, Cout)
        if _seq():  # pixel chunks of 4096 accumulated in fp32
            dw = np.zeros((cols.shape[1], Cout), F32)
            for p0 in range(0, cols.shape[0], 4096):
                dw += cols[p0:p0 + 4096].T @ g2[p0:p0 + 4096]
        else:
            dw = cols.T @ g2
        return dw.astype(np.int64).reshape(kh, kw, Cin, Cout)
    xp = _windows(xq.astype(np.float64), kh, kw, sh, sw, Ho, Wo, pt, pl)
    g = gq.astype(np.float64).reshape(-1, Cout)
    dw = np.zeros((kh, kw, Cin, Cout), dtype=np.float64)
    for i in range(kh):
        for j in range(kw):
            xs = xp[:, i:i + (Ho - 1) * sh + 1:sh, j:j + (Wo - 1) * sw + 1:sw, :]
            dw[i, j] = xs.reshape(-1, Cin).T @ g
    return np.rint(dw).astype(np.int64)


FLOAT_BITS = 16  # layers whose quantisers exceed this run on fp32 values (lbt_amd fp32.hip)


def conv_f32(x, w, strides, padding):
    """fp32 conv of float operands, accumulated exactly enough (float64) and rounded once."""
    N, H, W, Cin = x.shape
    kh, kw, _, Cout = w.shape
    sh, sw = strides
    Ho, Wo, pt, pb, pl, pr = conv_geometry(H, W, kh, kw, sh, sw, padding)
    xp = _windows(x.astype(np.float64), kh, kw, sh, sw, Ho, Wo, pt, pl)
    acc = np.zeros((N * Ho * Wo, Cout), dtype=np.float64)
    for i in range(kh):
        for j in range(kw):
            xs = xp[:, i:i + (Ho - 1) * sh + 1:sh, j:j + (Wo - 1) * sw + 1:sw, :]
            acc += xs.reshape(-1, Cin) @ w[i, j].astype(np.float64)
    return acc.reshape(N, Ho, Wo, Cout).astype(F32)


def conv_dgrad_f32(g, w, strides, padding, in_shape):
    N, H, W, Cin = in_shape
    kh, kw, _, Cout = w.shape
    sh, sw = strides
    Ho, Wo, pt, pb, pl, pr = conv_geometry(H, W, kh, kw, sh, sw, padding)
    Hp = max(H + pt, (Ho - 1) * sh + kh)
    Wp = max(W + pl, (Wo - 1) * sw + kw)
    dxp = np.zeros((N, Hp, Wp, Cin), dtype=np.float64)
    gg = g.astype(np.float64).reshape(-1, Cout)
    for i in range(kh):
        for j in range(kw):
            dxp[:, i:i + (Ho - 1) * sh + 1:sh, j:j + (Wo - 1) * sw + 1:sw, :] += \
                (gg @ w[i, j].astype(np.float64).T).reshape(N, Ho, Wo, Cin)
    return dxp[:, pt:pt + H, pl:pl + W, :].astype(F32)


def conv_wgrad_f64(x, g, strides, padding, kshape):
    N, H, W, Cin = x.shape
    kh, kw = kshape
    Cout = g.shape[-1]
    sh, sw = strides
    Ho, Wo, pt, pb, pl, pr = conv_geometry(H, W, kh, kw, sh, sw, padding)
    xp = _windows(x.astype(np.float64), kh, kw, sh, sw, Ho, Wo, pt, pl)
    gg = g.astype(np.float64).reshape(-1, Cout)
    dw = np.zeros((kh, kw, Cin, Cout), dtype=np.float64)
    for i in range(kh):
        for j in range(kw):
            xs = xp[:, i:i + (Ho - 1) * sh + 1:sh, j:j + (Wo - 1) * sw + 1:sw, :]
            dw[i, j] = xs.reshape(-1, Cin).T @ gg
    return dw


def scale_int(acc, e):
    """float32(acc) * 2**-e, the dequant epilogue of every integer GEMM."""
    return (np.asarray(acc).astype(np.float32) * F32(2.0 ** -e)).astype(np.float32)


class Ctx:
    """Per-step quantiser context: exponents I_t, overflow counts, noise key."""

    def __init__(self, ranges, step, seed, target=0.0):
        self.I = ranges            # name -> int exponent (I_t), shared with the model
        self.step = int(step)
        self.seed = int(seed)
        self.target = target
        self.counts = {}           # name -> (c1, c2, n, bits)
        self.rates = {}            # name -> (rate, rate_2x) as fp32 means (ARITH "tf32" only)
        self.record = {}           # name -> int codes (for parity tests)

    def fq(self, name, x, bits, stochastic=True):
        """weight_quantization's fp32 output: the dequantised codes, or x itself at 32 bits (:22-23)."""
        assert 1 <= bits <= 32, "invalid value for bits: %d" % bits
        if bits == 32:
            return np.asarray(x, dtype=np.float32)
        q, e = self.q(name, x, bits, stochastic)
        return dequant_f32(q, e)

    def q(self, name, x, bits, stochastic=True):
        """Quantise with I_t; record overflow counts of x against I_t."""
        x = np.asarray(x, dtype=np.float32)
        I = self.I[name]
        noise = dfxp.noise_for(x.shape, dfxp.qid_of(name), self.step, self.seed) if stochastic else None
        q = dfxp.quantize_int(x, bits, I, stochastic, noise)
        c1, c2 = dfxp.overflow_counts(x, bits, I)
        self.counts[name] = (c1, c2, x.size, bits)
        if _tf32():  # the reference's rates: fp32 reduce_mean of fp32 masks (:63-67)
            self.rates[name] = dfxp.overflow_rates_f32(x, bits, I)
        self.record[name] = q
        return q, dfxp.frac_bits(bits, I)

    def new_ranges(self):
        out = dict(self.I)
        for name, (c1, c2, n, bits) in self.counts.items():
            if name in self.rates:
                r1, r2 = self.rates[name]
                out[name] = dfxp.update_range_from_rates(r1, r2, self.target, bits, self.I[name])
            else:
                out[name] = dfxp.update_range_from_counts(c1, c2, n, self.target, bits, self.I[name])
        return out


class LayerQ:
    def forward(self, X, ctx):
        return X

    def backward(self, g, ctx):
        return g

    def params(self):
        return []

    def range_names(self):
        return []


def _bias_fwd(layer, y, ctx):
    """y + Q(b) (``:198-201``, ``:390-393``): b quantised at bits, noise over b.shape[1:] = () (one
    scalar); fp32 add."""
    bq, eb = ctx.q(layer.name + "/b_range", layer.b, layer.bits)
    return (y + dequant_f32(bq, eb)).astype(F32)


def _bias_bwd(layer, gq, eg):
    """db = sum of the dequantised grad codes over every axis but the last (``:209``, ``:459``),
    from the exact integer sum: float32(float64(S) * 2**-eg)."""
    layer.db_int = gq.reshape(-1, gq.shape[-1]).astype(np.int64).sum(0)
    layer.db = (layer.db_int.astype(np.float64) * 2.0 ** -eg).astype(F32)


def dequant_f32(q, e):
    return (np.asarray(q).astype(F32) * F32(2.0 ** -e)).astype(F32)


class Conv2dQ(LayerQ):
    """The integer weight-gradient numerator of the last backward is kept as ``acc_w`` (int64), and
    its exponent as ``ew_grad`` (e_x + e_g), for the data-parallel oracle (``dp_train_step``)."""

    def __init__(self, name, bits, ksize, strides, padding, weight_decay=0.0, grad_bits=None, weight_bits=None,
                 use_bias=False):
        self.name, self.bits, self.ksize = name, bits, tuple(ksize)
        self.grad_bits = grad_bits or bits
        self.weight_bits = weight_bits or bits  # config 5: 4-bit weights
        self.strides = (strides[1], strides[2]) if len(strides) == 4 else tuple(strides)
        self.padding, self.wd = padding, weight_decay
        self.use_bias = use_bias
        self.W = None
        self.b = np.zeros(self.ksize[3], F32) if use_bias else None
        self.fmode = max(bits + 1, self.grad_bits, self.weight_bits) > FLOAT_BITS

    def range_names(self):
        r = [self.name + "/W_range", self.name + "/X_range", self.name + "/grad_range"]
        return r + ([self.name + "/b_range"] if self.use_bias else [])

    def params(self):
        return [(self.name + "/W", self)] + ([(self.name + "/bias", self)] if self.use_bias else [])

    def forward(self, X, ctx):
        self.in_shape = X.shape
        if self.fmode:  # 17..32-bit quantisers: fp32 operands (X at bits + 1 <= 32, :287-288)
            self.xf = ctx.fq(self.name + "/X_range", X, self.bits + 1)
            self.wf = ctx.fq(self.name + "/W_range", self.W, self.weight_bits)
            y = conv_f32(self.xf, self.wf, self.strides, self.padding)
            if self.use_bias:
                y = (y + ctx.fq(self.name + "/b_range", self.b, self.bits)).astype(F32)
            return y
        self.xq, self.ex = ctx.q(self.name + "/X_range", X, self.bits + 1)
        self.wq, self.ew = ctx.q(self.name + "/W_range", self.W, self.weight_bits)
        acc = conv_fwd_int(self.xq, self.wq, self.strides, self.padding)
        y = scale_int(acc, self.ex + self.ew)
        return _bias_fwd(self, y, ctx) if self.use_bias else y

    def backward(self, g, ctx):
        if self.fmode:
            gf = ctx.fq(self.name + "/grad_range", g, self.grad_bits)
            c = F32(2 * self.wd)
            dw = conv_wgrad_f64(self.xf, gf, self.strides, self.padding, self.ksize[:2]).astype(F32)
            self.dW = (dw + (c * self.W).astype(F32)).astype(F32)
            if self.use_bias:
                self.db = gf.reshape(-1, gf.shape[-1]).astype(np.float64).sum(0).astype(F32)
            return conv_dgrad_f32(gf, self.wf, self.strides, self.padding, self.in_shape)
        gq, eg = ctx.q(self.name + "/grad_range", g, self.grad_bits)
        self.gq = gq
        acc_w = conv_wgrad_int(self.xq, gq, self.strides, self.padding, self.ksize[:2])
        self.acc_w, self.ew_grad = acc_w, self.ex + eg
        c = F32(2 * self.wd)
        self.dW = (scale_int(acc_w, self.ex + eg) + (c * self.W).astype(F32)).astype(F32)
        if self.use_bias:
            _bias_bwd(self, gq, eg)
        acc_x = conv_dgrad_int(gq, self.wq, self.strides, self.padding, self.in_shape)
        return scale_int(acc_x, eg + self.ew)


def _mm(a, b):
    """Integer-code GEMM: exact (float64, partial sums < 2**53), or tf.matmul's fp32 (ARITH tf32)."""
    dt = F32 if _tf32() else np.float64
    return np.asarray(a).astype(dt) @ np.asarray(b).astype(dt)


class DenseQ(LayerQ):
    def __init__(self, name, bits, in_units, units, weight_decay=0.0, grad_bits=None, weight_bits=None,
                 use_bias=False):
        self.name, self.bits, self.in_units, self.units, self.wd = name, bits, in_units, units, weight_decay
        self.grad_bits = grad_bits or bits
        self.weight_bits = weight_bits or bits
        self.use_bias = use_bias
        self.W = None
        self.b = np.zeros(units, F32) if use_bias else None
        self.fmode = max(bits, self.grad_bits, self.weight_bits) > FLOAT_BITS

    def range_names(self):
        r = [self.name + "/W_range", self.name + "/X_range", self.name + "/grad_range"]
        return r + ([self.name + "/b_range"] if self.use_bias else [])

    def params(self):
        return [(self.name + "/W", self)] + ([(self.name + "/bias", self)] if self.use_bias else [])

    def forward(self, X, ctx):
        if self.fmode:
            self.xf = ctx.fq(self.name + "/X_range", X, self.bits)
            self.wf = ctx.fq(self.name + "/W_range", self.W, self.weight_bits)
            y = (self.xf.astype(np.float64) @ self.wf.astype(np.float64)).astype(F32)
            if self.use_bias:
                y = (y + ctx.fq(self.name + "/b_range", self.b, self.bits)).astype(F32)
            return y
        self.xq, self.ex = ctx.q(self.name + "/X_range", X, self.bits)
        self.wq, self.ew = ctx.q(self.name + "/W_range", self.W, self.weight_bits)
        acc = np.rint(_mm(self.xq, self.wq)).astype(np.int64)
        y = scale_int(acc, self.ex + self.ew)
        return _bias_fwd(self, y, ctx) if self.use_bias else y

    def backward(self, g, ctx):
        if self.fmode:
            gf = ctx.fq(self.name + "/grad_range", g, self.grad_bits).astype(np.float64)
            c = F32(2 * self.wd)
            self.dW = ((self.xf.astype(np.float64).T @ gf).astype(F32) + (c * self.W).astype(F32)).astype(F32)
            if self.use_bias:
                self.db = gf.sum(0).astype(F32)
            return (gf @ self.wf.astype(np.float64).T).astype(F32)
        gq, eg = ctx.q(self.name + "/grad_range", g, self.grad_bits)
        self.gq = gq
        acc_w = np.rint(_mm(self.xq.T, gq)).astype(np.int64)
        self.acc_w, self.ew_grad = acc_w, self.ex + eg
        if self.use_bias:
            _bias_bwd(self, gq, eg)
        c = F32(2 * self.wd)
        self.dW = (scale_int(acc_w, self.ex + eg) + (c * self.W).astype(F32)).astype(F32)
        acc_x = np.rint(_mm(gq, self.wq.T)).astype(np.int64)
        return scale_int(acc_x, eg + self.ew)


class NormQ(LayerQ):
    """train False: the testing branch of ``:590-600`` (mean / var = the running averages, which do
    not move; backward dX = Gq / sigma since mean and var are constants of the graph)."""

    def __init__(self, name, bits, num_features, momentum=0.999, eps=1e-5, grad_bits=None):
        self.name, self.bits, self.C = name, bits, num_features
        self.grad_bits = grad_bits or bits
        self.momentum, self.eps = momentum, eps
        self.mean_running = np.zeros(num_features, F32)
        self.var_running = np.ones(num_features, F32)
        self.train = True
        self.fmode = max(bits, self.grad_bits) > FLOAT_BITS

    def range_names(self):
        return [self.name + "/X_range", self.name + "/grad_range"]

    def _forward_f32(self, X, ctx):
        """fp32 input (fake-quantised, or raw at 32 bits): moments from float64 sums (the build's
        fixed-order double sums), the same fp32 normalisation as the integer path."""
        x = ctx.fq(self.name + "/X_range", X, self.bits)
        C = X.shape[-1]
        xf = x.reshape(-1, C).astype(np.float64)
        n = xf.shape[0]
        if self.train:
            mean_d = xf.sum(0) / n
            var_d = (xf * xf).sum(0) / n - mean_d * mean_d
            mu, var = mean_d.astype(F32), var_d.astype(F32)
            m = F32(self.momentum)
            self.mean_running = ((m * self.mean_running).astype(F32) + (F32(1 - self.momentum) * mu).astype(F32)).astype(F32)
            self.var_running = ((m * self.var_running).astype(F32) + (F32(1 - self.momentum) * var).astype(F32)).astype(F32)
        else:
            mu, var = self.mean_running, self.var_running
        sigma = np.sqrt((var + F32(self.eps)).astype(F32)).astype(F32)
        self.xf, self.mu, self.sigma, self.n = x, mu, sigma, n
        return ((x - mu).astype(F32) / sigma).astype(F32)

    def forward(self, X, ctx):
        if self.fmode:
            return self._forward_f32(X, ctx)
        q, e = ctx.q(self.name + "/X_range", X, self.bits)
        s = 2.0 ** -e
        C = X.shape[-1]
        if not self.train:
            mu, var = self.mean_running, self.var_running
            sigma = np.sqrt((var + F32(self.eps)).astype(F32)).astype(F32)
            xhat = (((q.astype(F32) * F32(s)).astype(F32) - mu).astype(F32) / sigma).astype(F32)
            self.q, self.e, self.mu, self.sigma, self.xhat, self.n = q, e, mu, sigma, xhat, q.size // C
            return xhat
        qf = q.reshape(-1, C).astype(np.int64)
        n = qf.shape[0]
        if _tf32():  # tf.nn.moments: fp32 reduce_mean, then reduce_mean of squared_difference (:588)
            xq = (q.astype(F32) * F32(s)).astype(F32)
            x2 = xq.reshape(-1, C)
            mu = (f32_colsum(x2) / F32(n)).astype(F32)
            dd = (x2 - mu).astype(F32)
            var = (f32_colsum((dd * dd).astype(F32)) / F32(n)).astype(F32)
            sigma = np.power((var + F32(self.eps)).astype(F32), F32(0.5)).astype(F32)  # (:616) ** 0.5
            xhat = ((xq - mu).astype(F32) / sigma).astype(F32)
            self.var_tf = var
        else:
            S1 = qf.sum(0)
            S2 = (qf * qf).sum(0)
            if SYNC is not None:
                S1, S2, n = SYNC(S1, S2, n)
            mean_d = S1.astype(np.float64) * s / n
            var_d = S2.astype(np.float64) * (s * s) / n - mean_d * mean_d
            mu = mean_d.astype(F32)
            var = var_d.astype(F32)
            sigma = np.sqrt((var + F32(self.eps)).astype(F32)).astype(F32)
            xhat = (((q.astype(F32) * F32(s)).astype(F32) - mu).astype(F32) / sigma).astype(F32)
        m = F32(self.momentum)
        self.mean_running = ((m * self.mean_running).astype(F32) + (F32(1 - self.momentum) * mu).astype(F32)).astype(F32)
        self.var_running = ((m * self.var_running).astype(F32) + (F32(1 - self.momentum) * var).astype(F32)).astype(F32)
        self.q, self.e, self.mu, self.sigma, self.xhat, self.n = q, e, mu, sigma, xhat, n
        return xhat

    def backward(self, g, ctx):
        if self.fmode:
            gf = ctx.fq(self.name + "/grad_range", g, self.grad_bits)
            if not self.train:
                return (gf / self.sigma).astype(F32)
            C = g.shape[-1]
            g2 = gf.reshape(-1, C).astype(np.float64)
            x2 = self.xf.reshape(-1, C).astype(np.float64)
            Sg, Sgx = g2.sum(0), (g2 * x2).sum(0)
            mg = (Sg / self.n).astype(F32)
            mgx = ((Sgx - self.mu.astype(np.float64) * Sg) / (self.n * self.sigma.astype(np.float64))).astype(F32)
            xhat = ((self.xf - self.mu).astype(F32) / self.sigma).astype(F32)
            a = (gf - mg).astype(F32)
            b = (xhat * mgx).astype(F32)
            return ((a - b).astype(F32) / self.sigma).astype(F32)
        G, eg = ctx.q(self.name + "/grad_range", g, self.grad_bits)
        sg = 2.0 ** -eg
        s = 2.0 ** -self.e
        C = g.shape[-1]
        if not self.train:
            return ((G.astype(F32) * F32(sg)).astype(F32) / self.sigma).astype(F32)
        if _tf32():
            return self._backward_tf32(G, sg, s, C)
        Gf = G.reshape(-1, C).astype(np.int64)
        qf = self.q.reshape(-1, C).astype(np.int64)
        SG = Gf.sum(0)
        SGQ = (Gf * qf).sum(0)
        n = self.n  # (the global count under SYNC: set by the forward)
        if SYNC is not None:
            SG, SGQ, _ = SYNC(SG, SGQ, 0)
        mu_d = self.mu.astype(np.float64)
        sig_d = self.sigma.astype(np.float64)
        mg = (sg * SG.astype(np.float64) / n).astype(F32)
        mgx = (sg * (s * SGQ.astype(np.float64) - mu_d * SG.astype(np.float64)) / (n * sig_d)).astype(F32)
        ghat = (G.astype(F32) * F32(sg)).astype(F32)
        a = (ghat - mg).astype(F32)
        b = (self.xhat * mgx).astype(F32)
        return ((a - b).astype(F32) / self.sigma).astype(F32)


    def _backward_tf32(self, G, sg, s, C):
        """tf.gradients of y = (Xq - mean) / (var + eps) ** 0.5 with (mean, var) = tf.nn.moments(Xq)
        (:588,616,623) in fp32, term by term as TF's gradient functions build it: RealDiv (g / s and
        -sum(g * (-d / s) / s)), Pow (grad * 0.5 * pow(v, -0.5)), Mean (/ n), SquaredDifference
        (2 * grad * (x - mean), mean under stop_gradient), Sub (-sum), the three contributions to
        Xq added in that order."""
        g = (G.astype(F32) * F32(sg)).astype(F32).reshape(-1, C)
        x = (self.q.astype(F32) * F32(s)).astype(F32).reshape(-1, C)
        n = F32(self.n)
        d = (x - self.mu).astype(F32)
        sig = self.sigma
        g_d = (g / sig).astype(F32)
        g_s = f32_colsum((g * (((-d) / sig).astype(F32) / sig).astype(F32)).astype(F32))
        v = (self.var_tf + F32(self.eps)).astype(F32)
        g_v = ((g_s * F32(0.5)).astype(F32) * np.power(v, F32(-0.5)).astype(F32)).astype(F32)
        g_sq = (g_v / n).astype(F32)
        t_sq = ((F32(2.0) * g_sq).astype(F32) * d).astype(F32)
        g_mean = ((-f32_colsum(g_d)).astype(F32) / n).astype(F32)
        dx = ((g_d + t_sq).astype(F32) + g_mean).astype(F32)
        return dx.reshape(G.shape)


class RescaleQ(LayerQ):
    def __init__(self, name, bits, num_features, weight_decay=0.0, grad_bits=None):
        self.name, self.bits, self.C, self.wd = name, bits, num_features, weight_decay
        self.grad_bits = grad_bits or bits
        self.gamma = np.ones(num_features, F32)
        self.beta = np.zeros(num_features, F32)
        self.fmode = max(bits, self.grad_bits) > FLOAT_BITS

    def range_names(self):
        return [self.name + "/g_range", self.name + "/b_range", self.name + "/X_range", self.name + "/grad_range"]

    def params(self):
        return [(self.name + "/g", self), (self.name + "/b", self)]

    def forward(self, X, ctx):
        if self.fmode:
            self.xr = ctx.fq(self.name + "/X_range", X, self.bits)
            self.gq_f = ctx.fq(self.name + "/g_range", self.gamma, self.bits)
            bq_f = ctx.fq(self.name + "/b_range", self.beta, self.bits)
            return ((self.xr * self.gq_f).astype(F32) + bq_f).astype(F32)
        R, er = ctx.q(self.name + "/X_range", X, self.bits)
        gq, eg = ctx.q(self.name + "/g_range", self.gamma, self.bits)
        bq, eb = ctx.q(self.name + "/b_range", self.beta, self.bits)
        self.R, self.er = R, er
        self.gq_f = (gq.astype(F32) * F32(2.0 ** -eg)).astype(F32)
        bq_f = (bq.astype(F32) * F32(2.0 ** -eb)).astype(F32)
        xr = (R.astype(F32) * F32(2.0 ** -er)).astype(F32)
        return ((xr * self.gq_f).astype(F32) + bq_f).astype(F32)

    def backward(self, g, ctx):
        if self.fmode:
            gf = ctx.fq(self.name + "/grad_range", g, self.grad_bits)
            C = g.shape[-1]
            g2 = gf.reshape(-1, C).astype(np.float64)
            c = F32(2 * self.wd)
            self.dgamma = ((g2 * self.xr.reshape(-1, C).astype(np.float64)).sum(0).astype(F32)
                           + (c * self.gamma).astype(F32)).astype(F32)
            self.dbeta = g2.sum(0).astype(F32)
            return (gf * self.gq_f).astype(F32)
        G, eg = ctx.q(self.name + "/grad_range", g, self.grad_bits)
        C = g.shape[-1]
        Gf = G.reshape(-1, C).astype(np.int64)
        Rf = self.R.reshape(-1, C).astype(np.int64)
        sg = 2.0 ** -eg
        sr = 2.0 ** -self.er
        c = F32(2 * self.wd)
        if _tf32():  # Mul / Add gradients: fp32 reduce_sums over the broadcast axes (:689-691)
            ghat = (G.astype(F32) * F32(sg)).astype(F32).reshape(-1, C)
            xr = (self.R.astype(F32) * F32(sr)).astype(F32).reshape(-1, C)
            self.dgamma = (f32_colsum((ghat * xr).astype(F32)) + (c * self.gamma).astype(F32)).astype(F32)
            self.dbeta = f32_colsum(ghat)
            return (ghat * self.gq_f).astype(F32).reshape(G.shape)
        # integer numerators of dgamma / dbeta and their scales, for the data-parallel oracle
        self.sgr, self.sg, self.eg, self.sgsr = (Gf * Rf).sum(0), Gf.sum(0), sg, sg * sr
        self.dgamma = ((Gf * Rf).sum(0).astype(np.float64) * (sg * sr)).astype(F32)
        self.dgamma = (self.dgamma + (c * self.gamma).astype(F32)).astype(F32)
        self.dbeta = (Gf.sum(0).astype(np.float64) * sg).astype(F32)
        ghat = (G.astype(F32) * F32(sg)).astype(F32)
        return (ghat * self.gq_f).astype(F32)


class SequentialQ(LayerQ):
    def __init__(self, *layers):
        self.layers = list(layers)

    def forward(self, X, ctx):
        for l in self.layers:
            X = l.forward(X, ctx)
        return X

    def backward(self, g, ctx):
        for l in reversed(self.layers):
            g = l.backward(g, ctx)
        return g

    def params(self):
        return [p for l in self.layers for p in l.params()]

    def range_names(self):
        return [r for l in self.layers for r in l.range_names()]


def BatchNormQ(name, bits, num_features, weight_decay=0.0, grad_bits=None):
    return SequentialQ(NormQ(name + "-norm", bits, num_features, grad_bits=grad_bits),
                       RescaleQ(name + "-rescale", bits, num_features, weight_decay, grad_bits=grad_bits))


class ReluQ(LayerQ):
    def forward(self, X, ctx):
        self.X = X
        return np.maximum(F32(0), X).astype(F32)

    def backward(self, g, ctx):
        return np.where(self.X > 0, g, F32(0)).astype(F32)


class ResidualBlockQ(LayerQ):
    def __init__(self, name, bits, in_channels, channels, stride, weight_decay=0.0, weight_bits=None):
        wb = dict(weight_bits=weight_bits)
        self.residual = SequentialQ(
            Conv2dQ(name + "-1", bits, [3, 3, in_channels, channels], [1, stride, stride, 1], "SAME", weight_decay,
                    **wb),
            BatchNormQ(name + "-bn1", bits, channels, weight_decay),
            ReluQ(),
            Conv2dQ(name + "-2", bits, [3, 3, channels, channels], [1, 1, 1, 1], "SAME", weight_decay, **wb),
            BatchNormQ(name + "-bn2", bits, channels, weight_decay))
        if stride == 1 and in_channels == channels:
            self.shortcut = SequentialQ()
        else:
            self.shortcut = SequentialQ(
                Conv2dQ(name + "-shortcut", bits, [1, 1, in_channels, channels], [1, stride, stride, 1], "SAME",
                        weight_decay, **wb),
                BatchNormQ(name + "-shortcut-bn", bits, channels, weight_decay))
        self.relu = ReluQ()

    def forward(self, X, ctx):
        y1 = self.residual.forward(X, ctx)
        y2 = self.shortcut.forward(X, ctx)
        return self.relu.forward((y1 + y2).astype(F32), ctx)

    def backward(self, g, ctx):
        g = self.relu.backward(g, ctx)
        g1 = self.residual.backward(g, ctx)
        g2 = self.shortcut.backward(g, ctx)
        return (g1 + g2).astype(F32)

    def params(self):
        return self.residual.params() + self.shortcut.params()

    def range_names(self):
        return self.residual.range_names() + self.shortcut.range_names()


class MaxPoolQ(LayerQ):
    """``MaxPool_q`` (``dynamic_fixed_point.py:993-1006``, ``tf.nn.max_pool``; SAME pads with -inf).
    Backward = TF MaxPoolGrad: each output's gradient goes to the first maximum of its window in
    (kh, kw) order, accumulated per input in ascending output order (fp32, from 0)."""

    def __init__(self, ksize, strides, padding):
        self.kh, self.kw = ksize[1], ksize[2]
        self.sh, self.sw = strides[1], strides[2]
        self.padding = padding

    def forward(self, X, ctx):
        N, H, W, C = X.shape
        Ho, Wo, pt, pb, pl, pr = conv_geometry(H, W, self.kh, self.kw, self.sh, self.sw, self.padding)
        self.shape, self.geom = X.shape, (Ho, Wo, pt, pl)
        y = np.full((N, Ho, Wo, C), -np.inf, F32)
        amax = np.zeros((N, Ho, Wo, C), np.int64)
        for i in range(self.kh):
            for j in range(self.kw):
                for oh in range(Ho):
                    ih = oh * self.sh + i - pt
                    if not 0 <= ih < H:
                        continue
                    for ow in range(Wo):
                        iw = ow * self.sw + j - pl
                        if not 0 <= iw < W:
                            continue
                        v = X[:, ih, iw, :]
                        better = v > y[:, oh, ow, :]
                        y[:, oh, ow, :] = np.where(better, v, y[:, oh, ow, :])
                        amax[:, oh, ow, :] = np.where(better, i * self.kw + j, amax[:, oh, ow, :])
        self.amax = amax
        return y

    def backward(self, g, ctx):
        N, H, W, C = self.shape
        Ho, Wo, pt, pl = self.geom
        dx = np.zeros(self.shape, F32)
        for oh in range(Ho):
            for ow in range(Wo):
                a = self.amax[:, oh, ow, :]
                ih = oh * self.sh - pt + a // self.kw
                iw = ow * self.sw - pl + a % self.kw
                n_idx, c_idx = np.meshgrid(np.arange(N), np.arange(C), indexing="ij")
                dx[n_idx, ih, iw, c_idx] = (dx[n_idx, ih, iw, c_idx] + g[:, oh, ow, :]).astype(F32)
        return dx


class BottleneckQ(ResidualBlockQ):
    """``ResidualBottleneck_q`` (``:878-980``): 1x1 -> BN -> ReLU -> 3x3 (stride) -> BN -> ReLU ->
    1x1 (4x channels) -> BN, shortcut as ``_build_shortcut`` (``:825-856``) with expansion 4."""

    def __init__(self, name, bits, in_channels, channels, stride, weight_decay=0.0, grad_bits=None):
        out = 4 * channels
        gb = dict(grad_bits=grad_bits)
        self.residual = SequentialQ(
            Conv2dQ(name + "-1", bits, [1, 1, in_channels, channels], [1, 1, 1, 1], "SAME", weight_decay, **gb),
            BatchNormQ(name + "-bn1", bits, channels, weight_decay, **gb),
            ReluQ(),
            Conv2dQ(name + "-2", bits, [3, 3, channels, channels], [1, stride, stride, 1], "SAME", weight_decay, **gb),
            BatchNormQ(name + "-bn2", bits, channels, weight_decay, **gb),
            ReluQ(),
            Conv2dQ(name + "-3", bits, [1, 1, channels, out], [1, 1, 1, 1], "SAME", weight_decay, **gb),
            BatchNormQ(name + "-bn3", bits, out, weight_decay, **gb))
        if stride == 1 and in_channels == out:
            self.shortcut = SequentialQ()
        else:
            self.shortcut = SequentialQ(
                Conv2dQ(name + "-shortcut", bits, [1, 1, in_channels, out], [1, stride, stride, 1], "SAME",
                        weight_decay, **gb),
                BatchNormQ(name + "-shortcut-bn", bits, out, weight_decay, **gb))
        self.relu = ReluQ()


class AvgPoolQ(LayerQ):
    """``AvgPool_q`` (``:1009-1022``, tf.nn.avg_pool). Global (no ksize, or a VALID window equal to
    the map -- the ResNets' 8x8 pool): sequential fp32 sum then * 1/(H*W). Any other window:
    fp32 sum of the window's valid inputs in (kh, kw) order / count of valid positions (TF SAME
    leaves the padding out of the mean); backward: each input adds g[o] / count[o] over the windows
    holding it in ascending output order (TF AvgPoolGrad)."""

    def __init__(self, ksize=None, strides=None, padding="VALID"):
        self.ksize, self.strides, self.padding = ksize, strides, padding

    def _global(self, H, W):
        return self.ksize is None or (self.padding == "VALID" and self.ksize[1] == H and self.ksize[2] == W)

    def forward(self, X, ctx):
        N, H, W, C = X.shape
        self.shape = X.shape
        if not self._global(H, W):
            return self._forward_window(X)
        xs = X.reshape(N, H * W, C)
        acc = np.zeros((N, C), F32)
        for i in range(H * W):
            acc = (acc + xs[:, i, :]).astype(F32)
        return (acc * F32(1.0 / (H * W))).astype(F32).reshape(N, 1, 1, C)

    def _geom(self, H, W):
        kh, kw, sh, sw = self.ksize[1], self.ksize[2], self.strides[1], self.strides[2]
        Ho, Wo, pt, _, pl, _ = conv_geometry(H, W, kh, kw, sh, sw, self.padding)
        cnt = np.zeros((Ho, Wo), F32)
        for oh in range(Ho):
            for ow in range(Wo):
                rh = sum(0 <= oh * sh + i - pt < H for i in range(kh))
                rw = sum(0 <= ow * sw + j - pl < W for j in range(kw))
                cnt[oh, ow] = rh * rw
        return kh, kw, sh, sw, Ho, Wo, pt, pl, cnt

    def _forward_window(self, X):
        N, H, W, C = X.shape
        kh, kw, sh, sw, Ho, Wo, pt, pl, cnt = self._geom(H, W)
        acc = np.zeros((N, Ho, Wo, C), F32)
        for i in range(kh):
            for j in range(kw):
                for oh in range(Ho):
                    ih = oh * sh + i - pt
                    if not 0 <= ih < H:
                        continue
                    for ow in range(Wo):
                        iw = ow * sw + j - pl
                        if 0 <= iw < W:
                            acc[:, oh, ow, :] = (acc[:, oh, ow, :] + X[:, ih, iw, :]).astype(F32)
        return (acc / cnt[None, :, :, None]).astype(F32)

    def backward(self, g, ctx):
        N, H, W, C = self.shape
        if not self._global(H, W):
            kh, kw, sh, sw, Ho, Wo, pt, pl, cnt = self._geom(H, W)
            share = (g / cnt[None, :, :, None]).astype(F32)
            dx = np.zeros(self.shape, F32)
            for oh in range(Ho):
                for ow in range(Wo):
                    for i in range(kh):
                        ih = oh * sh + i - pt
                        if not 0 <= ih < H:
                            continue
                        for j in range(kw):
                            iw = ow * sw + j - pl
                            if 0 <= iw < W:
                                dx[:, ih, iw, :] = (dx[:, ih, iw, :] + share[:, oh, ow, :]).astype(F32)
            return dx
        return np.broadcast_to((g.reshape(N, 1, 1, C) * F32(1.0 / (H * W))).astype(F32), self.shape).copy()


class FlattenQ(LayerQ):
    def __init__(self, dim):
        self.dim = dim

    def forward(self, X, ctx):
        self.shape = X.shape
        return X.reshape(-1, self.dim)

    def backward(self, g, ctx):
        return g.reshape(self.shape)


def softmax_xent(logits, labels, norm=None):
    """mean sparse softmax cross-entropy (``models.py:30-32``) and d loss / d logits, fp32.
    norm: the batch the mean is over (default: these rows). A data-parallel shard passes the GLOBAL
    batch, so its loss is its share of the global mean and dz its rows of the global gradient."""
    z = logits.astype(F32)
    N = z.shape[0] if norm is None else int(norm)
    m = z.max(axis=1, keepdims=True)
    ez = np.exp((z - m).astype(F32)).astype(F32)
    s = ez.sum(axis=1, keepdims=True, dtype=F32)
    p = (ez / s).astype(F32)
    lse = (np.log(s).astype(F32) + m).astype(F32)
    rows = np.arange(z.shape[0])
    loss = float(np.sum((lse[:, 0] - z[rows, labels]).astype(np.float64)) / N)
    onehot = np.zeros_like(p)
    onehot[rows, labels] = 1
    dz = ((p - onehot).astype(F32) / F32(N)).astype(F32)
    return loss, dz
