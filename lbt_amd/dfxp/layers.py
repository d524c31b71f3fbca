"""The reference's quantised-layer API (``dynamic_fixed_point.py:97-1053``) on the gfx950 kernels.

Same class names, constructor signatures and ``Layer_q`` protocol as the reference:
``forward(X) -> y``, ``backward(grad, stochastic) -> dX``, ``grads_and_vars() -> [(dW, W)]``,
``info() -> str``. Tensors are CUDA (HIP) torch tensors in the reference's layouts: NHWC
activations, HWIO conv weights, ``[in, out]`` dense weights.

Differences from TF (documented in DESIGN.md):
* Range variables are slots of a device-resident :class:`~lbt_amd.runtime.DfxpContext`
  (``layer.X_range`` etc. are :class:`~lbt_amd.runtime.Quantizer` objects); their updates are
  applied by ``ctx.update_range_op()`` -- the reference's ``'update_range'`` collection.
* Quantised operands are kept as integer codes (int8 / offset-uint8 / int16) plus the shared
  exponent; the convolutions and matmuls run as exact integer GEMMs.
* Outputs live in per-layer buffers that are reused every step (static-graph semantics).
* ``Conv2d_q(..., input_nonnegative=True)`` declares a post-ReLU input: its (bits+1)-bit codes
  are unsigned and take the int8 MFMA path; otherwise the signed codes take the VALU path.
"""
import contextlib
import os

import numpy as np
import torch

from .. import _lib
from .._lib import NO_Q, OUT_F32, OUT_I8, OUT_I16, OUT_U8OFF, BnNorm, BwdBranch, ChainBranch, ChainBwdA, \
    ChainBwdB, ChainFwd, ptr
from ..runtime import default_context, qid_of
from . import ops


def _rng(ctx, name):
    return np.random.default_rng([ctx.seed & 0xFFFFFFFF, qid_of(name)])


class _Cache:
    """Per-layer device buffers, allocated on first use for a given shape and then reused."""

    def __init__(self):
        self.d = {}

    def sums(self, key, n, ctx):
        """An int64 reduction buffer from the context's sums arena, zeroed before use (unless a
        Trainer zeroes the whole arena once per step)."""
        t = self.d.get(key)
        if t is None or t.numel() < n:
            t = ctx.alloc_sums(n)
            self.d[key] = t
        t = t[:n]
        if not ctx.sums_managed:
            t.zero_()
        return t

    def get(self, key, shape, dtype, device, zero=False):
        t = self.d.get(key)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
            t = (torch.zeros if zero else torch.empty)(tuple(shape), dtype=dtype, device=device)
            self.d[key] = t
        return t


# ---- side stream for work nothing later in the backward reads (weight gradients, BN dgamma /
# dbeta): it runs concurrently with the dgrad / BN chain that is the backward's critical path.
# Contract: the OUTERMOST backward joins it before returning (backward_scope), so the caller of any
# layer's backward -- Model.backward, a user Sequential_q, or block.backward called directly --
# finds finished gradients on its stream. Side streams and pending joins are keyed by the main
# stream that forked them: one model's join never waits on, or clears, another stream's work.
# SIDE_STREAM is read once from LBT_SIDE_STREAM (0 = one stream); assign the attribute to change
# it (a HIP graph captured earlier keeps the schedule it was captured with). Off by default since
# round 4's fused epilogues: the forked graph measured 36.23 ms/step against 35.84 on one stream
# (ResNet-50, B=256, profiles/r10_side_stream_r50.txt); LBT_SIDE_STREAM=1 turns it back on.
SIDE_STREAM = os.environ.get("LBT_SIDE_STREAM", "0") == "1"
# ResidualBottleneck_q: bn1 / bn2's pass A inside conv-2 / conv-3's dgrad (ops.conv_dgrad_igemm_bna);
# LBT_DGRAD_BNA_PY=0: the separate dgrad + pass A launches (A/B, and the C-side LBT_DGRAD_BNA=0 keeps
# the entry point but never fuses)
DGRAD_BNA = os.environ.get("LBT_DGRAD_BNA_PY", "1") != "0"
# ... and bn3 (+ the projection shortcut's BN) pass A inside the NEXT block's conv-1 dgrad
# (ops.conv_dgrad_igemm_bn3): the next block hands back _DgradIn instead of its conv-1 dx
DGRAD_BN3 = os.environ.get("LBT_DGRAD_BN3_PY", "1") != "0"
# ... and the forward chains read their BN's moments from one lbt_bn_moments launch (nrm.ms_in)
CHAIN_MS = os.environ.get("LBT_CHAIN_MS", "1") != "0"


class _DgradIn:
    """A fused bottleneck's input gradient, not yet formed: conv's dgrad of the int16 codes gq (its
    conv-1) plus `other` (its shortcut branch's gradient). The previous fused block evaluates it with
    its own entry pass A in the dgrad's epilogue (ResidualBottleneck_q._entry_from_dgrad)."""

    def __init__(self, conv, gq, other):
        self.conv, self.gq, self.other = conv, gq, other
_SIDE = {}
_PENDING = {}
_DEPTH = [0]


def _stream_key(s):
    return (s.device, s.cuda_stream)


@contextlib.contextmanager
def side_work():
    main = torch.cuda.current_stream()
    if not SIDE_STREAM:
        yield
        return
    key = _stream_key(main)
    side = _SIDE.get(key)
    if side is None:
        side = _SIDE[key] = torch.cuda.Stream(device=main.device)
    side.wait_stream(main)  # its inputs were produced on the main stream
    # registered before anything is queued on it: a launch wrapper that raises part-way still
    # leaves the main stream joined to whatever it did queue
    _PENDING.setdefault(key, set()).add(side)
    with torch.cuda.stream(side):
        yield


def join_side_work():
    """Make the current stream wait for every side_work launch it forked so far."""
    main = torch.cuda.current_stream()
    pend = _PENDING.pop(_stream_key(main), None)
    for s in pend or ():
        main.wait_stream(s)


@contextlib.contextmanager
def backward_scope():
    """Wrap a backward: nested scopes (a block inside Model.backward) keep overlapping; the
    outermost one joins the side stream before returning, also when the backward raises."""
    _DEPTH[0] += 1
    try:
        yield
    finally:
        _DEPTH[0] -= 1
        if _DEPTH[0] == 0:
            join_side_work()


def _as_param(t, ctx):
    return torch.as_tensor(t, dtype=torch.float32).to(ctx.device).contiguous()


# ---- 17..32-bit quantisers (fp32.hip): weight_quantization's domain is 1 <= bits <= 32
# (dynamic_fixed_point.py:21-23). Above 16 bits the integer codes no longer fit the int8 / int16 GEMM
# operands; the quantiser then writes the fake-quantised fp32 values (the reference's own STE
# output) and the layer contracts fp32 operands (fp32.hip), as TF does. bits == 32 is the bypass:
# the tensor itself, no range update (:22-23).
FLOAT_BITS = 16  # a layer whose quantisers exceed this many bits runs in float mode


def _check_bits(bits):
    assert 1 <= bits <= 32, "invalid value for bits: %d" % bits  # the reference's own assertion (:21)


def _fq(x, q, cache, key):
    """weight_quantization(x) as fp32 values: the quantiser's fake-quant output, or x itself at 32 bits."""
    _check_bits(q.bits)
    if q.bits == 32:
        return x.contiguous()
    x = x.contiguous()
    return ops.quantize(x, q, OUT_F32, out=cache.get(key, x.shape, torch.float32, x.device))


_FSPLIT = 64  # pixel / row splits of the fp32 reductions (fixed: deterministic double sums)


def _chan_sums(a, b, C, cache, key):
    rows = a.numel() // C
    part = cache.get(key, (_FSPLIT, 2 * C), torch.float64, a.device)
    _lib.call("lbt_chan_sums_f32", ptr(a), ptr(b), rows, C, _FSPLIT, ptr(part), _lib.stream())
    return part


def _conv_f32(xq, wq, d, y):
    _lib.call("lbt_conv_fwd_f32", ptr(xq), ptr(wq), d, ptr(y), _lib.stream())


def _conv_bwd_f32(layer, gq, d, dev):
    """dW (+ 2*wd*W), db, dX of a float-mode conv / dense (layer.xq, layer.wq: its fp32 operands)."""
    K = d.KH * d.KW * d.Cin
    slab = layer._c.get("fslab", (_FSPLIT, K, d.Cout), torch.float64, dev)
    _lib.call("lbt_conv_wgrad_f32", ptr(layer.xq), ptr(gq), d, ptr(slab), _FSPLIT, _lib.stream())
    _lib.call("lbt_conv_wgrad_reduce_f32", ptr(slab), _FSPLIT, K * d.Cout, ptr(layer.W), ops.f32(2 * layer.weight_decay),
              ptr(layer.dW), _lib.stream())
    if layer.use_bias:
        part = _chan_sums(gq, None, d.Cout, layer._c, "bpart")
        scratch = layer._c.get("bscr", (d.Cout,), torch.float32, dev)
        _lib.call("lbt_affine_grads_f32", ptr(part), _FSPLIT, d.Cout, ptr(layer.b), 0.0, ptr(scratch), ptr(layer.db),
                  _lib.stream())
    if not getattr(layer, "need_input_grad", True):
        return None
    dx = layer._c.get("dx", (d.N, d.H, d.W, d.Cin), torch.float32, dev)
    _lib.call("lbt_conv_dgrad_f32", ptr(gq), ptr(layer.wq), d, ptr(dx), None, _lib.stream())
    return dx


class Layer_q:
    """Base class: identity forward, gradient pass-through backward (``:97-126``)."""
    _batched_q = False  # parameters quantised by the model's batched prologue (Model.forward)

    def forward(self, X):
        self.X = X
        self.y = X
        return self.y

    def backward(self, grad, stochastic=True):
        return grad

    def grads_and_vars(self):
        return []

    def param_slots(self):
        """[(owner, var_attr, grad_attr)] -- used to bind parameters into flat buffers."""
        return []

    def info(self):
        return "quantized layer (default identity)"


class Conv2d_q(Layer_q):
    """Quantised 2-D convolution (``:224-316``): Xq at bits+1, Wq / bq / gradq at bits."""

    def __init__(self, name, bits, ksize, strides, padding, use_bias=True, weight_decay=0,
                 target_overflow_rate=0, input_range=2, weight_range=2, bias_range=2, grad_range=2,
                 input_nonnegative=False, grad_bits=None, weight_bits=None, ctx=None):
        self.ctx = ctx = ctx or default_context()
        h, w, Cin, Cout = self.ksize = list(ksize)
        self.grad_bits = grad_bits = grad_bits or bits  # config 4: 16-bit gradients (the reference: one `bits`)
        self.weight_bits = weight_bits = weight_bits or bits  # config 5: 4-bit weights
        self.strides = list(strides)
        self.padding = padding
        self.name, self.use_bias, self.bits = name, use_bias, bits
        self.target_overflow_rate, self.weight_decay = target_overflow_rate, weight_decay
        self.input_nonnegative = input_nonnegative
        self.need_input_grad = True  # the model clears it for its first layer (TF prunes that dX)
        # float mode: a quantiser beyond 16 bits (X at bits + 1: bits >= 16; at bits == 32 the X
        # quantiser is 33 bits and the reference's assertion fires in forward, :21,287-288)
        self.fmode = max(bits + 1, grad_bits or bits, weight_bits or bits) > FLOAT_BITS
        limit = (3 / (h * w * Cin)) ** 0.5
        self.W = _as_param(_rng(ctx, name + "/W").uniform(-limit, limit, size=ksize).astype(np.float32), ctx)
        self.dW = torch.zeros_like(self.W)
        t = target_overflow_rate
        self.W_range = ctx.quantizer(name + "/W_range", weight_bits, weight_range, t)
        self.X_range = ctx.quantizer(name + "/X_range", min(bits + 1, 32), input_range, t)
        self.grad_range = ctx.quantizer(name + "/grad_range", grad_bits, grad_range, t)
        if use_bias:
            self.b = torch.zeros(Cout, dtype=torch.float32, device=ctx.device)
            self.db = torch.zeros_like(self.b)
            self.b_range = ctx.quantizer(name + "/b_range", bits, bias_range, t)
        if self.fmode:
            self.mfma = self.igemm_w = self.igemm_f = self.igemm_d = self.x_mfma = self.w4 = False
            self.x_kind = OUT_F32
            self._c = _Cache()
            return
        # int8 MFMA kernels: 8-bit codes on both GEMM sides (16-bit gradients: generic int64 kernels)
        self.mfma = ops.mfma_ok(Cin, Cout) and bits <= 8 and grad_bits <= 8
        # x codes: unsigned 9-bit (offset int8, MFMA) / signed <= 8 bit (int8, MFMA) / int16 (VALU)
        # wide layers (channels beyond the register-resident MFMA kernels, or 16-bit gradients):
        # LDS-tiled MFMA implicit GEMMs (igemm.hip) -- the weight gradient too when the input is a
        # post-ReLU 9-bit code (offset int8) and both channel counts are multiples of 64
        self.igemm_w = (not self.mfma and input_nonnegative and bits + 1 == 9 and Cin % 64 == 0
                        and Cout % 64 == 0)
        if bits + 1 <= 8:
            self.x_kind = OUT_I8
        elif bits + 1 == 9 and input_nonnegative and (self.mfma or self.igemm_w):
            self.x_kind = OUT_U8OFF  # offset codes are undone by the MFMA kernels only
        else:
            self.x_kind = OUT_I16
        self.x_mfma = self.mfma and self.x_kind != OUT_I16
        self.igemm_f = not self.x_mfma and ops.igemm_ok(Cin, Cout)
        self.igemm_d = not self.mfma and ops.igemm_ok(Cout, Cin)
        self.ksf = ops.packed_slices(h, w, Cin)
        self.ksd = ops.packed_slices(h, w, Cout)
        dev = ctx.device
        self.w_hwio = torch.zeros(ksize, dtype=torch.int8, device=dev)
        self.wf = torch.zeros((Cout, self.ksf * 16), dtype=torch.int8, device=dev)
        self.wd = torch.zeros((Cin, self.ksd * 16), dtype=torch.int8, device=dev)
        self.wcolsum = torch.zeros(Cout, dtype=torch.int32, device=dev)
        # W4 (weight_bits <= 4): the MFMA kernels read the packed images, two codes per byte
        self.w4 = self.mfma and weight_bits <= 4
        if self.w4:
            self.wf4 = torch.zeros((Cout, self.ksf * 8), dtype=torch.uint8, device=dev)
            self.wd4 = torch.zeros((Cin, self.ksd * 8), dtype=torch.uint8, device=dev)
        self._c = _Cache()

    def param_slots(self):
        s = [(self, "W", "dW")]
        if self.use_bias:
            s.append((self, "b", "db"))
        return s

    def stem(self, d):
        """int16 (9..12-bit) input codes and a small patch: the fp16-MFMA stem kernels."""
        return self.x_kind == OUT_I16 and self.X_range.bits <= 12 and self.bits <= 8 and ops.stem_ok(d)

    def stem_wide(self, d):
        """Signed <= 9-bit image codes and a large patch (the ImageNet conv1, 7x7x3): stem_wide.hip."""
        return (self.x_kind == OUT_I16 and not self.stem(d)
                and ops.stem_wide_ok(d, self.X_range.bits, self.weight_bits))

    def _wgrad_stem_wide(self):
        d = self.d
        K = d.KH * d.KW * d.Cin
        ns = ops.stem_wide_nsplit(d)
        slab = self._c.get("stemw_slab", (ns, K, d.Cout), torch.int64, self.ctx.device)
        ops.conv_stem_wide_wgrad(self.xq, self.X_range.bits, self.gradq, d, slab, ns)
        ops.conv_wgrad_reduce64(slab, ns, K, d.Cout, self.X_range.desc, self.grad_range.desc, self.W,
                                ops.f32(2 * self.weight_decay), self.dW)

    def fwd_codes(self, xq, N, H, W):
        """Forward from X codes the caller already quantised with self.X_range (offset int8,
        x_kind U8OFF): the LDS-tiled int8-MFMA implicit GEMM -> fp32 y (a fused block's conv)."""
        kh, kw, Cin, Cout = self.ksize
        self.d = d = ops.conv_desc(N, H, W, Cin, Cout, kh, kw, self.strides[1], self.strides[2], self.padding)
        self.xq = xq
        self.quantize_weights()
        y = self._c.get("y", (N, d.Ho, d.Wo, Cout), torch.float32, xq.device)
        ops.conv_fwd_igemm_ws(xq, 1, self.wf, self.ksf, d, self.X_range.desc, self.W_range.desc, y,
                              self._ws(d, 0, False))
        self.y = y
        return y

    def _ws(self, d, mode, a16):
        """Split-K workspace of this conv's wide GEMM (None when it does not split)."""
        n = ops.igemm_workspace_bytes(d, mode, a16)
        if n == 0:
            return None
        return self._c.get("ws%d" % mode, ((n + 3) // 4,), torch.int32, self.ctx.device)

    def bwd_codes16(self, gq16, add_src=None):
        """Backward from int16 gradient codes the caller already quantised with self.grad_range:
        wide MFMA wgrad (+ reduce) and dgrad (dx + add_src, the other branch's gradient)."""
        self.gradq = gq16
        with backward_scope():
            with side_work():  # dW is read only by the optimizer: off the dgrad chain's critical path
                self._wgrad_igemm(1)
            if not self.need_input_grad:
                return None
            d = self.d
            dx = self._c.get("dx", (d.N, d.H, d.W, d.Cin), torch.float32, gq16.device)
            ops.conv_dgrad_igemm_ws(gq16, 1, self.wd, self.ksd, d, self.grad_range.desc, self.W_range.desc, dx,
                                    self._ws(d, 1, True), add_src=add_src)
            return dx

    def quantize_weights(self):
        if self._batched_q and self.ctx.params_ready:
            return  # done by the model's batched prologue this step
        ops.quantize_weight(self.W, self.W_range, w_hwio=self.w_hwio,
                            wf=self.wf if (self.mfma or self.igemm_f) else None, ksf=self.ksf,
                            wd=self.wd if (self.mfma or self.igemm_d) else None, ksd=self.ksd,
                            colsum=self.wcolsum if self.mfma else None)
        if self.w4:
            ops.pack_int4(self.wf, self.wf4)
            ops.pack_int4(self.wd, self.wd4)

    def _forward_f32(self, X):
        _check_bits(self.bits + 1)  # bits == 32: the reference quantises X at 33 bits and asserts (:287-288)
        N, H, W, Cin = X.shape
        kh, kw, _, Cout = self.ksize
        self.d = d = ops.conv_desc(N, H, W, Cin, Cout, kh, kw, self.strides[1], self.strides[2], self.padding)
        self.xq = _fq(X, self.X_range, self._c, "xq")
        self.wq = _fq(self.W, self.W_range, self._c, "wq")
        y = self._c.get("y", (N, d.Ho, d.Wo, Cout), torch.float32, X.device)
        _conv_f32(self.xq, self.wq, d, y)
        if self.use_bias:
            ops.bias_add(y, _fq(self.b, self.b_range, self._c, "bq"), Cout)
        self.y = y
        return y

    def forward(self, X):
        self.X = X
        if self.fmode:
            return self._forward_f32(X)
        N, H, W, Cin = X.shape
        kh, kw, _, Cout = self.ksize
        self.d = d = ops.conv_desc(N, H, W, Cin, Cout, kh, kw, self.strides[1], self.strides[2], self.padding)
        self.xq = ops.quantize(X, self.X_range, self.x_kind, out=self._c.get("xq", X.shape, ops.out_dtype(self.x_kind),
                                                                                X.device))
        self.quantize_weights()
        y = self._c.get("y", (N, d.Ho, d.Wo, Cout), torch.float32, X.device)
        if self.x_mfma and self.w4:
            ops.conv_fwd_i8w4(self.xq, self.x_kind == OUT_U8OFF, self.wf4, self.ksf, self.wcolsum, d,
                              self.X_range.desc, self.W_range.desc, y)
        elif self.x_mfma:
            ops.conv_fwd_i8(self.xq, self.x_kind == OUT_U8OFF, self.wf, self.ksf, self.wcolsum, d,
                            self.X_range.desc, self.W_range.desc, y=y)
        elif self.stem(d):
            ops.conv_stem_fwd(self.xq, self.w_hwio, d, self.X_range.desc, self.W_range.desc, y=y)
        elif self.stem_wide(d):
            ops.conv_stem_wide_fwd(self.xq, self.w_hwio, d, self.X_range.desc, self.W_range.desc, y)
        elif self.igemm_f:
            a_kind = 2 if self.x_kind == OUT_I16 else (1 if self.x_kind == OUT_U8OFF else 0)
            ops.conv_fwd_igemm(self.xq, a_kind, self.wf, self.ksf, d, self.X_range.desc, self.W_range.desc, y)
        else:
            ops.conv_fwd_generic(self.xq, self.x_kind == OUT_I16, self.w_hwio, d, self.X_range.desc,
                                 self.W_range.desc, y)
        if self.use_bias:
            self.bq = ops.quantize(self.b, self.b_range, OUT_F32, out=self._c.get("bq", (Cout,), torch.float32,
                                                                                   X.device))
            ops.bias_add(y, self.bq, Cout)
        self.y = y
        return y

    def _backward_wide(self, grad):
        """9..16-bit gradient codes (config 4): int16 codes, int64 generic GEMMs."""
        d = self.d
        dev = grad.device
        K = d.KH * d.KW * d.Cin
        # db = sum of the quantised gradient per channel (:303-304): the quantiser's exact channel sums
        gsum = self._c.sums("gsum", ops.NSHARD * 2 * d.Cout, self.ctx) if self.use_bias else None
        self.gradq = ops.quantize(grad, self.grad_range, OUT_I16, out=self._c.get("gq16", grad.shape, torch.int16, dev),
                                  chsum=gsum, C=d.Cout if self.use_bias else 0)
        if self.use_bias:
            ops.bias_grad(gsum, d.Cout, self.grad_range.desc, self.db)
        if self.igemm_w:
            self._wgrad_igemm(1)
        elif self.stem_wide(d):
            self._wgrad_stem_wide()
        else:
            ns = ops.wgrad_nsplit(d, generic=True)
            slab = self._c.get("slab64", (ns, K, d.Cout), torch.int64, dev)
            ops.conv_wgrad_generic16(self.xq, self.x_kind == OUT_I16, self.gradq, d, slab, ns)
            ops.conv_wgrad_reduce64(slab, ns, K, d.Cout, self.X_range.desc, self.grad_range.desc, self.W,
                                    ops.f32(2 * self.weight_decay), self.dW)
        if not self.need_input_grad:
            return None
        dx = self._c.get("dx", (d.N, d.H, d.W, d.Cin), torch.float32, dev)
        if self.igemm_d:
            ops.conv_dgrad_igemm(self.gradq, 1, self.wd, self.ksd, d, self.grad_range.desc, self.W_range.desc, dx)
        else:
            ops.conv_dgrad_generic16(self.gradq, self.w_hwio, d, self.grad_range.desc, self.W_range.desc, dx)
        return dx

    def _wgrad_igemm(self, g_i16):
        """Weight gradient on the wide-layer MFMA kernel (int64 slab, one shard) + its reduce."""
        d = self.d
        K = d.KH * d.KW * d.Cin
        ns = ops.wgrad_store_nsplit(d, g_i16)
        slab = self._c.get("wslab64", (ns, K, d.Cout), torch.int64, self.ctx.device)  # fully written
        ops.conv_wgrad_igemm_store(self.xq, self.gradq, g_i16, d, slab, ns)
        ops.conv_wgrad_reduce64(slab, ns, K, d.Cout, self.X_range.desc, self.grad_range.desc, self.W,
                                ops.f32(2 * self.weight_decay), self.dW)

    def backward(self, grad, stochastic=True):
        if self.fmode:
            self.gradq = _fq(grad, self.grad_range, self._c, "gq")
            return _conv_bwd_f32(self, self.gradq, self.d, grad.device)
        if self.grad_bits > 8:
            return self._backward_wide(grad)
        d = self.d
        Cout, Cin = d.Cout, d.Cin
        dev = grad.device
        gsum = self._c.sums("gsum", ops.NSHARD * 2 * Cout, self.ctx)
        self.gradq = ops.quantize(grad, self.grad_range, OUT_I8, out=self._c.get("gq", grad.shape, torch.int8, dev),
                                  chsum=gsum, C=Cout)
        wd2 = ops.f32(2 * self.weight_decay)
        K = d.KH * d.KW * Cin
        if self.igemm_w:
            self._wgrad_igemm(0)
            slab = None
        elif self.x_mfma:
            nsplit, ns, slab = ops.wgrad_slab(self._c, "wslab", d, self.ctx)
            ops.conv_wgrad_i8(self.xq, self.x_kind == OUT_U8OFF, self.gradq, d, slab, nsplit, ns)
        elif self.stem(d):
            ns, slab = ops.stem_slab(self._c, "stem_slab", d, self.ctx)
            ops.conv_stem_wgrad(self.xq, self.gradq, d, slab, ns)
        elif self.stem_wide(d):
            self._wgrad_stem_wide()
            slab = None
        else:
            ns = ops.wgrad_nsplit(d, generic=True)
            slab = self._c.get("slab", (ns, K, Cout), torch.int32, dev)
            ops.conv_wgrad_generic(self.xq, self.x_kind == OUT_I16, self.gradq, d, slab, ns)
        if slab is not None:
            ops.conv_wgrad_reduce(slab, ns, K, Cout, self.x_kind == OUT_U8OFF, gsum, self.X_range.desc,
                                  self.grad_range.desc, self.W, wd2, self.dW)
        if self.use_bias:
            ops.bias_grad(gsum, Cout, self.grad_range.desc, self.db)
        if not self.need_input_grad:
            return None
        dx = self._c.get("dx", (d.N, d.H, d.W, Cin), torch.float32, dev)
        if self.w4:
            ops.conv_dgrad_i8w4(self.gradq, self.wd4, self.ksd, d, self.grad_range.desc, self.W_range.desc, dx)
        elif self.mfma:
            ops.conv_dgrad_i8(self.gradq, self.wd, self.ksd, d, self.grad_range.desc, self.W_range.desc, dx)
        elif self.igemm_d:
            ops.conv_dgrad_igemm(self.gradq, 0, self.wd, self.ksd, d, self.grad_range.desc, self.W_range.desc, dx)
        else:
            ops.conv_dgrad_generic(self.gradq, self.w_hwio, d, self.grad_range.desc, self.W_range.desc, dx)
        return dx

    def grads_and_vars(self):
        if self.use_bias:
            return [(self.dW, self.W), (self.db, self.b)]
        return [(self.dW, self.W)]

    def info(self):
        return "%d bits conv2d: %dx%dx%d stride %dx%d pad %s weight_decay %f" % (
            self.bits, self.ksize[0], self.ksize[1], self.ksize[3],
            self.strides[1], self.strides[2], self.padding, self.weight_decay)


Conv2d_pq = Conv2d_q  # byte-identical copy in the reference (``:129-221``)


class Dense_q(Layer_q):
    """Quantised fully-connected layer (``:319-470``): X, W, b and grad all at bits."""

    def __init__(self, name, bits, in_units, units, use_bias=True, weight_decay=0,
                 target_overflow_rate=0, input_range=2, weight_range=2, bias_range=2, grad_range=2, grad_bits=None,
                 weight_bits=None, ctx=None):
        self.ctx = ctx = ctx or default_context()
        self.name, self.bits, self.in_units, self.units = name, bits, in_units, units
        self.grad_bits = grad_bits = grad_bits or bits
        self.weight_bits = weight_bits = weight_bits or bits
        self.use_bias, self.weight_decay, self.target_overflow_rate = use_bias, weight_decay, target_overflow_rate
        limit = (6 / (in_units + units)) ** 0.5
        self.W = _as_param(_rng(ctx, name + "/W").uniform(-limit, limit, size=(in_units, units)).astype(np.float32),
                           ctx)
        self.dW = torch.zeros_like(self.W)
        t = target_overflow_rate
        self.W_range = ctx.quantizer(name + "/W_range", weight_bits, weight_range, t)
        self.X_range = ctx.quantizer(name + "/X_range", bits, input_range, t)
        self.grad_range = ctx.quantizer(name + "/grad_range", grad_bits, grad_range, t)
        if use_bias:
            self.b = torch.zeros(units, dtype=torch.float32, device=ctx.device)
            self.db = torch.zeros_like(self.b)
            self.b_range = ctx.quantizer(name + "/b_range", bits, bias_range, t)
        self.fmode = max(bits, grad_bits, weight_bits) > FLOAT_BITS
        self.x_kind = OUT_F32 if self.fmode else (OUT_I8 if bits <= 8 else OUT_I16)
        self.w_hwio = torch.zeros((in_units, units), dtype=torch.int8, device=ctx.device)
        # wide heads (ResNet-50's fc): int8-MFMA GEMMs on packed images of the quantised W
        self.mfma = ops.dense_mfma_ok(in_units, units, bits, weight_bits) and not self.fmode
        if self.mfma:
            self.wf = torch.zeros((units, -(-in_units // 64) * 64), dtype=torch.int8, device=ctx.device)
            self.wd = torch.zeros((in_units, -(-units // 64) * 64), dtype=torch.int8, device=ctx.device)
        self._c = _Cache()

    def param_slots(self):
        s = [(self, "W", "dW")]
        if self.use_bias:
            s.append((self, "b", "db"))
        return s

    def forward(self, X):
        self.X = X
        N = X.shape[0]
        dev = X.device
        self.d = d = _lib.ConvDesc(N, 1, 1, self.in_units, self.units, 1, 1, 1, 1, 0, 0, 0, 0, 1, 1)
        if self.fmode:  # Xq @ Wq on fp32 operands (a 1x1 conv on a 1x1 map)
            self.xq = _fq(X, self.X_range, self._c, "xq")
            self.wq = _fq(self.W, self.W_range, self._c, "wq")
            y = self._c.get("y", (N, self.units), torch.float32, dev)
            _conv_f32(self.xq, self.wq, d, y)
            if self.use_bias:
                ops.bias_add(y, _fq(self.b, self.b_range, self._c, "bq"), self.units)
            self.y = y
            return y
        self.xq = ops.quantize(X, self.X_range, self.x_kind, out=self._c.get("xq", X.shape,
                                                                              ops.out_dtype(self.x_kind), dev))
        if not (self._batched_q and self.ctx.params_ready):
            ops.quantize_weight(self.W, self.W_range, w_hwio=self.w_hwio)
        y = self._c.get("y", (N, self.units), torch.float32, dev)
        if self.mfma:
            ops.dense_pack(self.w_hwio, self.wf, self.wd)
            ops.dense_gemm(self.xq, self.wf, self.in_units, self.X_range.desc, self.W_range.desc, y,
                           kernel="dense_fwd_kernel")
        else:
            ops.conv_fwd_generic(self.xq, self.x_kind == OUT_I16, self.w_hwio, d, self.X_range.desc,
                                 self.W_range.desc, y)
        if self.use_bias:
            self.bq = ops.quantize(self.b, self.b_range, OUT_F32, out=self._c.get("bq", (self.units,), torch.float32,
                                                                                   dev))
            ops.bias_add(y, self.bq, self.units)
        self.y = y
        return y

    def backward(self, grad, stochastic=True):
        self.grad = grad  # kept for pre_dense_func (the reference's self.grad, :442)
        d = self.d
        dev = grad.device
        if self.fmode:
            self.gradq = _fq(grad, self.grad_range, self._c, "gq")
            dx = _conv_bwd_f32(self, self.gradq, d, dev)
            return dx.view(d.N, self.in_units)
        if self.grad_bits > 8:
            gsum = self._c.sums("gsum", ops.NSHARD * 2 * self.units, self.ctx) if self.use_bias else None
            self.gradq = ops.quantize(grad, self.grad_range, OUT_I16, out=self._c.get("gq16", grad.shape, torch.int16,
                                                                                       dev),
                                      chsum=gsum, C=self.units if self.use_bias else 0)
            if self.use_bias:  # db = the quantised gradient summed per unit (:457)
                ops.bias_grad(gsum, self.units, self.grad_range.desc, self.db)
            if self.mfma:
                return self._backward_mfma(dev)
            ns = ops.wgrad_nsplit(d, generic=True)
            slab = self._c.get("slab64", (ns, self.in_units, self.units), torch.int64, dev)
            ops.conv_wgrad_generic16(self.xq, self.x_kind == OUT_I16, self.gradq, d, slab, ns)
            ops.conv_wgrad_reduce64(slab, ns, self.in_units, self.units, self.X_range.desc, self.grad_range.desc,
                                    self.W, ops.f32(2 * self.weight_decay), self.dW)
            dx = self._c.get("dx", (d.N, self.in_units), torch.float32, dev)
            ops.conv_dgrad_generic16(self.gradq, self.w_hwio, d, self.grad_range.desc, self.W_range.desc, dx)
            return dx
        gsum = self._c.sums("gsum", ops.NSHARD * 2 * self.units, self.ctx)
        self.gradq = ops.quantize(grad, self.grad_range, OUT_I8, out=self._c.get("gq", grad.shape, torch.int8, dev),
                                  chsum=gsum, C=self.units)
        if self.mfma:
            if self.use_bias:
                ops.bias_grad(gsum, self.units, self.grad_range.desc, self.db)
            return self._backward_mfma(dev)
        ns = ops.wgrad_nsplit(d, generic=True)
        slab = self._c.get("slab", (ns, self.in_units, self.units), torch.int32, dev)
        ops.conv_wgrad_generic(self.xq, self.x_kind == OUT_I16, self.gradq, d, slab, ns)
        ops.conv_wgrad_reduce(slab, ns, self.in_units, self.units, 0, None, self.X_range.desc,
                              self.grad_range.desc, self.W, ops.f32(2 * self.weight_decay), self.dW)
        if self.use_bias:
            ops.bias_grad(gsum, self.units, self.grad_range.desc, self.db)
        dx = self._c.get("dx", (d.N, self.in_units), torch.float32, dev)
        ops.conv_dgrad_generic(self.gradq, self.w_hwio, d, self.grad_range.desc, self.W_range.desc, dx)
        return dx

    def _backward_mfma(self, dev):
        """dW (VALU, exact int64, reduce fused) and dX (int8 MFMA; int16 codes split hi/lo)."""
        ops.dense_wgrad(self.xq, self.gradq, self.X_range.desc, self.grad_range.desc, self.W,
                        ops.f32(2 * self.weight_decay), self.dW)
        dx = self._c.get("dx", (self.d.N, self.in_units), torch.float32, dev)
        ops.dense_gemm(self.gradq, self.wd, self.units, self.grad_range.desc, self.W_range.desc, dx,
                       kernel="dense_dgrad_kernel")
        return dx

    def pre_dense_func(self, grad=None):
        """``Dense_q.pre_dense_func`` (:397-439; dormant in the reference's trainer, which never
        fetches ``pre_dense_op``): the per-element small-gradient accumulator applied in place to
        ``grad`` (default: the last backward's incoming gradient), eps = 2^-(bits - grad_range).
        State (:364-366, :449): accu = 0.001, init_flag = 1, rem_flag = 0, [in_units, units]."""
        grad = self.grad if grad is None else grad
        if not hasattr(self, "_pd_accu"):
            dev = self.ctx.device
            self._pd_accu = torch.full((self.in_units, self.units), 0.001, dtype=torch.float32, device=dev)
            self._pd_init = torch.ones((self.in_units, self.units), dtype=torch.int32, device=dev)
            self._pd_rem = torch.zeros((self.in_units, self.units), dtype=torch.int32, device=dev)
        return ops.pre_dense(grad, self.grad_range.desc, self._pd_accu, self._pd_init, self._pd_rem)

    def grads_and_vars(self):
        if self.use_bias:
            return [(self.dW, self.W), (self.db, self.b)]
        return [(self.dW, self.W)]

    def info(self):
        return "%d bits dense: %dx%d weight_decay %f" % (self.bits, self.in_units, self.units, self.weight_decay)


class GradientBuffer_q(Layer_q):
    """Gradient buffer (``:472-509``): identity forward; backward quantises the incoming gradient
    plus the buffered residue (zero-padded to ``shape``) and keeps the new residue
    (error feedback): ``total = pad(grad) + buffer; gq = Q(total); buffer = total - gq``."""

    def __init__(self, name, bits, shape, target_overflow_rate=0, grad_range=2, ctx=None):
        self.ctx = ctx = ctx or default_context()
        self.name, self.bits, self.shape = name, bits, tuple(int(s) for s in shape)
        self.target_overflow_rate = target_overflow_rate
        self.buffer = torch.zeros(self.shape, dtype=torch.float32, device=ctx.device)
        self.grad_range = ctx.quantizer(name + "/grad_range", bits, grad_range, target_overflow_rate) \
            if bits != 32 else None

    def backward(self, grad, stochastic=True):
        if tuple(grad.shape[1:]) != self.shape[1:] or grad.shape[0] > self.shape[0]:
            raise ValueError("gradient %s does not fit the buffer %s" % (tuple(grad.shape), self.shape))
        inner = int(np.prod(self.shape[1:])) if len(self.shape) > 1 else 1
        if self.grad_range is not None:
            self.grad_range.observe(self.buffer.numel())
            desc = self.grad_range.desc
        else:
            desc = _lib.QDesc()
            desc.bits = 32
        self.gradq = ops.grad_buffer_bwd(grad.contiguous(), self.buffer, desc, inner)
        return self.gradq

    def info(self):
        return "Gradient buffer"


class Sequential_q(Layer_q):
    def __init__(self, *args):
        self.layers = args

    def forward(self, X):
        self.X = X
        for layer in self.layers:
            X = layer.forward(X)
        self.y = X
        return self.y

    def backward(self, grad, stochastic=True):
        for layer in reversed(self.layers):
            grad = layer.backward(grad, stochastic)
        return grad

    def grads_and_vars(self):
        res = []
        for layer in self.layers:
            res += layer.grads_and_vars()
        return res

    def param_slots(self):
        return [s for layer in self.layers for s in layer.param_slots()]

    def info(self):
        return "\n\t".join(["Sequential layer:"] + [layer.info() for layer in self.layers])


class Normalization_q(Layer_q):
    """BN normalisation half (``:539-623``): quantise X, biased batch moments, normalise."""

    def __init__(self, name, bits, num_features, training=True, momentum=0.999, eps=1e-5, target_overflow_rate=0,
                 input_range=2, grad_range=2, grad_bits=None, ctx=None):
        self.ctx = ctx = ctx or default_context()
        self.name, self.bits, self.C, self.train = name, bits, num_features, training
        self.grad_bits = grad_bits = grad_bits or bits
        self.momentum, self.eps, self.target_overflow_rate = momentum, eps, target_overflow_rate
        self.X_range = ctx.quantizer(name + "/X_range", bits, input_range, target_overflow_rate)
        self.grad_range = ctx.quantizer(name + "/grad_range", grad_bits, grad_range, target_overflow_rate)
        self.X_mean_running = torch.zeros(num_features, dtype=torch.float32, device=ctx.device)
        self.X_var_running = torch.ones(num_features, dtype=torch.float32, device=ctx.device)
        self.ms = torch.zeros(2 * num_features, dtype=torch.float32, device=ctx.device)
        self.fmode = max(bits, grad_bits) > FLOAT_BITS
        self._c = _Cache()

    def norm_desc(self, q, chsum, n):
        return BnNorm(ptr(q).value, self.X_range.desc, ptr(chsum).value, n, ops.f32(self.eps),
                      ops.f32(self.momentum), ops.f32(1 - self.momentum), self.ms.data_ptr(),
                      self.X_mean_running.data_ptr(), self.X_var_running.data_ptr(), 0 if self.train else 1)

    def forward(self, X):
        """Training: batch moments of Xq (and the running averages move); testing (train False,
        Model.set_testing): the running averages normalise and nothing moves (:590-612)."""
        self.X = X
        if self.fmode:  # fp32 statistics of the fake-quantised (or, at 32 bits, raw) input
            C = X.shape[-1]
            self.q = _fq(X, self.X_range, self._c, "xq")
            part = _chan_sums(self.q, None, C, self._c, "part") if self.train else None
            y = self._c.get("y", X.shape, torch.float32, X.device)
            _lib.call("lbt_bn_f32_fwd", ptr(self.q), ptr(part), _FSPLIT, X.numel() // C, C, ops.f32(self.eps),
                      ops.f32(self.momentum), ops.f32(1 - self.momentum), ptr(self.ms), ptr(self.X_mean_running),
                      ptr(self.X_var_running), 0 if self.train else 1, ptr(y), _lib.stream())
            self.y = y
            return y
        dev = X.device
        C = X.shape[-1]
        rows, inner = ops.rows_inner(tuple(X.shape))
        chsum = self._c.sums("chsum", ops.NSHARD * 2 * C, self.ctx)
        self.q = ops.quantize(X, self.X_range, OUT_I8, out=self._c.get("q", X.shape, torch.int8, dev), chsum=chsum,
                              C=C)
        self.n = X.numel() // C
        y = self._c.get("y", X.shape, torch.float32, dev)
        a = ChainFwd()
        a.b1.nrm = self.norm_desc(self.q, chsum, self.n)
        a.relu = 0
        a.y = y.data_ptr()
        a.rows, a.inner, a.C = rows, inner, C
        ops.chain_fwd(a)
        self.y = y
        return y

    def backward(self, grad, stochastic=True):
        dev = grad.device
        C = self.C
        if self.fmode:
            gq = _fq(grad, self.grad_range, self._c, "gq")
            part = _chan_sums(gq, self.q, C, self._c, "gpart") if self.train else None
            dx = self._c.get("dx", grad.shape, torch.float32, dev)
            _lib.call("lbt_bn_f32_bwd", ptr(gq), ptr(self.q), ptr(self.ms), ptr(part), _FSPLIT, grad.numel() // C, C,
                      0 if self.train else 1, ptr(dx), _lib.stream())
            return dx
        rows, inner = ops.rows_inner(tuple(grad.shape))
        sums = self._c.sums("sums", ops.NSHARD * 4 * C, self.ctx)
        if self.grad_bits > 8:  # 16-bit gradient codes (config 4)
            if not self.train:
                raise NotImplementedError("Normalization_q testing-mode backward with > 8-bit gradient codes")
            self.grad_range.observe(grad.numel())
            G16 = self._c.get("G16", grad.shape, torch.int16, dev)
            dx = self._c.get("dx", grad.shape, torch.float32, dev)
            pix = grad.numel() // C
            ops.bn_bwd_a_wide(grad, NO_Q, None, None, self.grad_range.desc, self.q, G16, None, sums, pix, inner, C)
            ops.bn_bwd_b_wide(G16, self.grad_range.desc, self.q, self.X_range.desc, self.ms, sums, self.n, dx, pix, C)
            return dx
        G = self._c.get("G", grad.shape, torch.int8, dev)
        self.grad_range.observe(grad.numel())
        a = ChainBwdA()
        a.g = grad.data_ptr()
        a.b1 = BwdBranch(NO_Q, None, NO_Q, None, self.grad_range.desc, self.q.data_ptr(), G.data_ptr(), None,
                         sums.data_ptr())
        a.rows, a.inner, a.C = rows, inner, C
        ops.chain_bwd_a(a)
        dx = self._c.get("dx", grad.shape, torch.float32, dev)
        # testing mode: mean / variance are constants, dX = Gq / sigma -- pass B with zero sums
        # (mg = mgx = 0 makes its ((g - mg) - xhat*mgx) / sigma exactly g / sigma)
        bsums = sums if self.train else self._c.get("zsums", sums.shape, torch.int64, dev, zero=True)
        b = ChainBwdB(G.data_ptr(), self.grad_range.desc, self.q.data_ptr(), self.X_range.desc, self.ms.data_ptr(),
                      bsums.data_ptr(), self.n, dx.data_ptr(), None, NO_Q, None, rows, inner, C)
        ops.chain_bwd_b(b)
        return dx

    def info(self):
        return "BatchNorm normalization"


class Rescale_q(Layer_q):
    """BN rescale half (``:626-694``): y = Q(X) * Q(gamma) + Q(beta)."""

    def __init__(self, name, bits, num_features, weight_decay=0, target_overflow_rate=0, input_range=2,
                 gamma_range=2, beta_range=2, grad_range=2, grad_bits=None, ctx=None):
        self.ctx = ctx = ctx or default_context()
        self.name, self.bits, self.C, self.weight_decay = name, bits, num_features, weight_decay
        self.target_overflow_rate = target_overflow_rate
        dev = ctx.device
        self.gamma = torch.ones(num_features, dtype=torch.float32, device=dev)
        self.beta = torch.zeros(num_features, dtype=torch.float32, device=dev)
        self.dgamma = torch.zeros_like(self.gamma)
        self.dbeta = torch.zeros_like(self.beta)
        t = target_overflow_rate
        self.g_range = ctx.quantizer(name + "/g_range", bits, gamma_range, t)
        self.b_range = ctx.quantizer(name + "/b_range", bits, beta_range, t)
        self.X_range = ctx.quantizer(name + "/X_range", bits, input_range, t)
        self.grad_bits = grad_bits = grad_bits or bits
        self.grad_range = ctx.quantizer(name + "/grad_range", grad_bits, grad_range, t)
        self.gb = torch.zeros(2 * num_features, dtype=torch.float32, device=dev)
        self.fmode = max(bits, grad_bits) > FLOAT_BITS
        self._c = _Cache()

    def param_slots(self):
        return [(self, "gamma", "dgamma"), (self, "beta", "dbeta")]

    def quantize_params(self):
        if self._batched_q and self.ctx.params_ready:
            return
        C = self.C
        if self.fmode:
            self.gb[:C].copy_(_fq(self.gamma, self.g_range, self._c, "gq_"))
            self.gb[C:].copy_(_fq(self.beta, self.b_range, self._c, "bq_"))
            return
        ops.quantize(self.gamma, self.g_range, OUT_F32, out=self.gb[:C])
        ops.quantize(self.beta, self.b_range, OUT_F32, out=self.gb[C:])

    def forward(self, X):
        self.X = X
        dev = X.device
        C = self.C
        rows, inner = ops.rows_inner(tuple(X.shape))
        self.quantize_params()
        if self.fmode:
            self.xr = _fq(X, self.X_range, self._c, "xr")
            y = self._c.get("y", X.shape, torch.float32, dev)
            _lib.call("lbt_affine_f32", ptr(self.xr), ptr(self.gb), X.numel(), C, 0, ptr(y), _lib.stream())
            self.y = y
            return y
        self.R = self._c.get("R", X.shape, torch.int8, dev)
        y = self._c.get("y", X.shape, torch.float32, dev)
        self.X_range.observe(X.numel())
        a = ChainFwd()
        a.b1.xin = X.data_ptr()
        a.b1.qr = self.X_range.desc
        a.b1.rout = self.R.data_ptr()
        a.b1.gb = self.gb.data_ptr()
        a.y = y.data_ptr()
        a.rows, a.inner, a.C = rows, inner, C
        ops.chain_fwd(a)
        self.y = y
        return y

    def backward(self, grad, stochastic=True):
        dev = grad.device
        C = self.C
        rows, inner = ops.rows_inner(tuple(grad.shape))
        dx = self._c.get("dx", grad.shape, torch.float32, dev)
        if self.fmode:
            g2 = _fq(grad, self.grad_range, self._c, "g2")
            _lib.call("lbt_affine_f32", ptr(g2), ptr(self.gb), grad.numel(), C, 1, ptr(dx), _lib.stream())
            part = _chan_sums(g2, self.xr, C, self._c, "part")
            _lib.call("lbt_affine_grads_f32", ptr(part), _FSPLIT, C, ptr(self.gamma), ops.f32(2 * self.weight_decay),
                      ptr(self.dgamma), ptr(self.dbeta), _lib.stream())
            return dx
        sums = self._c.sums("sums", ops.NSHARD * 4 * C, self.ctx)
        self.grad_range.observe(grad.numel())
        if self.grad_bits > 8:  # 16-bit gradient codes (config 4)
            ops.bn_bwd_a_wide(grad, self.grad_range.desc, self.R, self.gb[:C], NO_Q, None, None, dx, sums,
                              grad.numel() // C, inner, C)
            ops.bn_param_grads(sums, C, self.grad_range.desc, self.X_range.desc, self.gamma,
                               ops.f32(2 * self.weight_decay), self.dgamma, self.dbeta)
            return dx
        a = ChainBwdA()
        a.g = grad.data_ptr()
        a.b1 = BwdBranch(self.grad_range.desc, self.R.data_ptr(), self.X_range.desc, self.gb.data_ptr(), NO_Q,
                         None, None, dx.data_ptr(), sums.data_ptr())
        a.rows, a.inner, a.C = rows, inner, C
        ops.chain_bwd_a(a)
        ops.bn_param_grads(sums, C, self.grad_range.desc, self.X_range.desc, self.gamma,
                           ops.f32(2 * self.weight_decay), self.dgamma, self.dbeta)
        return dx

    def grads_and_vars(self):
        return [(self.dgamma, self.gamma), (self.dbeta, self.beta)]

    def info(self):
        return "BatchNorm rescale"


class BatchNorm_q(Sequential_q):
    """``Sequential_q(Normalization_q(name-norm), Rescale_q(name-rescale))`` (``:697-743``)."""

    def __init__(self, name, bits, num_features, training=True, momentum=0.999, eps=1e-5, weight_decay=0,
                 target_overflow_rate=0, input_range=2, gamma_range=2, beta_range=2, grad_range=2, grad_bits=None,
                 ctx=None):
        super().__init__(
            Normalization_q(name=name + "-norm", bits=bits, num_features=num_features, training=training,
                            momentum=momentum, eps=eps, target_overflow_rate=target_overflow_rate,
                            input_range=input_range, grad_range=grad_range, grad_bits=grad_bits, ctx=ctx),
            Rescale_q(name=name + "-rescale", bits=bits, num_features=num_features, weight_decay=weight_decay,
                      target_overflow_rate=target_overflow_rate, input_range=2, gamma_range=gamma_range,
                      beta_range=beta_range, grad_range=grad_range, grad_bits=grad_bits, ctx=ctx))

    def info(self):
        return "BatchNorm"


class ReLU_q(Layer_q):
    def __init__(self):
        self._c = _Cache()

    def forward(self, X):
        self.X = X
        if self.act_in_pool and X.shape[-1] % 4 == 0:
            self.y = X
            return X  # the pool computes pool(relu(X)) (ops.maxpool_relu_fwd)
        self.y = self._c.get("y", X.shape, torch.float32, X.device)
        ops.relu_fwd(X, self.y)
        return self.y

    # set by a following MaxPool_q that applies this mask in its own backward (pool_relu)
    mask_in_pool = False
    # set by the model builder when that pool also applies the activation (forward returns X)
    act_in_pool = False

    def backward(self, grad, stochastic=True):
        if self.mask_in_pool:
            return grad
        dx = self._c.get("dx", grad.shape, torch.float32, grad.device)
        ops.relu_bwd(grad, self.X, dx)
        return dx

    def info(self):
        return "ReLU"


class ResidualBlock_q(Layer_q):
    """Basic residual block (``:746-875``): conv-BN-ReLU-conv-BN + (identity | 1x1 conv-BN), ReLU."""
    expansion = 1

    def __init__(self, name, bits, in_channels, channels, stride, training=True, batch_norm=True, weight_decay=0,
                 target_overflow_rate=0, input_range=2, weight_range=2, bias_range=2, grad_range=2, weight_bits=None,
                 ctx=None):
        self.train = training
        self.name = name
        common = dict(bits=bits, use_bias=not batch_norm, weight_decay=weight_decay, input_range=input_range,
                      weight_range=weight_range, bias_range=bias_range, grad_range=grad_range,
                      input_nonnegative=True, weight_bits=weight_bits, ctx=ctx)
        bn = dict(bits=bits, num_features=channels, training=training, weight_decay=weight_decay,
                  target_overflow_rate=target_overflow_rate, input_range=input_range, grad_range=grad_range, ctx=ctx)
        self.residual = Sequential_q(
            Conv2d_q(name=name + "-1", ksize=[3, 3, in_channels, channels], strides=[1, stride, stride, 1],
                     padding="SAME", **common),
            BatchNorm_q(name=name + "-bn1", **bn) if batch_norm else Layer_q(),
            ReLU_q(),
            Conv2d_q(name=name + "-2", ksize=[3, 3, channels, channels], strides=[1, 1, 1, 1], padding="SAME",
                     **common),
            BatchNorm_q(name=name + "-bn2", **bn) if batch_norm else Layer_q(),
        )
        if stride == 1 and in_channels == self.expansion * channels:
            self.shortcut = Sequential_q()
        else:
            self.shortcut = Sequential_q(
                Conv2d_q(name=name + "-shortcut", ksize=[1, 1, in_channels, self.expansion * channels],
                         strides=[1, stride, stride, 1], padding="SAME", target_overflow_rate=target_overflow_rate,
                         **common),
                BatchNorm_q(name=name + "-shortcut-bn", **bn) if batch_norm else Layer_q(),
            )
        self.relu = ReLU_q()
        self._c = _Cache()

    def forward(self, X):
        self.X = X
        self.y1 = self.residual.forward(X)
        self.y2 = self.shortcut.forward(X)
        s = self._c.get("sum", self.y1.shape, torch.float32, X.device)
        ops.add(self.y1, self.y2, s)
        self.y = self.relu.forward(s)
        return self.y

    def backward(self, grad, stochastic=True):
        grad = self.relu.backward(grad, stochastic)
        g1 = self.residual.backward(grad, stochastic)
        g2 = self.shortcut.backward(grad, stochastic)
        out = self._c.get("dx", g1.shape, torch.float32, grad.device)
        ops.add(g1, g2, out)
        return out

    def grads_and_vars(self):
        return self.residual.grads_and_vars() + self.shortcut.grads_and_vars()

    def param_slots(self):
        return self.residual.param_slots() + self.shortcut.param_slots()

    def info(self):
        return "Residual block with " + self.residual.info()


class ResidualBottleneck_q(ResidualBlock_q):
    """Bottleneck residual block (``:878-980``): 1x1 -> BN -> ReLU -> 3x3 (stride) -> BN -> ReLU ->
    1x1 (4x channels) -> BN, plus the shortcut of ``_build_shortcut`` (``:825-856``), ReLU."""
    expansion = 4

    def __init__(self, name, bits, in_channels, channels, stride, training=True, batch_norm=True, weight_decay=0,
                 target_overflow_rate=0, input_range=2, weight_range=2, bias_range=2, grad_range=2, grad_bits=None,
                 ctx=None):
        self.train = training
        self.name = name
        out = self.expansion * channels
        common = dict(bits=bits, use_bias=not batch_norm, weight_decay=weight_decay, input_range=input_range,
                      weight_range=weight_range, bias_range=bias_range, grad_range=grad_range,
                      input_nonnegative=True, grad_bits=grad_bits, ctx=ctx)
        bn = dict(bits=bits, training=training, weight_decay=weight_decay, target_overflow_rate=target_overflow_rate,
                  input_range=input_range, grad_range=grad_range, grad_bits=grad_bits, ctx=ctx)
        self.residual = Sequential_q(
            Conv2d_q(name=name + "-1", ksize=[1, 1, in_channels, channels], strides=[1, 1, 1, 1], padding="SAME",
                     **common),
            BatchNorm_q(name=name + "-bn1", num_features=channels, **bn) if batch_norm else Layer_q(),
            ReLU_q(),
            Conv2d_q(name=name + "-2", ksize=[3, 3, channels, channels], strides=[1, stride, stride, 1],
                     padding="SAME", **common),
            BatchNorm_q(name=name + "-bn2", num_features=channels, **bn) if batch_norm else Layer_q(),
            ReLU_q(),
            Conv2d_q(name=name + "-3", ksize=[1, 1, channels, out], strides=[1, 1, 1, 1], padding="SAME", **common),
            BatchNorm_q(name=name + "-bn3", num_features=out, **bn) if batch_norm else Layer_q(),
        )
        if stride == 1 and in_channels == out:
            self.shortcut = Sequential_q()
        else:
            self.shortcut = Sequential_q(
                Conv2d_q(name=name + "-shortcut", ksize=[1, 1, in_channels, out], strides=[1, stride, stride, 1],
                         padding="SAME", target_overflow_rate=target_overflow_rate, **common),
                BatchNorm_q(name=name + "-shortcut-bn", num_features=out, **bn) if batch_norm else Layer_q(),
            )
        self.relu = ReLU_q()
        self._c = _Cache()


    # ---- fused execution of the block (bit-identical to the Sequential_q composition above)
    next_block = None  # set by the model builder: the block that consumes this block's output
    prev_block = None  # ... and the block whose output this block consumes
    _x_pre = None      # the input tensor whose conv codes the previous block already wrote

    def _fusable(self):
        """16-bit gradients (config 4) and every conv on the wide MFMA kernels with offset int8 X
        codes: then forward / backward run the block as one fused kernel schedule."""
        if getattr(self, "_fuse", None) is None:
            r = self.residual.layers
            if len(r) != 8 or not isinstance(r[1], BatchNorm_q):
                self._fuse = False
            else:
                convs = [r[0], r[3], r[6]] + ([self.shortcut.layers[0]] if self.shortcut.layers else [])
                self._fuse = (os.environ.get("LBT_FUSE_BOTTLENECK", "1") == "1"
                              and all(c.grad_bits > 8 and c.x_kind == OUT_U8OFF and c.igemm_f and c.igemm_d
                                      and c.igemm_w and not c.use_bias for c in convs))
        return self._fuse

    def forward(self, X):
        if not self._fusable():
            return super().forward(X)
        return self._forward_fused(X)

    def backward(self, grad, stochastic=True):
        if not self._fusable():
            return super().backward(grad, stochastic)
        with backward_scope():  # dW / dgamma / dbeta of the side stream are joined by the outermost backward
            return self._backward_fused(grad)

    @staticmethod
    def _chain(c, bn, y, relu, res=None, bn2=None, out=None, o1=None, o1_conv=None, o2=None, o2_conv=None,
               ybits=None):
        """One forward element chain: bn (norm of its input codes -> rescale quantiser ->
        affine) [+ bn2 | + res] [-> ReLU] -> fp32 out and / or the next convs' X codes."""
        a = ChainFwd()
        for br, b in ((a.b1, bn), (a.b2, bn2)):
            if b is None:
                continue
            n, r = b.layers
            r.quantize_params()
            r.X_range.observe(y.numel())
            br.nrm = n.norm_desc(n.q, n._chsum, n.n)
            if CHAIN_MS:  # the BN's moments once (one thread per channel), not in every chain workgroup
                ops.bn_moments(br.nrm, y.shape[-1])
                br.nrm.ms_in = 1
            br.qr = r.X_range.desc
            br.rout = r.R.data_ptr()
            br.gb = r.gb.data_ptr()
        a.has_b2 = int(bn2 is not None)
        a.res = res.data_ptr() if res is not None else None
        a.relu = int(relu)
        a.y = out.data_ptr() if out is not None else None
        a.ybits = ybits.data_ptr() if ybits is not None else None
        if o1 is not None:
            o1_conv.X_range.observe(y.numel())
            a.o1, a.o1_kind, a.qo1 = o1.data_ptr(), OUT_U8OFF, o1_conv.X_range.desc
        if o2 is not None:
            o2_conv.X_range.observe(y.numel())
            a.o2, a.o2_kind, a.qo2 = o2.data_ptr(), OUT_U8OFF, o2_conv.X_range.desc
        a.rows, a.inner = ops.rows_inner(tuple(y.shape))
        a.C = y.shape[-1]
        ops.chain_fwd(a)

    @staticmethod
    def _conv_norm(conv, bn, xq, N, H, W, ctx):
        """conv forward + bn's input quantiser: in the GEMM epilogue when the GEMM does not split K
        (int8 codes straight from the MFMA accumulators), else fp32 y + the quantise pass."""
        kh, kw, Cin, Cout = conv.ksize
        d = ops.conv_desc(N, H, W, Cin, Cout, kh, kw, conv.strides[1], conv.strides[2], conv.padding)
        # the quantising epilogue (exact): with the 256-row LDS-DMA GEMM it beats fp32 y + the quantise
        # pass by 0.2-0.5 ms per ResNet-50 step (round 3 A/B; with the round-2 GEMM it lost); LBT_FUSE_CONV_QUANT=0: off,
        # 2: also the GEMMs that would split K (the unsplit quantising kernel instead of split-K + the quantise pass)
        mode = os.environ.get("LBT_FUSE_CONV_QUANT", "1")
        if mode == "0" or (mode != "2" and ops.igemm_workspace_bytes(d, 0, False)):
            y = conv.fwd_codes(xq, N, H, W)
            ResidualBottleneck_q._norm_in(bn, y, ctx)
            return y
        conv.d, conv.xq = d, xq
        conv.quantize_weights()
        n, r = bn.layers
        shape = (N, d.Ho, d.Wo, Cout)
        n._chsum = n._c.sums("chsum", ops.NSHARD * 2 * Cout, ctx)
        n.q = n._c.get("q", shape, torch.int8, xq.device)
        ops.conv_fwd_igemm_q(xq, 1, conv.wf, conv.ksf, d, conv.X_range.desc, conv.W_range.desc, n.q, n.X_range,
                             n._chsum)
        n.n = N * d.Ho * d.Wo
        r.R = r._c.get("R", shape, torch.int8, xq.device)
        return n.q  # the chain needs only its shape

    @staticmethod
    def _norm_in(bn, y, ctx):
        """Normalization_q's input quantiser on a conv output (codes + exact channel sums) and
        the Rescale_q code buffer the chain will fill."""
        n, r = bn.layers
        C = y.shape[-1]
        n._chsum = n._c.sums("chsum", ops.NSHARD * 2 * C, ctx)
        n.q = ops.quantize(y, n.X_range, OUT_I8, out=n._c.get("q", y.shape, torch.int8, y.device), chsum=n._chsum, C=C)
        n.n = y.numel() // C
        r.R = r._c.get("R", y.shape, torch.int8, y.device)

    def _forward_fused(self, X):
        """conv-1 -> [bn1 + ReLU + conv-2's X quantiser] -> conv-2 -> [bn2 + ReLU + conv-3's X
        quantiser] -> conv-3 (+ shortcut conv) -> [bn3 (+ shortcut bn | + X) + ReLU]: 3 element
        chains instead of 9 element layers (dynamic_fixed_point.py:858-862, :878-980)."""
        r = self.residual.layers
        c1, bn1, c2, bn2, c3, bn3 = r[0], r[1], r[3], r[4], r[6], r[7]
        sc = self.shortcut.layers
        ctx = c1.ctx
        self.X = X
        N, H, W, _ = X.shape
        dev = X.device
        x1 = self._c.get("x1", X.shape, torch.int8, dev)
        xs = self._c.get("xs", X.shape, torch.int8, dev) if sc else None
        if self._x_pre is not X:  # not already written by the previous block's last chain
            ops.quantize(X, c1.X_range, OUT_U8OFF, out=x1)
            if sc:
                ops.quantize(X, sc[0].X_range, OUT_U8OFF, out=xs)
        self._x_pre = None
        y1 = self._conv_norm(c1, bn1, x1, N, H, W, ctx)
        x2 = self._c.get("x2", y1.shape, torch.int8, dev)
        self._chain(c1, bn1, y1, True, o1=x2, o1_conv=c2)
        y2 = self._conv_norm(c2, bn2, x2, N, y1.shape[1], y1.shape[2], ctx)
        x3 = self._c.get("x3", y2.shape, torch.int8, dev)
        self._chain(c2, bn2, y2, True, o1=x3, o1_conv=c3)
        y3 = self._conv_norm(c3, bn3, x3, N, y2.shape[1], y2.shape[2], ctx)
        out = self._c.get("y", y3.shape, torch.float32, dev)
        # the next block's input quantisers (conv-1, shortcut conv) ride in this chain as well
        nb = self.next_block if (self.next_block is not None and self.next_block._fusable()) else None
        o = {}
        if nb is not None:
            nsc = nb.shortcut.layers
            o = dict(o1=nb._c.get("x1", y3.shape, torch.int8, dev), o1_conv=nb.residual.layers[0])
            if nsc:
                o.update(o2=nb._c.get("xs", y3.shape, torch.int8, dev), o2_conv=nsc[0])
        # the backward's ReLU mask as one byte per channel quad (pass A reads 1/16 of fp32 y's bytes)
        ybits = (self._c.get("ybits", (y3.numel() // 4,), torch.uint8, dev)
                 if os.environ.get("LBT_YBITS", "1") == "1" else None)
        self.ybits = ybits
        if sc:
            self._conv_norm(sc[0], sc[1], xs, N, H, W, ctx)
            self._chain(c3, bn3, y3, True, bn2=sc[1], out=out, ybits=ybits, **o)
        else:
            self._chain(c3, bn3, y3, True, res=X, out=out, ybits=ybits, **o)
        if nb is not None:
            nb._x_pre = out
        self.y = out
        return out

    @staticmethod
    def _bn_bwd(bn, conv_out, g, ctx, y_mask=None, mask_r=False, gmask_out=None, g2=None, y_bits=None):
        """One BN's backward with the ReLU mask in front (pass A: rescale + norm gradient
        quantisers, dgamma / dbeta), then pass B straight into the producing conv's 16-bit
        gradient quantiser: returns that conv's int16 gradient codes."""
        n, r = bn.layers
        C = g.shape[-1]
        rows, inner = g.numel() // C, g.numel() // g.shape[0]
        dev = g.device
        sums = r._c.sums("fsums", ops.NSHARD * 4 * C, ctx)
        r.grad_range.observe(g.numel())
        n.grad_range.observe(g.numel())
        G16 = n._c.get("G16", g.shape, torch.int16, dev)
        ops.bn_bwd_a_wide_masked(g, y_mask, mask_r, r.X_range.desc, r.gb, gmask_out, r.grad_range.desc, r.R,
                                 n.grad_range.desc, n.q, G16, sums, rows, inner, C, g2=g2, y_bits=y_bits)
        return ResidualBottleneck_q._bn_bwd_b(bn, conv_out, G16, sums, g.numel(), rows, inner, C)

    @staticmethod
    def _dgrad_bn_bwd(conv, gq16, bn, conv_out, ctx):
        """_bn_bwd(bn, conv_out, conv.bwd_codes16(gq16), mask_r=True) with bn's pass A evaluated on
        conv's dgrad (ops.conv_dgrad_igemm_bna): in the 256-row GEMM's epilogue, no fp32 dx, when that
        kernel takes the dgrad. bn is the BN in front of conv's input (bn2 behind conv-3, bn1 behind
        conv-2); returns conv_out's int16 gradient codes."""
        if not DGRAD_BNA:
            return ResidualBottleneck_q._bn_bwd(bn, conv_out, conv.bwd_codes16(gq16), ctx, mask_r=True)
        n, r = bn.layers
        conv.gradq = gq16
        with backward_scope():
            with side_work():  # dW: read only by the optimizer
                conv._wgrad_igemm(1)
            d = conv.d
            C = d.Cin
            shape = (d.N, d.H, d.W, C)
            numel = d.N * d.H * d.W * C
            rows, inner = numel // C, numel // d.N
            dev = gq16.device
            sums = r._c.sums("fsums", ops.NSHARD * 4 * C, ctx)
            r.grad_range.observe(numel)
            n.grad_range.observe(numel)
            G16 = n._c.get("G16", shape, torch.int16, dev)
            dx = conv._c.get("dx", shape, torch.float32, dev)  # used only when the dgrad cannot fuse
            ops.conv_dgrad_igemm_bna(gq16, conv.wd, conv.ksd, d, conv.grad_range.desc, conv.W_range.desc,
                                     r.X_range.desc, r.R, r.gb, r.grad_range, n.grad_range, n.q, G16, sums, dx,
                                     conv._ws(d, 1, True))
            return ResidualBottleneck_q._bn_bwd_b(bn, conv_out, G16, sums, numel, rows, inner, C)

    @staticmethod
    def _bn_bwd_b(bn, conv_out, G16, sums, numel, rows, inner, C):
        """dgamma / dbeta (side stream) and pass B into conv_out's 16-bit gradient quantiser."""
        n, r = bn.layers
        with side_work():
            ops.bn_param_grads(sums, C, r.grad_range.desc, r.X_range.desc, r.gamma, ops.f32(2 * r.weight_decay),
                               r.dgamma, r.dbeta)
        conv_out.grad_range.observe(numel)
        gq = conv_out._c.get("gq16", G16.shape, torch.int16, G16.device)
        ops.bn_bwd_b_wide_q(G16, n.grad_range.desc, n.q, n.X_range.desc, n.ms, sums, n.n, gq,
                            conv_out.grad_range.desc, rows, inner, C)
        return gq

    def _backward_fused(self, grad):
        """grad: the block output's gradient, or the pair (g1, g2) of the next fused block's two
        branch gradients, whose sum g1 + g2 is formed inside this block's first pass A. Returns
        the pair (residual-branch dX, shortcut dX) when the previous block is fused too, else
        their sum (dgrad epilogue add)."""
        r = self.residual.layers
        c1, bn1, c2, bn2, c3, bn3 = r[0], r[1], r[3], r[4], r[6], r[7]
        sc = self.shortcut.layers
        ctx = c1.ctx
        if isinstance(grad, _DgradIn):
            g3, gs, gmask = self._entry_from_dgrad(grad, ctx)
        else:
            gin, gin2 = grad if isinstance(grad, tuple) else (grad, None)
            dev = gin.device
            # block ReLU mask from the block output; bn3 (and the shortcut bn) see the same masked g
            gmask = None if sc else self._c.get("gmask", gin.shape, torch.float32, dev)
            ym = dict(y_bits=self.ybits) if self.ybits is not None else dict(y_mask=self.y)
            g3 = self._bn_bwd(bn3, c3, gin, ctx, gmask_out=gmask, g2=gin2, **ym)
            gs = self._bn_bwd(sc[1], sc[0], gin, ctx, g2=gin2, **ym) if sc else None
        g2 = self._dgrad_bn_bwd(c3, g3, bn2, c2, ctx)
        g1 = self._dgrad_bn_bwd(c2, g2, bn1, c1, ctx)
        other = sc[0].bwd_codes16(gs) if sc else gmask
        pb = self.prev_block
        if pb is not None and pb._fusable():
            if DGRAD_BN3 and pb.ybits is not None:
                return _DgradIn(c1, g1, other)
            return (c1.bwd_codes16(g1), other)
        return c1.bwd_codes16(g1, add_src=other)

    def _entry_from_dgrad(self, din, ctx):
        """This block's entry passes A (ReLU mask y_bits on dx + other; bn3, and the projection
        shortcut's BN) in the epilogue of the next block's conv-1 dgrad (ops.conv_dgrad_igemm_bn3), then
        each BN's pass B: returns (conv-3's gradient codes, the shortcut conv's or None, gmask)."""
        r = self.residual.layers
        c3, bn3 = r[6], r[7]
        sc = self.shortcut.layers
        conv = din.conv
        conv.gradq = din.gq
        with backward_scope():
            with side_work():  # dW of the next block's conv-1: read only by the optimizer
                conv._wgrad_igemm(1)
            d = conv.d
            C = d.Cin
            shape = (d.N, d.H, d.W, C)
            numel = d.N * d.H * d.W * C
            rows, inner = numel // C, numel // d.N
            dev = din.gq.device
            gmask = None if sc else self._c.get("gmask", shape, torch.float32, dev)
            pairs = [(bn3, c3)] + ([(sc[1], sc[0])] if sc else [])
            bns = []
            for bn, _ in pairs:
                n, rs = bn.layers
                sums = rs._c.sums("fsums", ops.NSHARD * 4 * C, ctx)
                rs.grad_range.observe(numel)
                n.grad_range.observe(numel)
                G16 = n._c.get("G16", shape, torch.int16, dev)
                bns.append((rs.R, rs.gb, rs.grad_range, n.grad_range, n.q, G16, sums))
            dx = conv._c.get("dx", shape, torch.float32, dev)  # used only when the dgrad cannot fuse
            ops.conv_dgrad_igemm_bn3(din.gq, conv.wd, conv.ksd, d, conv.grad_range.desc, conv.W_range.desc, din.other,
                                     self.ybits, gmask, bns, dx, conv._ws(d, 1, True))
            gq = [self._bn_bwd_b(bn, conv_out, b[5], b[6], numel, rows, inner, C)
                  for (bn, conv_out), b in zip(pairs, bns)]
        return gq[0], (gq[1] if sc else None), gmask


class MaxPool_q(Layer_q):
    """``MaxPool_q`` (``:993-1006``, ``tf.nn.max_pool``) and its TF gradient (lbt_maxpool_fwd/_bwd)."""

    def __init__(self, ksize, strides, padding):
        self.ksize, self.strides, self.padding = ksize, strides, padding
        self._c = _Cache()

    def forward(self, X):
        N, H, W, C = X.shape
        self.X = X
        self.d = d = ops.conv_desc(N, H, W, C, C, self.ksize[1], self.ksize[2], self.strides[1], self.strides[2],
                                   self.padding)
        y = self._c.get("y", (N, d.Ho, d.Wo, C), torch.float32, X.device)
        self.amax = self._c.get("amax", (N, d.Ho, d.Wo, C), torch.uint8, X.device)
        self.amax_masked = self.pool_relu is not None and self.pool_relu.act_in_pool and C % 4 == 0
        if self.amax_masked:
            ops.maxpool_relu_fwd(X, y, self.amax, d)  # X is the ReLU's input; amax carries the ReLU mask
        else:
            ops.maxpool_fwd(X, y, self.amax, d)
        self.y = y
        return y

    # the ReLU_q in front of this pool whose backward this one performs (its input > 0 mask): set
    # by the model builder, see ops.maxpool_relu_bwd
    pool_relu = None
    amax_masked = False  # amax from maxpool_relu_fwd: the ReLU mask is in the codes (forward)

    def backward(self, grad, stochastic=True):
        dx = self._c.get("dx", self.X.shape, torch.float32, grad.device)
        fuse = self.pool_relu is not None and self.d.Cin % 4 == 0
        if self.pool_relu is not None:
            self.pool_relu.mask_in_pool = fuse
        if fuse:
            ops.maxpool_relu_bwd(grad.contiguous(), self.amax, None if self.amax_masked else self.y, dx, self.d)
        else:
            ops.maxpool_bwd(grad.contiguous(), self.amax, dx, self.d)
        return dx

    def info(self):
        return "max pool: %dx%d stride %dx%d" % (self.ksize[1], self.ksize[2], self.strides[1], self.strides[2])


class AvgPool_q(Layer_q):
    """``AvgPool_q`` (``:1009-1022``, tf.nn.avg_pool). The window that covers the whole map (VALID) --
    the ResNets' global pool -- sums in order and scales by 1/(H*W) (lbt_avgpool_fwd); any other
    window / stride / SAME padding takes lbt_avgpool_gen_fwd (sum / count of valid positions)."""

    def __init__(self, ksize, strides, padding):
        self.ksize, self.strides, self.padding = ksize, strides, padding
        self._c = _Cache()

    def _global(self, H, W):
        return self.padding == "VALID" and self.ksize[1] == H and self.ksize[2] == W

    def forward(self, X):
        N, H, W, C = X.shape
        self.X = X
        if self._global(H, W):
            y = self._c.get("y", (N, 1, 1, C), torch.float32, X.device)
            ops.avgpool_fwd(X, y, N, H * W, C)
        else:
            self.d = d = ops.conv_desc(N, H, W, C, C, self.ksize[1], self.ksize[2], self.strides[1], self.strides[2],
                                       self.padding)
            y = self._c.get("y", (N, d.Ho, d.Wo, C), torch.float32, X.device)
            ops.avgpool_gen_fwd(X.contiguous(), y, d)
        self.y = y
        return y

    def backward(self, grad, stochastic=True):
        N, H, W, C = self.X.shape
        dx = self._c.get("dx", self.X.shape, torch.float32, grad.device)
        if self._global(H, W):
            ops.avgpool_bwd(grad.contiguous(), dx, N, H * W, C)
        else:
            ops.avgpool_gen_bwd(grad.contiguous(), dx, self.d)
        return dx

    def info(self):
        return "avg pool: %dx%d stride %dx%d" % (self.ksize[1], self.ksize[2], self.strides[1], self.strides[2])


class Flatten_q(Layer_q):
    def __init__(self, dim):
        self.dim = dim

    def forward(self, X):
        self.X = X
        self.y = X.reshape(-1, self.dim)
        return self.y

    def backward(self, grad, stochastic=True):
        return grad.reshape(self.X.shape)

    def info(self):
        return "flatten"
