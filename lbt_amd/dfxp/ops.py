"""Typed wrappers over the C-ABI (include/lbt_dfxp.h). Tensors in, kernels launched on the
current torch stream, nothing synchronised. All shape logic of the HIP path lives here."""
import ctypes
import math
import os

import torch

from .. import _lib
from .._lib import NSHARD, OUT_F32, OUT_I8, OUT_I16, OUT_U8OFF, ConvDesc, QDesc, call, ptr, stream

NO_Q = _lib.NO_Q

# --------------------------------------------------------------------------- launch timing hook
# When PROFILE is a dict, every wrapped launch is bracketed by HIP events on the current stream
# and its algorithmic bytes (each operand read once, each output written once) are recorded as
# PROFILE[kernel] -> [(start_event, end_event, bytes), ...]  (see lbt_amd/roofline.py).
PROFILE = None


class _Timed:
    def __init__(self, kernel, nbytes):
        self.kernel, self.nbytes = kernel, nbytes

    def __enter__(self):
        if PROFILE is not None:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e1 = torch.cuda.Event(enable_timing=True)
            self.e0.record()
        return self

    def __exit__(self, *exc):
        if PROFILE is not None and exc[0] is None:
            self.e1.record()
            PROFILE.setdefault(self.kernel, []).append((self.e0, self.e1, int(self.nbytes)))
        return False


def _code_bytes(kind):
    return {OUT_I8: 1, OUT_U8OFF: 1, OUT_I16: 2, OUT_F32: 4}[kind]


def _check(t, dtype, name):
    if not t.is_cuda:
        raise ValueError("%s must be a CUDA (HIP) tensor" % name)
    if t.dtype != dtype:
        raise ValueError("%s must be %s, got %s" % (name, dtype, t.dtype))
    if not t.is_contiguous():
        raise ValueError("%s must be contiguous" % name)


def rows_inner(shape):
    """(rows, inner) of the reference's noise broadcast: noise over shape[1:], rows = shape[0]."""
    if len(shape) <= 1:
        return (int(shape[0]) if len(shape) else 1), 1
    return int(shape[0]), int(math.prod(shape[1:]))


def out_dtype(kind):
    return {OUT_I8: torch.int8, OUT_U8OFF: torch.int8, OUT_I16: torch.int16, OUT_F32: torch.float32}[kind]


def new_sums(C, per_shard, device):
    return torch.zeros(NSHARD * per_shard * C, dtype=torch.int64, device=device)


# ----------------------------------------------------------------------------- quantiser
def quantize(x, q, kind, out=None, chsum=None, C=0, stats=True):
    """weight_quantization of x with quantiser q (dynamic_fixed_point.py:4-45) -> codes in `kind`."""
    _check(x, torch.float32, "x")
    rows, inner = rows_inner(tuple(x.shape))
    if out is None:
        out = torch.empty(x.shape, dtype=out_dtype(kind), device=x.device)
    if stats:
        q.observe(x.numel())
    desc = q.desc if stats else q.desc_nostats()
    vec = inner % 4 == 0 and inner >= 64 and x.data_ptr() % 16 == 0 and (chsum is None or C % 4 == 0)
    with _Timed("quantize_rows_kernel" if vec else "quantize_generic_kernel", x.numel() * (4 + _code_bytes(kind))):
        call("lbt_dfxp_quantize", ptr(x), ptr(out), kind, rows, inner, desc, ptr(chsum), int(C), stream())
    return out


def quantize_weight(w, q, w_hwio=None, wf=None, ksf=0, wd=None, ksd=0, colsum=None):
    """Weight quantiser + GEMM operand packing. w: fp32 HWIO [KH,KW,Cin,Cout] (or [in,out])."""
    _check(w, torch.float32, "w")
    if w.dim() == 2:
        # Dense_q W [in, out]: noise over shape[1:] = [out]. Presented as KH=in, KW=Cin=1 the
        # HWIO flat index and the noise period (KW*Cin*Cout = out) are exactly [in, out]'s.
        if wf is not None or wd is not None:
            raise ValueError("2-D weights are packed for the generic kernels only")
        KH, Cout = w.shape
        KW = Cin = 1
    else:
        KH, KW, Cin, Cout = w.shape
    q.observe(w.numel())
    call("lbt_dfxp_quantize_weight", ptr(w), KH, KW, Cin, Cout, q.desc, ptr(w_hwio), ptr(wf), int(ksf), ptr(wd),
         int(ksd), ptr(colsum), stream())


def quantize_weights_flat(jobs, starts, njobs, nblocks):
    """Every job of a device array of lbt_wjob in one element-parallel launch (batched.hip)."""
    with _Timed("quantize_weights_flat_kernel", 0):
        call("lbt_dfxp_quantize_weights_flat", ptr(jobs), ptr(starts), int(njobs), int(nblocks), stream())


def quantize_many(jobs, njobs):
    call("lbt_dfxp_quantize_many", ptr(jobs), int(njobs), stream())


def packed_slices(KH, KW, C):
    """16-byte k-slices per GEMM column for a tap-major (tap, 16-channel slice) k order, padded to 4."""
    s = KH * KW * ((C + 15) // 16)
    return (s + 3) // 4 * 4


# ----------------------------------------------------------------------------- conv geometry
def tf_same(in_size, k, s):
    out = -(-in_size // s)
    total = max((out - 1) * s + k - in_size, 0)
    return out, total // 2, total - total // 2


def conv_desc(N, H, W, Cin, Cout, KH, KW, SH, SW, padding):
    """TF 'SAME' / 'VALID' (dynamic_fixed_point.py:291 tf.nn.conv2d) or explicit symmetric int
    padding (the torch face), resolved to (top, bottom, left, right)."""
    if padding == "SAME":
        Ho, pt, pb = tf_same(H, KH, SH)
        Wo, pl, pr = tf_same(W, KW, SW)
    elif padding == "VALID":
        Ho = -(-(H - KH + 1) // SH)
        Wo = -(-(W - KW + 1) // SW)
        pt = pb = pl = pr = 0
    else:
        ph, pw = (padding, padding) if isinstance(padding, int) else padding
        pt = pb = ph
        pl = pr = pw
        Ho = (H + 2 * ph - KH) // SH + 1
        Wo = (W + 2 * pw - KW) // SW + 1
    if Ho <= 0 or Wo <= 0:
        raise ValueError("empty conv output for input %dx%d kernel %dx%d" % (H, W, KH, KW))
    return ConvDesc(N, H, W, Cin, Cout, KH, KW, SH, SW, pt, pb, pl, pr, Ho, Wo)


def mfma_ok(Cin, Cout):
    """Shapes the int8 MFMA kernels take (16-channel slices, 1/2/4/8 of them on each side)."""
    return Cin in (16, 32, 64, 128) and Cout in (16, 32, 64, 128)


def conv_fwd_i8(xq, x_u8off, wf, ksf, wcolsum, d, qx, qw, y=None, yq=None, qout=None, ychsum=None):
    M = d.N * d.Ho * d.Wo
    nb = xq.numel() + wf.numel() + (M * d.Cout * 4 if y is not None else 0) + (M * d.Cout if yq is not None else 0)
    with _Timed("conv_fwd_i8", nb):
        _conv_fwd_i8(xq, x_u8off, wf, ksf, wcolsum, d, qx, qw, y, yq, qout, ychsum)


def _conv_fwd_i8(xq, x_u8off, wf, ksf, wcolsum, d, qx, qw, y, yq, qout, ychsum):
    call("lbt_conv_fwd_i8", ptr(xq), int(x_u8off), ptr(wf), int(ksf), ptr(wcolsum), d, qx, qw, ptr(y), ptr(yq),
         qout if qout is not None else NO_Q, ptr(ychsum), stream())


def conv_dgrad_i8(gq, wd, ksd, d, qg, qw, dx, add_src=None):
    nb = gq.numel() + wd.numel() + dx.numel() * (8 if add_src is not None else 4)
    with _Timed("conv_dgrad_i8", nb):
        _conv_dgrad_i8(gq, wd, ksd, d, qg, qw, dx, add_src)


def _conv_dgrad_i8(gq, wd, ksd, d, qg, qw, dx, add_src):
    call("lbt_conv_dgrad_i8", ptr(gq), ptr(wd), int(ksd), d, qg, qw, ptr(dx), ptr(add_src), stream())


def pack_int4(src, dst):
    """Two signed 4-bit codes per byte (the W4 weight images)."""
    call("lbt_pack_int4", ptr(src), ptr(dst), src.numel(), stream())


def conv_fwd_i8w4(xq, x_u8off, wf4, ksf, wcolsum, d, qx, qw, y):
    M = d.N * d.Ho * d.Wo
    with _Timed("conv_fwd_i8w4", xq.numel() + wf4.numel() + M * d.Cout * 4):
        call("lbt_conv_fwd_i8w4", ptr(xq), int(x_u8off), ptr(wf4), int(ksf), ptr(wcolsum), d, qx, qw, ptr(y), None,
             NO_Q, None, stream())


def conv_dgrad_i8w4(gq, wd4, ksd, d, qg, qw, dx):
    with _Timed("conv_dgrad_i8w4", gq.numel() + wd4.numel() + dx.numel() * 4):
        call("lbt_conv_dgrad_i8w4", ptr(gq), ptr(wd4), int(ksd), d, qg, qw, ptr(dx), None, stream())


def wgrad_nsplit(d, generic=False):
    P = d.N * d.Ho * d.Wo
    taps = d.KH * d.KW
    if generic:
        lo = -(-P // 8192)
        return max(lo, min(256, -(-P // (8 if P <= 4096 else 32))))
    # MFMA wgrad grid = (nsplit, taps, Cout/16): ~512 workgroups of >= 512 pixels each
    lo = -(-P // 65536)
    want = max(1, -(-512 // (taps * (d.Cout // 16))))
    return max(lo, min(want, max(1, P // 512)))


def wgrad_s1_ok(d):
    """lbt_conv_wgrad_many_i8's staged 3x3 / stride-1 body takes this conv (64-pixel chunks of
    whole image rows); mirrors wgrad_s1_ok in conv_mfma.hip."""
    return (d.KH == 3 and d.KW == 3 and d.SH == 1 and d.SW == 1 and d.PT == 1 and d.PB == 1 and d.PL == 1
            and d.PR == 1 and d.Ho == d.H and d.Wo == d.W and d.W <= 64 and 64 % d.W == 0
            and d.H % (64 // d.W) == 0 and (64 // d.W + 2) * (d.W + 2) <= 192)


WGRAD_CPW = int(os.environ.get("LBT_WGRAD_CPW", "8"))  # batched staged wgrad: 64-pixel chunks per wave
WGRAD_MIN_UNITS = int(os.environ.get("LBT_WGRAD_MIN_UNITS", "32"))  # batched staged wgrad: workgroups per job, at least
WGRAD_UNITS = int(os.environ.get("LBT_WGRAD_UNITS", "64"))  # batched per-tap wgrad: workgroups per conv (sweep: 32 / 48 / 64 / 80 / 96 / 128 -> 49 / 30 / 26 / 29 / 29 / 30 us)


def wgrad_nsplit_batched(d, chunks_per_wave=None):
    """Pixel splits of a conv's wgrad inside the batched launch (8-wave workgroups). Staged 3x3
    body: each split = 8 waves x `chunks_per_wave` 64-pixel chunks, a divisor of the chunk count.
    Other convs: ~128 workgroups (split x tap x co slice) per conv."""
    P = d.N * d.Ho * d.Wo
    if wgrad_s1_ok(d):
        chunks = P // 64
        ns = max(1, chunks // (8 * (chunks_per_wave or WGRAD_CPW)))
        if chunks_per_wave is None:
            # small batches: more, shorter splits (down to one chunk per wave) until the job has
            # WGRAD_MIN_UNITS workgroups -- a job takes as long as one workgroup's serial chunk loop, so
            # at 16 images per GPU 8 chunks per wave left the launch at 8-16 workgroups (B=128: unchanged)
            units = (d.Cin // 16) * (d.Cout // 16)
            while ns * units < WGRAD_MIN_UNITS and 2 * ns * 8 <= chunks:
                ns *= 2
        while chunks % ns:
            ns -= 1
        return ns
    lo = -(-P // 65536)
    return max(lo, min(max(1, WGRAD_UNITS // (d.KH * d.KW * (d.Cout // 16))), max(1, P // 512)))


def wgrad_nshard(d, nsplit):
    """Shards of the MFMA wgrad slab: each covers <= 65536 pixels (int32-exact partial sums)."""
    P = d.N * d.Ho * d.Wo
    per = -(-P // nsplit)
    return -(-nsplit // max(1, 65536 // per))


def wgrad_slab(cache, key, d, ctx, batched=False):
    """(nsplit, nshard, zeroed int32 slab [nshard, K, Cout]) carved from the context's sums arena
    (batched: the split of the conv's job in lbt_conv_wgrad_many_i8)."""
    ns = wgrad_nsplit_batched(d) if batched else wgrad_nsplit(d)
    nh = wgrad_nshard(d, ns)
    n = nh * d.KH * d.KW * d.Cin * d.Cout
    slab = cache.sums(key, (n + 1) // 2, ctx).view(torch.int32)[:n].view(nh, d.KH * d.KW * d.Cin, d.Cout)
    return ns, nh, slab


def conv_wgrad_i8(xq, x_u8off, gq, d, slab, nsplit, nshard):
    with _Timed("conv_wgrad_i8", xq.numel() + gq.numel() + nshard * d.KH * d.KW * d.Cin * d.Cout * 4):
        _conv_wgrad_i8(xq, x_u8off, gq, d, slab, nsplit, nshard)


def _conv_wgrad_i8(xq, x_u8off, gq, d, slab, nsplit, nshard):
    call("lbt_conv_wgrad_i8", ptr(xq), int(x_u8off), ptr(gq), d, ptr(slab), int(nsplit), int(nshard), stream())


# ---- the exact data-parallel exchange of the layer-wise models (Trainer, lbt_amd/distributed.py): while a
# sink is set, every gradient reduction writes the INTEGER numerator of its gradient into the int64
# exchange buffer at the gradient's offset in the flat gradient buffer (the *_x entry points), and the
# softmax normalises by the global batch and leaves its loss sum in the buffer's loss slot; the
# trainer all-reduces the buffer and dequantises once (lbt_step_finish).
_XSINK = None


def set_exchange_sink(gbase=None, n=0, xbuf=None, loss_off=0, world=1):
    """gbase: the flat gradient buffer (n fp32); xbuf: the int64 exchange buffer. No args: unset."""
    global _XSINK
    _XSINK = None if gbase is None else dict(gbase=gbase.data_ptr(), n=int(n), xbuf=xbuf.data_ptr(),
                                             loss=xbuf.data_ptr() + 8 * int(loss_off), world=int(world))


def _num(dw):
    """The exchange slot of gradient tensor dw (None: no sink)."""
    s = _XSINK
    if s is None:
        return None
    off = dw.data_ptr() - s["gbase"]
    if off < 0 or off + 4 * dw.numel() > 4 * s["n"] or off % 4:
        raise RuntimeError("exact exchange: a gradient outside the flat gradient buffer")
    return _lib.ctypes.c_void_p(s["xbuf"] + 2 * off)  # int64 index = fp32 index


def conv_wgrad_reduce(slab, nsplit, K, Cout, x_u8off, gcolsum, qx, qg, w, wd2, dw):
    num = _num(dw)
    if num is not None:
        call("lbt_conv_wgrad_reduce_x", ptr(slab), int(nsplit), int(K), int(Cout), int(x_u8off), ptr(gcolsum), num,
             stream())
        return
    call("lbt_conv_wgrad_reduce", ptr(slab), int(nsplit), int(K), int(Cout), int(x_u8off), ptr(gcolsum), qx, qg,
         ptr(w), float(wd2), ptr(dw), stream())


def conv_fwd_generic(xq, x_i16, w_hwio, d, qx, qw, y):
    call("lbt_conv_fwd_generic", ptr(xq), int(x_i16), ptr(w_hwio), d, qx, qw, ptr(y), stream())


def conv_dgrad_generic(gq, w_hwio, d, qg, qw, dx, add_src=None):
    call("lbt_conv_dgrad_generic", ptr(gq), ptr(w_hwio), d, qg, qw, ptr(dx), ptr(add_src), stream())


def conv_wgrad_generic(xq, x_i16, gq, d, slab, nsplit):
    call("lbt_conv_wgrad_generic", ptr(xq), int(x_i16), ptr(gq), d, ptr(slab), int(nsplit), stream())


def stem_ok(d):
    """The fp16-MFMA stem kernels take this conv (small patch, 16-multiple Cout)."""
    K = d.KH * d.KW * d.Cin
    return 0 < K <= 32 and d.Cout in (16, 32, 64)


def stem_nsplit(d):
    """Shards of the stem wgrad slab (>= 32; each <= 31 workgroups for int32 exactness)."""
    blocks = -(-(d.N * d.Ho * d.Wo) // _lib.STEM_WG_PIXELS)
    return max(32, -(-blocks // 31))


def stem_slab(cache, key, d, ctx):
    """Zeroed int32 [nshard, K, Cout] stem-wgrad slab carved from the context's sums arena."""
    ns = stem_nsplit(d)
    n = ns * d.KH * d.KW * d.Cin * d.Cout
    return ns, cache.sums(key, (n + 1) // 2, ctx).view(torch.int32)[:n].view(ns, d.KH * d.KW * d.Cin, d.Cout)


def conv_stem_fwd(x16, w_hwio, d, qx, qw, y=None, yq=None, qout=None, ychsum=None):
    M = d.N * d.Ho * d.Wo
    nb = x16.numel() * 2 + (M * d.Cout * 4 if y is not None else 0) + (M * d.Cout if yq is not None else 0)
    with _Timed("stem_fwd_kernel", nb):
        call("lbt_conv_stem_fwd", ptr(x16), ptr(w_hwio), d, qx, qw, ptr(y), ptr(yq),
             qout if qout is not None else NO_Q, ptr(ychsum), stream())


def conv_stem_wgrad(x16, gq, d, slab, nsplit):
    with _Timed("stem_wgrad_kernel", x16.numel() * 2 + gq.numel() + slab.numel() * 4):
        call("lbt_conv_stem_wgrad", ptr(x16), ptr(gq), d, ptr(slab), int(nsplit), stream())


def stem_wide_ok(d, x_bits, w_bits):
    """The wide fp16-MFMA stem (stem_wide.hip) takes this conv: the ImageNet conv1 shape class --
    signed <= 9-bit image codes, K <= 480 patch elements, exact fp32 sums (K*2^(xb-1)*2^(wb-1) <= 2^24)."""
    K = d.KH * d.KW * d.Cin
    return (0 < K <= 480 and d.Cout % 16 == 0 and x_bits <= 9 and w_bits <= 8
            and K * 2 ** (x_bits - 1) * 2 ** (w_bits - 1) <= 2 ** 24)


def conv_stem_wide_fwd(x16, w_hwio, d, qx, qw, y):
    M = d.N * d.Ho * d.Wo
    with _Timed("stem_wide_fwd_kernel", x16.numel() * 2 + w_hwio.numel() + M * d.Cout * 4):
        call("lbt_conv_stem_wide_fwd", ptr(x16), ptr(w_hwio), d, qx, qw, ptr(y), stream())


def stem_wide_nsplit(d):
    return int(_lib.load().lbt_stem_wide_nsplit(d))


def conv_stem_wide_wgrad(x16, x_bits, g, d, slab, nsplit):
    """int64 slab [nsplit][K][Cout], every element written; g int8 or int16 codes."""
    with _Timed("stem_wide_wgrad_kernel", x16.numel() * 2 + g.numel() * g.element_size() + slab.numel() * 8):
        call("lbt_conv_stem_wide_wgrad", ptr(x16), int(x_bits), ptr(g), int(g.dtype == torch.int16), d, ptr(slab),
             int(nsplit), stream())


# ----------------------------------------------------------------------------- BN chains
def _chain_fwd_bytes(a):
    per = 0
    for b in ([a.b1, a.b2] if a.has_b2 else [a.b1]):
        per += 1 if b.nrm.q else 4
        per += 1 if b.rout else 0
    per += 4 if a.res else 0
    per += 4 if a.y else 0
    per += 0.25 if a.ybits else 0
    per += _code_bytes(a.o1_kind) if a.o1 else 0
    per += _code_bytes(a.o2_kind) if a.o2 else 0
    return int(per * a.rows * a.inner)


def _chain_bwd_a_bytes(a):
    per = 4 + (4 if a.y_mask else 0) + (4 if a.gmask_out else 0)
    for b in ([a.b1, a.b2] if a.has_b2 else [a.b1]):
        per += 1 if (b.R and (b.qrg.bits or a.mask_from_r)) else 0
        per += 1 if b.qng.bits else 0
        per += 1 if b.gout else (4 if b.dout else 0)
    return per * a.rows * a.inner


def _dgrad_chain_bytes(gq_numel, wd_numel, a, add):
    """lbt_conv_dgrad_chain_i8: the dgrad operands + pass A's element traffic without its fp32 g
    input (it never leaves the GEMM), + the residual addend, + each quantiser's noise table."""
    per = (4 if add else 0) + (4 if a.y_mask else 0) + (4 if a.gmask_out else 0)
    nb = 2 if a.has_b2 else 1
    per += 3 * nb  # R, qn codes in; G codes out
    return gq_numel + wd_numel + per * a.rows * a.inner + nb * 2 * 4 * a.inner


def _chain_bwd_b_bytes(a):
    return (2 + (4 if a.dx else 0) + (1 if a.gq else 0)) * a.rows * a.inner


def bn_moments(nrm, C):
    """Normalization_q's batch moments once (lbt_bn_moments): nrm.ms = [mu | sigma], running averages."""
    with _Timed("bn_moments_kernel", 2 * NSHARD * 2 * C * 8 + 8 * C):
        call("lbt_bn_moments", _lib.ctypes.byref(nrm), int(C), stream())


def chain_fwd(desc):
    with _Timed("chain_fwd_kernel", _chain_fwd_bytes(desc)):
        call("lbt_bn_chain_fwd", _lib.ctypes.byref(desc), stream())


def chain_bwd_a(desc):
    with _Timed("chain_bwd_a_kernel", _chain_bwd_a_bytes(desc)):
        call("lbt_bn_chain_bwd_a", _lib.ctypes.byref(desc), stream())


def chain_bwd_b(desc):
    with _Timed("chain_bwd_b_kernel", _chain_bwd_b_bytes(desc)):
        call("lbt_bn_chain_bwd_b", _lib.ctypes.byref(desc), stream())


# ---- the layer-wise backward's gradient reductions batched: every BN's parameter gradients in ONE
# lbt_bn_param_grads_many launch (53 lbt_bn_param_grads per ResNet-50 step) and every conv's int64 slab
# reduce in ONE lbt_conv_wgrad_reduce64_many launch (53 per step), both at the end of the
# deferred_reductions scope (the Trainer's backward). Nothing reads dW / dgamma / dbeta before the
# backward ends, each layer's slab and pass-A sums are its own (per-layer caches; the sums arena is
# cleared at the next step's start), and the batched kernels do each output's arithmetic as the per-layer
# ones: the same values. Job arrays are uploaded once per distinct job list, outside any graph capture (the
# Trainer's warm-up runs the step eagerly first). LBT_BATCH_PGRADS=0: per layer. The reduces stay per
# layer by default (LBT_BATCH_WREDUCE=1 batches them): deferred, the 1.8 GB of int64 slabs a ResNet-50
# step reduces come back from HBM instead of the cache the wgrad just wrote them through -- 31.9 -> 32.4 ms
# (profiles/round6/batched_reductions_ab.txt); the parameter gradients alone: 32.11 -> 31.79 ms.
_PDEFER = None
_RDEFER = None
_JOBS_DEV = {}


class deferred_reductions:
    def __enter__(self):
        global _PDEFER, _RDEFER
        self.own_p = _PDEFER is None and os.environ.get("LBT_BATCH_PGRADS", "1") == "1"
        self.own_r = _RDEFER is None and os.environ.get("LBT_BATCH_WREDUCE", "0") == "1"
        if self.own_p:
            _PDEFER = []
        if self.own_r:
            _RDEFER = []
        return self

    def __exit__(self, et, ev, tb):
        global _PDEFER, _RDEFER
        pj, rj = (_PDEFER if self.own_p else None), (_RDEFER if self.own_r else None)
        if self.own_p:
            _PDEFER = None
        if self.own_r:
            _RDEFER = None
        if et is None:
            if rj:
                _flush_reduce64(rj)
            if pj:
                _flush_param_grads(pj)
        return False


def _jobs_dev(jobs, T):
    """The device copy of a job list (None inside a capture when it was never uploaded)."""
    key = (T.__name__, b"".join(bytes(j) for j in jobs))
    arr = _JOBS_DEV.get(key)
    if arr is None and not torch.cuda.is_current_stream_capturing():
        buf = (T * len(jobs))(*jobs)
        arr = torch.frombuffer(bytearray(bytes(buf)), dtype=torch.uint8).to(
            torch.device("cuda", torch.cuda.current_device()))
        _JOBS_DEV[key] = arr
    return arr


def _flush_param_grads(jobs):
    arr = _jobs_dev(jobs, _lib.PJob)
    if arr is None:  # per-layer launches
        for j in jobs:
            call("lbt_bn_param_grads", j.sums, int(j.C), j.qrg, j.qr, j.gamma, float(j.wd2), j.dgamma, j.dbeta,
                 stream())
        return
    call("lbt_bn_param_grads_many", ptr(arr), len(jobs), max(int(j.C) for j in jobs), stream())


def _flush_reduce64(jobs):
    nb = 0
    for j in jobs:
        j.first_block = nb
        nb += (int(j.K) * int(j.Cout) + 63) // 64
    arr = _jobs_dev(jobs, _lib.R64Job)
    if arr is None:
        for j in jobs:
            call("lbt_conv_wgrad_reduce64", j.slab, int(j.nsplit), int(j.K), int(j.Cout), j.qx, j.qg, j.w,
                 float(j.wd2), j.dw, stream())
        return
    call("lbt_conv_wgrad_reduce64_many", ptr(arr), len(jobs), nb, stream())


def bn_param_grads(sums, C, qrg, qr, gamma, wd2, dgamma, dbeta):
    ng = _num(dgamma)
    if ng is not None:
        call("lbt_bn_param_grads_x", ptr(sums), int(C), ng, _num(dbeta), stream())
        return
    if _PDEFER is not None:
        _PDEFER.append(_lib.PJob(sums.data_ptr(), int(C), qrg, qr, gamma.data_ptr(), float(wd2), dgamma.data_ptr(),
                                 dbeta.data_ptr()))
        return
    call("lbt_bn_param_grads", ptr(sums), int(C), qrg, qr, ptr(gamma), float(wd2), ptr(dgamma), ptr(dbeta), stream())


# ----------------------------------------------------------------------------- glue
def relu_fwd(x, y):
    call("lbt_relu_fwd", ptr(x), ptr(y), x.numel(), stream())


def relu_bwd(g, x, dx):
    call("lbt_relu_bwd", ptr(g), ptr(x), ptr(dx), g.numel(), stream())


def add(a, b, y):
    call("lbt_add", ptr(a), ptr(b), ptr(y), a.numel(), stream())


def avgpool_fwd(x, y, N, HW, C):
    call("lbt_avgpool_fwd", ptr(x), ptr(y), int(N), int(HW), int(C), stream())


def avgpool_bwd(g, dx, N, HW, C):
    call("lbt_avgpool_bwd", ptr(g), ptr(dx), int(N), int(HW), int(C), stream())


def avgpool_gen_fwd(x, y, d):
    _check(x, torch.float32, "x")
    call("lbt_avgpool_gen_fwd", ptr(x), ptr(y), d, stream())


def avgpool_gen_bwd(g, dx, d):
    _check(g, torch.float32, "g")
    call("lbt_avgpool_gen_bwd", ptr(g), ptr(dx), d, stream())


def softmax_xent(z, labels, loss, dz):
    N, K = z.shape
    s = _XSINK
    if s is not None:  # exact exchange: the mean over the GLOBAL batch, the loss sum into its slot
        call("lbt_softmax_xent_n", ptr(z), ptr(labels), int(N), int(K), int(N * s["world"]), ptr(loss), ptr(dz),
             _lib.ctypes.c_void_p(s["loss"]), stream())
        return
    if K > 64:  # wide heads: one wave per row (the narrow kernel keeps the fused head's order)
        with _Timed("softmax_xent_wide_kernel", 8 * z.numel()):
            call("lbt_softmax_xent_wide", ptr(z), ptr(labels), int(N), int(K), ptr(loss), ptr(dz), stream())
        return
    call("lbt_softmax_xent", ptr(z), ptr(labels), int(N), int(K), ptr(loss), ptr(dz), stream())


def dense_mfma_ok(in_units, units, x_bits, w_bits):
    """Dense_q shapes the int8-MFMA dense kernels take (dense.hip)."""
    return x_bits <= 8 and w_bits <= 8 and in_units % 8 == 0 and units % 8 == 0


def dense_pack(w_hwio, wf, wd):
    IN, OUT = w_hwio.shape
    call("lbt_dense_pack", ptr(w_hwio), int(IN), int(OUT), ptr(wf), int(wf.shape[1]), ptr(wd), int(wd.shape[1]),
         stream())


def dense_gemm(a, b, kvalid, qa, qb, out, kernel="dense_gemm_kernel"):
    rows, cols = out.shape
    with _Timed(kernel, a.numel() * a.element_size() + b.numel() + 4 * out.numel()):
        call("lbt_dense_gemm", ptr(a), int(a.dtype == torch.int16), int(a.shape[1]), int(kvalid), ptr(b),
             int(b.shape[1]), int(rows), int(cols), qa, qb, ptr(out), stream())


def dense_wgrad(xq, g, qx, qg, w, wd2, dw):
    N, IN = xq.shape
    num = _num(dw)
    if num is not None:
        call("lbt_dense_wgrad_x", ptr(xq), ptr(g), int(g.dtype == torch.int16), int(N), int(IN), int(g.shape[1]), num,
             stream())
        return
    with _Timed("dense_wgrad_kernel", xq.numel() + g.numel() * g.element_size() + 8 * w.numel()):
        call("lbt_dense_wgrad", ptr(xq), ptr(g), int(g.dtype == torch.int16), int(N), int(IN), int(g.shape[1]), qx,
             qg, ptr(w), wd2, ptr(dw), stream())


def sgd_momentum(w, a, g, lr, mu, gscale=1.0):
    call("lbt_sgd_momentum", ptr(w), ptr(a), ptr(g), w.numel(), float(lr), float(mu), float(gscale), stream())


def bias_add(y, bq, C):
    call("lbt_bias_add", ptr(y), ptr(bq), y.numel(), int(C), stream())


def bias_grad(chsum, C, qg, db):
    call("lbt_bias_grad", ptr(chsum), int(C), qg, ptr(db), stream())


def f32(x):
    return torch.tensor(x, dtype=torch.float32).item()


# ---------------------------------------------------------------- either side of the hot path
def grad_buffer_bwd(g, buffer, q_desc, inner):
    """GradientBuffer_q.backward (lbt_grad_buffer_bwd): returns gq [g.shape]; buffer updated."""
    _check(g, torch.float32, "g")
    _check(buffer, torch.float32, "buffer")
    gq = torch.empty_like(g)
    call("lbt_grad_buffer_bwd", ptr(g), g.numel(), ptr(buffer), buffer.numel(), int(inner), q_desc, ptr(gq), stream())
    return gq


def pre_dense(grad, qg_desc, accu, init_flag, rem_flag):
    """Dense_q._pre_dense_func (lbt_pre_dense), in place on grad [rows, cols]."""
    _check(grad, torch.float32, "grad")
    rows, cols = grad.shape
    call("lbt_pre_dense", ptr(grad), rows, cols, accu.shape[0], accu.shape[1], qg_desc, ptr(accu), ptr(init_flag),
         ptr(rem_flag), stream())
    return grad


def augment_flip_crop(x, pad, seed, counter, out=None):
    """preprocess_image (trainer.py:24-28) on device: random flip + zero pad + random crop."""
    _check(x, torch.float32, "x")
    N, H, W, C = x.shape
    if out is None:
        out = torch.empty_like(x)
    call("lbt_augment_flip_crop", ptr(x), ptr(out), N, H, W, C, int(pad), int(seed) & 0xFFFFFFFFFFFFFFFF,
         int(counter) & 0xFFFFFFFFFFFFFFFF, stream())
    return out


def maxpool_fwd(x, y, amax, d):
    _check(x, torch.float32, "x")
    with _Timed("maxpool_fwd_kernel", 4 * x.numel() + 5 * y.numel()):
        call("lbt_maxpool_fwd", ptr(x), ptr(y), ptr(amax), d, stream())


def maxpool_relu_fwd(x, y, amax, d):
    """MaxPool_q of the preceding ReLU_q's output, from the ReLU's input x (one pass)."""
    _check(x, torch.float32, "x")
    with _Timed("maxpool_fwd_kernel", 4 * x.numel() + 5 * y.numel()):
        call("lbt_maxpool_relu_fwd", ptr(x), ptr(y), ptr(amax), d, stream())


def maxpool_bwd(g, amax, dx, d):
    _check(g, torch.float32, "g")
    with _Timed("maxpool_bwd_kernel", 5 * g.numel() + 4 * dx.numel()):
        call("lbt_maxpool_bwd", ptr(g), ptr(amax), ptr(dx), d, stream())


def maxpool_relu_bwd(g, amax, y, dx, d):
    """MaxPool_q backward with the preceding ReLU_q's backward folded in (y: the pool's output; None when
    amax comes from maxpool_relu_fwd, whose codes carry the mask)."""
    with _Timed("maxpool_bwd_kernel", (9 if y is not None else 5) * g.numel() + 4 * dx.numel()):
        call("lbt_maxpool_relu_bwd", ptr(g), ptr(amax), ptr(y), ptr(dx), d, stream())


# ---------------------------------------------------------------- 9..16-bit gradient codes
def conv_dgrad_generic16(gq, w_hwio, d, qg, qw, dx, add_src=None):
    with _Timed("conv_dgrad_generic_kernel16", 2 * gq.numel() + w_hwio.numel() + 4 * dx.numel()):
        call("lbt_conv_dgrad_generic16", ptr(gq), ptr(w_hwio), d, qg, qw, ptr(dx), ptr(add_src), stream())


def conv_wgrad_generic16(xq, x_i16, gq, d, slab, nsplit):
    with _Timed("conv_wgrad_generic_kernel16", xq.numel() * xq.element_size() + 2 * gq.numel() + 8 * slab.numel()):
        call("lbt_conv_wgrad_generic16", ptr(xq), int(x_i16), ptr(gq), d, ptr(slab), int(nsplit), stream())


def conv_wgrad_reduce64(slab, nsplit, K, Cout, qx, qg, w, wd2, dw):
    num = _num(dw)
    if num is not None:
        call("lbt_conv_wgrad_reduce64_x", ptr(slab), int(nsplit), int(K), int(Cout), num, stream())
        return
    if _RDEFER is not None:
        _RDEFER.append(_lib.R64Job(slab.data_ptr(), int(nsplit), int(K), int(Cout), 0, qx, qg, w.data_ptr(),
                                   float(wd2), dw.data_ptr()))
        return
    call("lbt_conv_wgrad_reduce64", ptr(slab), int(nsplit), int(K), int(Cout), qx, qg, ptr(w), wd2, ptr(dw), stream())


def bn_bwd_a_wide(g, qrg, R, gamma_q, qng, qn, gout, dout, sums, rows, inner, C):
    call("lbt_bn_bwd_a_wide", ptr(g), qrg, ptr(R), ptr(gamma_q), qng, ptr(qn), ptr(gout), ptr(dout), ptr(sums),
         int(rows), int(inner), int(C), stream())


def bn_bwd_b_wide(G, qng, qn, qn_q, ms, sums, n, dx, rows, C):
    call("lbt_bn_bwd_b_wide", ptr(G), qng, ptr(qn), qn_q, ptr(ms), ptr(sums), int(n), ptr(dx), int(rows), int(C),
         stream())


# ---------------------------------------------------------------- wide layers (igemm.hip)
def bn_bwd_a_wide_masked(g, y_mask, mask_r, qr, gb, gmask_out, qrg, R, qng, qn, gout, sums, rows, inner, C, g2=None,
                         y_bits=None):
    """y_bits: the ReLU mask as chain_fwd's ybits (one byte per channel quad) instead of fp32 y_mask."""
    with _Timed("bn_bwd_a_wide_kernel", g.numel() * (4 + 1 + 1 + 2) + (4 * g.numel() if y_mask is not None else 0)
                + (g.numel() // 4 if y_bits is not None else 0)
                + (4 * g.numel() if gmask_out is not None else 0) + (4 * g.numel() if g2 is not None else 0)):
        call("lbt_bn_bwd_a_wide_masked", ptr(g), ptr(g2), ptr(y_mask), ptr(y_bits), int(mask_r), qr, ptr(gb),
             ptr(gmask_out), qrg, ptr(R), qng, ptr(qn), ptr(gout), None, ptr(sums), int(rows), int(inner), int(C),
             stream())


def bn_bwd_b_wide_q(G, qng, qn, qn_q, ms, sums, n, gq, qo, rows, inner, C):
    with _Timed("bn_bwd_b_wide_kernel", G.numel() * (2 + 1 + 2)):
        call("lbt_bn_bwd_b_wide_q", ptr(G), qng, ptr(qn), qn_q, ptr(ms), ptr(sums), int(n), ptr(gq), qo, int(rows),
             int(inner), int(C), stream())


def igemm_ok(c_gather, c_out):
    """Shapes the LDS-tiled MFMA implicit GEMM takes: gathered channels % 64, outputs % 16."""
    return c_gather % 64 == 0 and c_out % 16 == 0


def igemm_tuning():
    """The 256-row LDS-DMA GEMM's selection (lbt_igemm_get_tuning): dict big / min_tiles / stages / max_bn,
    and `launches`, the number of 256-row GEMM launches this process has issued."""
    t = _lib.IgemmTuning()
    call("lbt_igemm_get_tuning", _lib.ctypes.byref(t))
    return {f: getattr(t, f) for f, _ in t._fields_}


class igemm_forced:
    """Context manager: set the 256-row GEMM's selection for the calls made inside (tests force it onto
    any shape / variant), restore the previous selection on exit."""

    def __init__(self, **kw):
        self.kw = kw

    def __enter__(self):
        self.saved = igemm_tuning()
        t = _lib.IgemmTuning(**dict(self.saved, **self.kw))
        call("lbt_igemm_set_tuning", _lib.ctypes.byref(t))
        return self

    def __exit__(self, *exc):
        call("lbt_igemm_set_tuning", _lib.ctypes.byref(_lib.IgemmTuning(**self.saved)))
        return False


def igemm_workspace_bytes(d, mode, a16):
    return int(_lib.load().lbt_igemm_workspace_bytes(d, int(mode), int(a16)))


def conv_fwd_igemm_ws(xq, a_kind, wf, ksf, d, qx, qw, y, ws):
    M = d.N * d.Ho * d.Wo
    with _Timed("igemm_kernel<fwd>", xq.numel() * xq.element_size() + wf.numel() + 4 * M * d.Cout):
        call("lbt_conv_fwd_igemm_ws", ptr(xq), int(a_kind), ptr(wf), int(ksf), None, d, qx, qw, ptr(y), ptr(ws),
             0 if ws is None else ws.numel() * ws.element_size(), stream())


def conv_dgrad_igemm_ws(gq, g_i16, wd, ksd, d, qg, qw, dx, ws, add_src=None):
    with _Timed("igemm_kernel<dgrad>", gq.numel() * gq.element_size() + wd.numel() + 4 * dx.numel()):
        call("lbt_conv_dgrad_igemm_ws", ptr(gq), int(g_i16), ptr(wd), int(ksd), d, qg, qw, ptr(dx), ptr(add_src),
             ptr(ws), 0 if ws is None else ws.numel() * ws.element_size(), stream())


NOISE_TABLES = os.environ.get("LBT_EPI_NOISE_TABLE", "1") == "1"


def conv_dgrad_igemm_bna(gq16, wd, ksd, d, qg, qw, qr, R, gb, qrg, qng, qn, gout, sums, dx, ws):
    """16-bit-gradient dgrad whose dx is the incoming gradient of a ReLU_q + BN pass A (mask from the
    Rescale_q codes R, lbt_conv_dgrad_igemm_bna): G codes `gout` + the channel sums + both quantisers'
    counters, in the 256-row GEMM's epilogue when that kernel takes the GEMM (no fp32 dx), else through
    dx (scratch) and bn_bwd_a_wide_masked. qrg / qng: Quantizer objects (stochastic ones read this
    step's noise tables over H*W*Cin); qr: the R codes' descriptor."""
    inner = d.H * d.W * d.Cin
    descs = []
    for q in (qrg, qng):
        descs.append(q.ctx.noise_table_desc(q, inner) if (NOISE_TABLES and q.stochastic) else q.desc)
    b = _lib.DgradBna(qr, ptr(R), ptr(gb), descs[0], descs[1], ptr(qn), ptr(gout), ptr(sums))
    n = d.N * inner
    with _Timed("igemm_kernel<dgrad+bn_a>", gq16.numel() * 2 + wd.numel() + 4 * n):
        call("lbt_conv_dgrad_igemm_bna", ptr(gq16), ptr(wd), int(ksd), d, qg, qw, ctypes.byref(b), ptr(dx), ptr(ws),
             0 if ws is None else ws.numel() * ws.element_size(), stream())


def conv_dgrad_igemm_bn3(gq16, wd, ksd, d, qg, qw, g2, y_bits, gmask_out, bns, dx, ws):
    """16-bit-gradient dgrad whose dx, plus g2 and masked by y_bits, is the gradient entering a
    bottleneck block (lbt_conv_dgrad_igemm_bn3): the masked sum optionally out (gmask_out), then pass A
    of each BN in `bns` -- tuples (R, gamma_q, qrg, qng, qn, gout, sums), qrg / qng Quantizer objects --
    in the 256-row GEMM's epilogue when that kernel takes the GEMM, else through dx (scratch)."""
    inner = d.H * d.W * d.Cin
    b = _lib.DgradBn3()
    b.g2, b.y_bits, b.gmask_out, b.nbn = ptr(g2), ptr(y_bits), ptr(gmask_out), len(bns)
    for k, (R, gamma_q, qrg, qng, qn, gout, sums) in enumerate(bns):
        dr, dn = [q.ctx.noise_table_desc(q, inner) if (NOISE_TABLES and q.stochastic) else q.desc for q in (qrg, qng)]
        b.bn[k] = _lib.BnaBn(dr, ptr(R), ptr(gamma_q), dn, ptr(qn), ptr(gout), ptr(sums))
    n = d.N * inner
    nb = gq16.numel() * 2 + wd.numel() + n * (4 + 0.25 + (4 if gmask_out is not None else 0) + 4 * len(bns))
    with _Timed("igemm_kernel<dgrad+bn3_a>", int(nb)):
        call("lbt_conv_dgrad_igemm_bn3", ptr(gq16), ptr(wd), int(ksd), d, qg, qw, ctypes.byref(b), ptr(dx), ptr(ws),
             0 if ws is None else ws.numel() * ws.element_size(), stream())


def conv_fwd_igemm_q(xq, a_kind, wf, ksf, d, qx, qw, yq, qout, chsum):
    """Wide fwd + the Normalization_q input quantiser in its epilogue (int8 codes, sums, counters).
    A stochastic qout reads its noise from the context's per-step table (one Philox call per 4 noise
    values per step instead of one per 4 outputs of every sample)."""
    M = d.N * d.Ho * d.Wo
    qout.observe(M * d.Cout)
    qd = qout.desc
    if NOISE_TABLES and qout.stochastic:
        qd = qout.ctx.noise_table_desc(qout, d.Ho * d.Wo * d.Cout)
    with _Timed("igemm_kernel<fwd>", xq.numel() * xq.element_size() + wf.numel() + M * d.Cout):
        call("lbt_conv_fwd_igemm_q", ptr(xq), int(a_kind), ptr(wf), int(ksf), d, qx, qw, ptr(yq), qd,
             ptr(chsum), stream())


def conv_fwd_igemm(xq, a_kind, wf, ksf, d, qx, qw, y):
    M = d.N * d.Ho * d.Wo
    with _Timed("igemm_kernel<fwd>", xq.numel() * xq.element_size() + wf.numel() + 4 * M * d.Cout):
        call("lbt_conv_fwd_igemm", ptr(xq), int(a_kind), ptr(wf), int(ksf), None, d, qx, qw, ptr(y), stream())


def conv_dgrad_igemm(gq, g_i16, wd, ksd, d, qg, qw, dx, add_src=None):
    with _Timed("igemm_kernel<dgrad>", gq.numel() * gq.element_size() + wd.numel() + 4 * dx.numel()):
        call("lbt_conv_dgrad_igemm", ptr(gq), int(g_i16), ptr(wd), int(ksd), d, qg, qw, ptr(dx), ptr(add_src),
             stream())


def wgrad_igemm_nsplit(d):
    """Pixel splits of the wide wgrad: ~1024 workgroups, int32 MFMA sums exact (<= 2^17 pixels a wave)."""
    P = d.N * d.Ho * d.Wo
    tiles = d.KH * d.KW * (d.Cin // 64) * (d.Cout // 64)
    lo = -(-P // (4 * 131072))
    return max(lo, min(max(1, P // 256), -(-1024 // tiles)))


WGRAD3 = os.environ.get("LBT_WGRAD3", "1") != "0"


def wgrad3_ok(d):
    """lbt_conv_wgrad_igemm_store's all-taps 3x3 body takes this conv (wgrad3_ok in igemm.hip)."""
    if not WGRAD3:
        return False
    if (d.KH, d.KW, d.SH, d.SW, d.PT, d.PB, d.PL, d.PR) != (3, 3, 1, 1, 1, 1, 1, 1) or d.Ho != d.H or d.Wo != d.W:
        return False
    if d.W > 64 or d.Cin % 64 or d.Cout % 64:
        return False
    return (64 // d.W + 2) * (d.W + 2) <= 192


WGRAD1 = os.environ.get("LBT_WGRAD1", "1") != "0"


def wgrad1_wci(d):
    """lbt_conv_wgrad_igemm_store's 1x1 body (16-bit G) takes this conv with (64 wci) x (256 / wci)
    channel tiles (wgrad1_wci in igemm.hip); 0: not taken."""
    if not WGRAD1 or (d.KH, d.KW, d.PT, d.PL) != (1, 1, 0, 0) or d.PB < 0 or d.PR < 0:
        return 0
    if (d.Ho - 1) * d.SH >= d.H or (d.Wo - 1) * d.SW >= d.W:
        return 0
    if d.Cin % 128 == 0 and d.Cout % 128 == 0:
        return 2
    if d.Cin % 64 == 0 and d.Cout % 256 == 0:
        return 1
    if d.Cin % 256 == 0 and d.Cout % 64 == 0:
        return 4
    return 0


def wgrad_store_nsplit(d, g_i16=True):
    """Pixel splits of the storing wide wgrad: >= ~512 workgroups, each split's slab written once.
    All-taps 3x3 body: splits of whole-row chunks, ~256 workgroups (one per CU; each covers all 9
    taps of a 64 x 64 channel block), <= 1024 chunks a split. 1x1 body (16-bit G): 64-pixel
    chunks, ~512 workgroups, <= 2047 chunks a split (int32 MFMA sums < 2^31)."""
    wci = wgrad1_wci(d) if g_i16 else 0
    if wci:
        chunks = -(-(d.N * d.Ho * d.Wo) // 64)
        nblk = (d.Cin // (64 * wci)) * (d.Cout // (256 // wci))
        return min(chunks, max(-(-chunks // 2047), -(-512 // nblk)))
    if wgrad3_ok(d):
        rb = 64 // d.W
        chunks = d.N * (-(-d.H // rb))
        nblk = (d.Cin // 64) * (d.Cout // 64)
        return min(chunks, max(-(-chunks // 1024), -(-256 // nblk)))
    P = d.N * d.Ho * d.Wo
    tiles = d.KH * d.KW * (d.Cin // 64) * (d.Cout // 64)
    lo = -(-P // (4 * 131072))
    return max(lo, min(max(1, P // 1024), -(-512 // tiles)))


def conv_wgrad_igemm_store(xq, gq, g_i16, d, slab, nsplit):
    with _Timed("wgrad_wide_kernel", xq.numel() + gq.numel() * gq.element_size() + 8 * slab.numel()):
        call("lbt_conv_wgrad_igemm_store", ptr(xq), ptr(gq), int(g_i16), d, ptr(slab), int(nsplit), stream())


def conv_wgrad_igemm(xq, gq, g_i16, d, slab, nsplit, nshard):
    with _Timed("wgrad_wide_kernel", xq.numel() + gq.numel() * gq.element_size() + 8 * slab.numel()):
        call("lbt_conv_wgrad_igemm", ptr(xq), ptr(gq), int(g_i16), d, ptr(slab), int(nsplit), int(nshard), stream())
