"""Drop-in counterpart of the reference module ``dynamic_fixed_point.py`` (TF face).

``import lbt_amd.dynamic_fixed_point as dfxp`` gives the names ``models.py`` uses:
``weight_quantization``, ``overflow_rate``, ``update_range`` (``:4-94``) and the Layer_q classes
(``:97-1053``), all running on the gfx950 HIP kernels of ``liblbt_dfxp.so``.

A range variable (the reference's int32 ``integer_bits`` tf.Variable) is a
:class:`lbt_amd.runtime.Quantizer`; create one with ``ctx.quantizer(name, bits, initial)``.
"""
import torch

from . import _lib
from ._lib import CSTRIDE, NSHARD, OUT_F32, QDesc
from .dfxp import ops
from .dfxp.layers import (AvgPool_q, BatchNorm_q, Conv2d_pq, Conv2d_q, Dense_q, Flatten_q,  # noqa: F401
                          GradientBuffer_q, Layer_q, MaxPool_q, Normalization_q, ReLU_q, Rescale_q,
                          ResidualBlock_q, ResidualBottleneck_q, Sequential_q)
from .runtime import DfxpContext, Quantizer, default_context  # noqa: F401


def _desc_for(q, bits, stochastic):
    if bits != q.bits:
        raise ValueError("range variable %s was registered for %d bits, called with %d" % (q.name, q.bits, bits))
    d = QDesc.from_buffer_copy(q.desc)
    d.stochastic = 1 if stochastic else 0
    return d


def weight_quantization(X, target_overflow_rate, bits, integer_bits, stochastic=False):
    """Fake-quantise X to DFXP (``dynamic_fixed_point.py:4-45``); the overflow statistics feed
    ``integer_bits``'s pending range update (``ctx.update_range_op()``). Returns fp32 q * 2^-e."""
    assert 1 <= bits <= 32, "invalid value for bits: %d" % bits
    if bits == 32:
        return X
    q = integer_bits
    X = X.contiguous()
    rows, inner = ops.rows_inner(tuple(X.shape))
    out = torch.empty_like(X)
    q.observe(X.numel())
    _lib.call("lbt_dfxp_quantize", _lib.ptr(X), _lib.ptr(out), OUT_F32, rows, inner,
              _desc_for(q, bits, stochastic), None, 0, _lib.stream())
    return out


def _scratch_counts(X, bits, integer_bits):
    """Overflow counts of X against integer_bits's current I, without touching its pending stats."""
    ctx = integer_bits.ctx
    X = X.contiguous()
    exps = ctx.exps[integer_bits.slot:integer_bits.slot + 1].clone()
    counts = torch.zeros(NSHARD * CSTRIDE, dtype=torch.int32, device=X.device)
    d = QDesc(exps.data_ptr(), counts.data_ptr(), ctx.step.data_ptr(), ctx.seed, integer_bits.qid, 0, bits, 0)
    rows, inner = ops.rows_inner(tuple(X.shape))
    out = torch.empty_like(X)
    _lib.call("lbt_dfxp_quantize", _lib.ptr(X), _lib.ptr(out), OUT_F32, rows, inner, d, None, 0, _lib.stream())
    c = counts.view(NSHARD, CSTRIDE)[:, :2].sum(0).tolist()
    return c[0], c[1], exps


def overflow_rate(X, bits, integer_bits):
    """(overflow_rate(X), overflow_rate(2X)) of ``dynamic_fixed_point.py:48-67`` (host floats)."""
    c1, c2, _ = _scratch_counts(X, bits, integer_bits)
    n = torch.tensor(float(X.numel()), dtype=torch.float32)
    return (torch.tensor(float(c1), dtype=torch.float32) / n).item(), \
        (torch.tensor(float(c2), dtype=torch.float32) / n).item()


def update_range(X, target_overflow_rate, bits, integer_bits):
    """Apply ``update_range`` (``dynamic_fixed_point.py:70-94``) for tensor X to integer_bits now."""
    ctx = integer_bits.ctx
    X = X.contiguous()
    exps = ctx.exps[integer_bits.slot:integer_bits.slot + 1]
    counts = torch.zeros(NSHARD * CSTRIDE, dtype=torch.int32, device=X.device)
    d = QDesc(exps.data_ptr(), counts.data_ptr(), ctx.step.data_ptr(), ctx.seed, integer_bits.qid, 0, bits, 0)
    rows, inner = ops.rows_inner(tuple(X.shape))
    out = torch.empty_like(X)
    _lib.call("lbt_dfxp_quantize", _lib.ptr(X), _lib.ptr(out), OUT_F32, rows, inner, d, None, 0, _lib.stream())
    dev = X.device
    bits_t = torch.tensor([bits], dtype=torch.int32, device=dev)
    tgt = torch.tensor([target_overflow_rate], dtype=torch.float32, device=dev)
    nel = torch.tensor([float(X.numel())], dtype=torch.float32, device=dev)
    dummy_step = torch.zeros(1, dtype=torch.int64, device=dev)
    _lib.call("lbt_dfxp_range_update", _lib.ptr(exps), _lib.ptr(counts), _lib.ptr(bits_t), _lib.ptr(tgt),
              _lib.ptr(nel), 1, _lib.ptr(dummy_step), _lib.stream())
    return integer_bits


def update_range_op(ctx=None):
    """Run the whole ``'update_range'`` collection (``trainer.py:63,157``)."""
    (ctx or default_context()).update_range_op()
