"""Components either side of the hot path (oracle; test infrastructure only).

* ``GradientBufferQ``  -- ``GradientBuffer_q`` (``dynamic_fixed_point.py:473-509``): error-feedback
  gradient quantisation. backward: ``total = pad(grad, buffer.shape) + buffer``;
  ``gq = weight_quantization(total, bits, grad_range, stochastic=True)`` (``:501-502``);
  ``buffer <- total - gq`` (``:503``); returns ``gq[:grad.shape[0]]`` (``:506``).
* ``pre_dense``        -- ``Dense_q._pre_dense_func`` (``:405-439``), the per-element small-gradient
  accumulator (state initialised at ``:364-366,449``: init_flag = 1, rem_flag = 0, accu = 0.001;
  eps = 1 / 2**(bits - grad_range), ``:444``). Restated loop for loop, in float32.
* ``augment_flip_crop`` -- ``preprocess_image`` (``trainer.py:24-28``): random left-right flip,
  ``pad_to_bounding_box(4, 4, 40, 40)``, ``random_crop([32, 32, 3])``. TF's draws are not
  reproducible outside TF; the build draws per sample with Philox4x32-10 (see
  ``lbt_amd/csrc/aux.hip``) and this restates that draw, so the transform is pinned given it.
"""
import numpy as np

from . import dfxp
from .philox import philox4x32_10

F32 = np.float32
AUG_STREAM = 0x41554721


class GradientBufferQ:
    def __init__(self, name, bits, shape):
        self.name, self.bits = name, bits
        self.buffer = np.zeros(shape, dtype=F32)

    def backward(self, grad, ctx):
        grad = np.asarray(grad, dtype=F32)
        pad = [(0, s - g) for s, g in zip(self.buffer.shape, grad.shape)]
        total = (np.pad(grad, pad) + self.buffer).astype(F32)
        if self.bits == 32:
            gq = total
        else:
            q, e = ctx.q(self.name + "/grad_range", total, self.bits)
            gq = (q.astype(F32) * F32(2.0 ** -e)).astype(F32)
        self.buffer = (total - gq).astype(F32)
        return gq[:grad.shape[0]]


def pre_dense(grad, eps, accu, init_flag, rem_flag):
    """In place on copies: returns (grad, accu, init_flag, rem_flag) after _pre_dense_func."""
    grad = np.array(grad, dtype=F32)
    accu = np.array(accu, dtype=F32)
    init_flag = np.array(init_flag)
    rem_flag = np.array(rem_flag)
    eps = F32(eps)
    for i in range(grad.shape[0]):
        for j in range(grad.shape[1]):
            if init_flag[i, j] == 1:
                if eps > np.absolute(grad[i, j]):
                    init_flag[i, j] = 0
                    if rem_flag[i, j] == 1:
                        accu[i, j] = F32(accu[i, j] + grad[i, j])
                    else:
                        accu[i, j] = grad[i, j]
            else:
                accu[i, j] = F32(accu[i, j] + grad[i, j])
                if np.absolute(accu[i, j]) > eps:
                    init_flag[i, j] = 1
                    grad[i, j] = accu[i, j]
                    if accu[i, j] > 0:
                        accu[i, j] = F32(accu[i, j] - F32(accu[i, j] // eps) * eps)
                    else:
                        accu[i, j] = F32(accu[i, j] + F32((-accu[i, j]) // eps) * eps)
                    rem_flag[i, j] = 1
    return grad, accu, init_flag, rem_flag


def pre_dense_eps(bits, grad_range):
    return F32(1.0 / (2 ** (bits - grad_range)))


def augment_draws(N, pad, seed, counter):
    n = np.arange(N, dtype=np.uint32)
    r = philox4x32_10(n, np.full(N, AUG_STREAM, np.uint32), np.full(N, counter & 0xFFFFFFFF, np.uint32),
                      np.full(N, (counter >> 32) & 0xFFFFFFFF, np.uint32), seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    span = np.uint32(2 * pad + 1)
    return (r[0] & np.uint32(1)).astype(np.int64), (r[1] % span).astype(np.int64), (r[2] % span).astype(np.int64)


def augment_flip_crop(x, pad, seed, counter):
    x = np.asarray(x, dtype=F32)
    N, H, W, C = x.shape
    flip, oy, ox = augment_draws(N, pad, seed, counter)
    out = np.zeros_like(x)
    for n in range(N):
        img = x[n, :, ::-1, :] if flip[n] else x[n]
        padded = np.zeros((H + 2 * pad, W + 2 * pad, C), dtype=F32)
        padded[pad:pad + H, pad:pad + W] = img
        out[n] = padded[oy[n]:oy[n] + H, ox[n]:ox[n] + W]
    return out
