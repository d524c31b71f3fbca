"""DFXP quantiser + overflow-rate range controller (oracle; test infrastructure only).

Restates ``dynamic_fixed_point.py:4-94`` of the reference:

* ``weight_quantization`` (``:4-45``): ``bits == 32`` bypass (``:21-23``); the
  nearest STE ``round(clip(X*m, -L, L-1)) / m`` (``:26-30``, ``tf.round`` is
  round-half-to-even); the stochastic STE
  ``floor(clip(X*m + U[0,1)^{X.shape[1:]}, -L, L-1)) / m`` (``:33-38``);
  ``m = 2**(bits-I-1)``, ``L = 2**(bits-1)``.
* ``overflow_rate`` (``:48-67``): fractions of ``X*m >= L or X*m < -L`` and of
  ``X*m >= L/2 or X*m < -L/2`` on the *unquantised* X (note the asymmetric
  ``>=`` / ``<`` boundaries, ``:63-66``).
* ``update_range`` (``:70-94``): ``delta = +1 if ovf > t else (-1 if ovf2 <= t
  else 0)``; ``I <- min(bits-1, I+delta)``.

Build decisions (documented in DESIGN.md):
* The quantiser uses I_t and its statistics are taken against I_t; I_{t+1} is
  applied after the step (the reference leaves this ordering racy).
* The reference computes ``2**e`` in int32, so it is only defined for
  ``0 <= e = bits-I-1 <= 30``. The build clamps I to ``[bits-31, bits-1]``
  (the upper clamp is the reference's own ``tf.minimum``; the lower one keeps e
  inside the reference's defined domain).
* Quantised values are returned as integers ``q`` with the shared exponent ``e``
  (value = q * 2**-e): that is what the HIP path stores (int8 / offset-uint8).
"""
import zlib

import numpy as np

from .philox import uniform_noise

E_MAX = 30


def qid_of(name):
    """Stable 31-bit quantiser id from the range variable's name (e.g. ``block16-1-1/X_range``)."""
    return zlib.crc32(name.encode("utf-8")) & 0x7FFFFFFF


def frac_bits(bits, I):
    """e = bits - I - 1 (``dynamic_fixed_point.py:27,34``)."""
    e = int(bits) - int(I) - 1
    if not 0 <= e <= E_MAX:
        raise ValueError("DFXP exponent outside the reference's defined range: bits=%d I=%d" % (bits, I))
    return e


def clamp_I(bits, I):
    return max(int(bits) - 1 - E_MAX, min(int(bits) - 1, int(I)))


def noise_for(shape, qid, step, seed):
    """U[0,1) noise of shape X.shape[1:] (``dynamic_fixed_point.py:36``)."""
    inner = int(np.prod(shape[1:])) if len(shape) > 1 else 1
    u = uniform_noise(inner, qid, step, seed)
    return u.reshape(shape[1:]) if len(shape) > 1 else u.reshape(())


def quantize_int(x, bits, I, stochastic, noise=None):
    """Integer DFXP code of ``x`` (fp32). Returns int32 array q with value q * 2**-e."""
    x = np.asarray(x, dtype=np.float32)
    e = frac_bits(bits, I)
    m = np.float32(2.0 ** e)
    L = np.float32(2.0 ** (bits - 1))
    xm = (x * m).astype(np.float32)
    if stochastic:
        v = (xm + np.asarray(noise, dtype=np.float32)).astype(np.float32)
        q = np.floor(np.clip(v, -L, L - np.float32(1)))
    else:
        q = np.rint(np.clip(xm, -L, L - np.float32(1)))
    return q.astype(np.int32)


def dequant(q, e):
    return (np.asarray(q).astype(np.float32) * np.float32(2.0 ** -e)).astype(np.float32)


def overflow_counts(x, bits, I):
    """Counts behind ``overflow_rate`` (``dynamic_fixed_point.py:60-67``)."""
    x = np.asarray(x, dtype=np.float32)
    e = frac_bits(bits, I)
    m = np.float32(2.0 ** e)
    L = np.float32(2.0 ** (bits - 1))
    xm = (x * m).astype(np.float32)
    c1 = int(np.count_nonzero(xm >= L) + np.count_nonzero(xm < -L))
    c2 = int(np.count_nonzero(xm >= L / np.float32(2)) + np.count_nonzero(xm < -(L / np.float32(2))))
    return c1, c2


def overflow_rate(x, bits, I):
    c1, c2 = overflow_counts(x, bits, I)
    n = np.float32(np.asarray(x).size)
    return np.float32(c1) / n, np.float32(c2) / n


def update_range_from_counts(c1, c2, n, target, bits, I):
    """``update_range`` (``dynamic_fixed_point.py:83-94``) given overflow counts over n elements."""
    r1 = np.float32(c1) / np.float32(n)
    r2 = np.float32(c2) / np.float32(n)
    t = np.float32(target)
    delta = 1 if r1 > t else (-1 if r2 <= t else 0)
    return clamp_I(bits, min(int(bits) - 1, int(I) + delta))


def overflow_rates_f32(x, bits, I):
    """``overflow_rate`` as the reference computes it (``:60-67``): fp32 masks, fp32 reduce_mean
    (pairwise fp32 sum / n). Equal to count / n whenever n < 2**24 (every partial sum of 0/1/2
    values is then an exact integer)."""
    x = np.asarray(x, dtype=np.float32).reshape(-1)
    e = frac_bits(bits, I)
    m = np.float32(2.0 ** e)
    L = np.float32(2.0 ** (bits - 1))
    xm = (x * m).astype(np.float32)
    m1 = (xm >= L).astype(np.float32) + (xm < -L).astype(np.float32)
    m2 = (xm >= L / np.float32(2)).astype(np.float32) + (xm < -(L / np.float32(2))).astype(np.float32)
    n = np.float32(x.size)
    return (np.add.reduce(m1, dtype=np.float32) / n).astype(np.float32), \
        (np.add.reduce(m2, dtype=np.float32) / n).astype(np.float32)


def update_range_from_rates(r1, r2, target, bits, I):
    """``update_range`` (``:83-94``) given the two fp32 rates."""
    t = np.float32(target)
    delta = 1 if np.float32(r1) > t else (-1 if np.float32(r2) <= t else 0)
    return clamp_I(bits, min(int(bits) - 1, int(I) + delta))


def update_range(x, target, bits, I):
    c1, c2 = overflow_counts(x, bits, I)
    return update_range_from_counts(c1, c2, np.asarray(x).size, target, bits, I)


def weight_quantization(x, target, bits, I, stochastic=False, noise=None):
    """Fake-quantised fp32 output and the next exponent (``dynamic_fixed_point.py:4-45``)."""
    assert 1 <= bits <= 32, "invalid value for bits: %d" % bits
    x = np.asarray(x, dtype=np.float32)
    if bits == 32:
        return x, I
    q = quantize_int(x, bits, I, stochastic, noise)
    return dequant(q, frac_bits(bits, I)), update_range(x, target, bits, I)
