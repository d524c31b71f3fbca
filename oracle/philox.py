"""Philox4x32-10 counter-based RNG in numpy (oracle; test infrastructure only).

The reference draws its rounding noise with ``tf.random_uniform(X.shape[1:], 0, 1)``
(``dynamic_fixed_point.py:36``): one U[0,1) value per element of ``X.shape[1:]``,
broadcast over dim 0. TF's stateful Philox stream is not reproducible outside
TF, so the build fixes its own stream and both this oracle and the HIP kernels
(``lbt_amd/csrc/dfxp_device.h``) implement it identically:

    noise index i in [0, prod(X.shape[1:]))
    counter = (i >> 2, qid, step_lo, step_hi), key = (seed_lo, seed_hi)
    r = Philox4x32_10(counter, key)[i & 3]
    u = (r >> 8) * 2**-24                      # exact in fp32, u in [0, 1)

Pinned by the Random123 known-answer vectors (tests/golden/kat_philox.json).
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32 with 10 rounds. All inputs uint32 (arrays or scalars)."""
    c0 = np.asarray(c0, dtype=np.uint32)
    c1 = np.asarray(c1, dtype=np.uint32)
    c2 = np.asarray(c2, dtype=np.uint32)
    c3 = np.asarray(c3, dtype=np.uint32)
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    with np.errstate(over="ignore"):
        for r in range(10):
            if r:
                k0 = np.uint32(k0 + W0)
                k1 = np.uint32(k1 + W1)
            p0 = M0 * c0.astype(np.uint64)
            p1 = M1 * c2.astype(np.uint64)
            hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
            lo0 = (p0 & MASK32).astype(np.uint32)
            hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
            lo1 = (p1 & MASK32).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
    return c0, c1, c2, c3


def uniform_noise(inner, qid, step, seed):
    """The ``inner`` noise values for quantiser ``qid`` at training step ``step``.

    Returns float32 array of shape [inner] with values k * 2**-24, k in [0, 2**24).
    """
    inner = int(inner)
    nblk = (inner + 3) // 4
    blk = np.arange(nblk, dtype=np.uint64).astype(np.uint32)
    qid = np.uint32(int(qid) & 0xFFFFFFFF)
    step = int(step)
    s_lo = np.uint32(step & 0xFFFFFFFF)
    s_hi = np.uint32((step >> 32) & 0xFFFFFFFF)
    seed = int(seed)
    r = philox4x32_10(blk, np.full(nblk, qid, np.uint32), np.full(nblk, s_lo, np.uint32),
                      np.full(nblk, s_hi, np.uint32), seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    out = np.stack(r, axis=1).reshape(-1)[:inner]
    return ((out >> np.uint32(8)).astype(np.float32) * np.float32(2.0 ** -24)).astype(np.float32)
