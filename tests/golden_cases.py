"""Inputs of the frozen oracle fixtures (tests/golden/dfxp_quant.npz, tests/golden/resnet20_b128.npz).

Test infrastructure. ``tools/gen_golden.py`` runs the oracle on these inputs once and commits the
outputs; ``tests/test_golden.py`` (CPU) re-runs the oracle and must reproduce them bit for bit, and
``tests/test_gpu_golden.py`` (MI355X) compares the HIP path with the committed files directly -- so a
change that moved the oracle and the kernels together would fail the first test.

Every input is regenerated from a seed (numpy PCG64 / the bench's torch CPU generator); the fixtures
hold the sha256 of each input so a generator drift is reported as such, not as a parity failure.
"""
import hashlib

import numpy as np

QUANT_SEED = 4321  # the noise key's seed (DfxpContext(seed=...) / oracle noise_for)

# (range-variable name, shape, bits, I, stochastic, output kind, lo, hi): one case per tensor class of the
# ResNet-20 step (dynamic_fixed_point.py:4-94 on each), activations at N = 8; the name keys the noise
# stream (qid = crc32(name)), the inputs are uniform on [lo, hi) -- ranges chosen so that every case
# overflows at one or both thresholds for some elements, or at neither, as the controller's three
# branches need (:83-94)
QUANT_CASES = [
    ("conv1/X_range", (8, 32, 32, 3), 9, 0, True, "i16", -1.0, 1.0),                 # the image (Conv2d_pq)
    ("block16-1/residual/conv1/X_range", (8, 32, 32, 16), 9, 2, True, "u8off", 0.0, 4.5),  # post-ReLU conv input
    ("block16-1/residual/bn1/norm/X_range", (8, 32, 32, 16), 8, 2, True, "i8", -5.0, 5.0),  # BN input
    ("block32-1/residual/bn2/norm/X_range", (8, 16, 16, 32), 8, 3, True, "i8", -12.0, 12.0),
    ("block64-2/residual/bn1/rescale/X_range", (8, 8, 8, 64), 8, 2, False, "i8", -5.0, 5.0),  # nearest (:26-30)
    ("block16-2/residual/conv2/grad_range", (8, 32, 32, 16), 8, -6, True, "i8", -0.03, 0.03),
    ("block64-3/residual/conv1/grad_range", (8, 8, 8, 64), 8, -3, True, "i8", -0.2, 0.2),
    ("block16-1/residual/conv1/W_range", (3, 3, 16, 16), 8, 0, True, "i8", -0.5, 0.5),
    ("block64-1/residual/conv2/W_range", (3, 3, 64, 64), 8, -1, False, "i8", -0.2, 0.2),
    ("softmax/W_range", (64, 10), 8, 1, True, "i8", -1.5, 1.5),
    ("block64-3/residual/bn2/rescale/g_range", (64,), 8, 2, True, "f32", -3.0, 3.0),
    ("softmax/grad_range", (128, 10), 8, -5, True, "i8", -0.01, 0.01),
    ("block32-2/residual/conv2/W_range", (3, 3, 32, 32), 4, 0, True, "i8", -1.2, 1.2),      # configs[4] W4
    ("block128-1/residual/conv2/grad_range", (8, 16, 16, 32), 16, -4, True, "i16", -0.1, 0.1),  # configs[3] 16-bit G
]


def quant_input(i):
    """Input of QUANT_CASES[i]."""
    name, shape, bits, I, stoch, kind, lo, hi = QUANT_CASES[i]
    rng = np.random.default_rng(1000 + i)
    return rng.uniform(lo, hi, size=shape).astype(np.float32)


def digest(a):
    """sha256 of an array's bytes in a canonical dtype (int64 for integers, float32 for floats)."""
    a = np.ascontiguousarray(a)
    if np.issubdtype(a.dtype, np.integer):
        a = a.astype(np.int64)
    else:
        a = a.astype(np.float32)
    return hashlib.sha256(a.tobytes()).hexdigest()


# ---- ResNet-20 step fixtures: bench.py's timed configuration (configs[1]): B = 128, the bench's four
# synthetic batches (bench.synthetic_batches(4, 128, 1000)), lr 1e-2, momentum 0.9, weight decay 2e-4,
# noise seed 0, the reference's default ranges (every *_range at I = 2); weights initialised as
# bench.py's cpu_baseline does (uniform +-sqrt(3 / fan_in), gamma 1, beta 0) from PARAM_SEED
STEP_B = 128
PARAM_SEED = 0
TRAJ_STEPS = 20
BENCH_GRAD_RANGE = -6  # bench.py --grad-range default: the timed configuration (resnet20_b128_gr6.npz)
B16 = 16  # one rank's images in configs[2]'s 8 x 16 partition of B = 128


def init_ranges(model, grad_range=None):
    """Initial exponents of an oracle model: every *_range at I = 2 (the reference's defaults,
    dynamic_fixed_point.py:225,321,541,628), the gradient quantisers at grad_range when given (the
    layers' grad_range argument, CIFAR10_Resnet20(..., grad_range=-6) on the build side)."""
    from oracle import resnet as R
    r = R.init_ranges(model)
    if grad_range is not None:
        r = {k: (grad_range if k.endswith("grad_range") else v) for k, v in r.items()}
    return r


def init_params(model):
    """{name: array} for an oracle model (the oracle's parameter names = the build's)."""
    rng = np.random.default_rng(PARAM_SEED)
    params = {}
    for name, owner in model.params():
        if name.endswith("/W"):
            shp = owner.ksize if hasattr(owner, "ksize") else (owner.in_units, owner.units)
            lim = np.sqrt(3 / float(np.prod(shp[:-1])))
            params[name] = rng.uniform(-lim, lim, size=shp).astype(np.float32)
        elif name.endswith("/g"):
            params[name] = np.ones(owner.C, np.float32)
        else:
            params[name] = np.zeros(owner.C, np.float32)
    return params


def bench_batches():
    """The bench's four B=128 batches as numpy arrays (torch CPU generator, as bench.py draws them)."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    xs, ys = bench.synthetic_batches(4, STEP_B, 1000, "cpu")
    return [x.numpy() for x in xs], [y.numpy() for y in ys]
