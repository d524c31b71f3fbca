"""The top of the reference's bit-width domain: ``weight_quantization`` asserts ``1 <= bits <= 32``
and returns the tensor itself at ``bits == 32`` (``dynamic_fixed_point.py:21-23``); ``main.py:113``
exposes it as ``--bits``. Quantisers of 17..31 bits write fake-quantised fp32 values (their integer
codes exceed the int8 / int16 GEMM operands) and the layers contract fp32 operands (``fp32.hip``),
as TF does on the fake-quantised tensors.

Tolerance: the quantiser outputs, overflow counters and exponent updates are integer work and
bit-exact. The contractions and BN moments accumulate in double in a fixed order on the GPU and in
numpy's (BLAS) order in the oracle; both round once to fp32, so results agree to within 1 ulp:
``rtol 2e-7`` on the layer outputs / gradients (``F32_RTOL`` below, ~1.7 ulp), and -- for a whole
network, where a 1-ulp difference can flip one stochastic floor of a downstream 20-bit quantiser
(one code step = 2**-(bits-I-1)) -- ``max|a-b| <= 1e-4 * max|b|``.
"""
import numpy as np
import pytest
import torch

from lbt_amd import dynamic_fixed_point as D
from lbt_amd.runtime import DfxpContext
from oracle import nn as onn
from oracle import resnet as oresnet

DEV = "cuda"
F32 = np.float32
F32_RTOL = 2e-7


def _close(a, b, rtol=F32_RTOL, what=""):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    err = np.abs(a - b) - rtol * np.abs(b)
    assert np.all(err <= 1e-30), "%s: worst %g (|b| %g)" % (what, err.max(), np.abs(b).max())


# ------------------------------------------------------------------------------ CPU
def test_bits_domain_matches_reference_assertion():
    """1..32 accepted, 0 and 33 rejected with the reference's own message (:21); 32 is the bypass."""
    ctx = DfxpContext(device="cpu", seed=0)
    for b in (1, 2, 8, 16, 17, 31, 32):
        ctx.quantizer("q%d/X_range" % b, b, 0 if b < 32 else 2)
    for b in (0, 33):
        with pytest.raises(ValueError, match="invalid value for bits"):
            ctx.quantizer("bad%d/X_range" % b, b, 0)
    octx = onn.Ctx({"w/W_range": 3}, 0, 0)
    x = np.array([1.5, -7.25, 1e-9], F32)
    assert np.array_equal(octx.fq("w/W_range", x, 32), x)  # the tensor itself
    with pytest.raises(AssertionError, match="invalid value for bits: 33"):
        octx.fq("w/W_range", x, 33)


def test_oracle_wide_quantiser_known_answer():
    """A 20-bit quantiser at I = 3 rounds to multiples of 2**-16 (nearest, half to even) and
    overflows at +-2**3: pinned by hand."""
    octx = onn.Ctx({"w/W_range": 3}, 0, 0)
    x = np.array([1 + 2 ** -17, 1 + 3 * 2 ** -17, -2.0 ** -18, 9.0, -8.0, -8.5], F32)
    y = octx.fq("w/W_range", x, 20, stochastic=False)
    assert list(y) == [1.0, 1 + 2 * 2 ** -16, 0.0, 8 - 2 ** -16, -8.0, -8.0]
    c1, c2, n, _ = octx.counts["w/W_range"]
    assert (c1, c2, n) == (2, 3, 6)  # >= 2**19 codes: 9, -8.5 (-8 is in range); >= 2**18: also -8


# ------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("bits,N,H,Cin,Cout,k,s,bias", [(20, 4, 12, 8, 16, 3, 1, False),
                                                         (31, 3, 9, 5, 12, 3, 2, True),
                                                         (17, 2, 8, 16, 16, 1, 2, False)])
def test_conv_wide_bits_matches_oracle(bits, N, H, Cin, Cout, k, s, bias):
    """Conv2d_q at 17..31 bits (X at bits + 1; 31 -> a 32-bit X quantiser, the bypass): the fake-
    quantised operands bit-exact, y / dW / db / dX within 1 ulp, exponents identical."""
    rng = np.random.default_rng(bits + N + H)
    ctx = DfxpContext(seed=31)
    gl = D.Conv2d_q("c", bits, [k, k, Cin, Cout], [1, s, s, 1], "SAME", use_bias=bias, weight_decay=2e-4, ctx=ctx)
    ol = onn.Conv2dQ("c", bits, [k, k, Cin, Cout], [1, s, s, 1], "SAME", 2e-4, use_bias=bias)
    ol.W = gl.W.cpu().numpy().copy()
    if bias:
        b = (0.1 * rng.standard_normal(Cout)).astype(F32)
        gl.b.copy_(torch.from_numpy(b))
        ol.b = b.copy()
    assert gl.fmode and ol.fmode
    x = rng.uniform(-1.5, 1.5, size=(N, H, H, Cin)).astype(F32)
    octx = onn.Ctx(ctx.ranges(), 0, 31)
    y = gl.forward(torch.from_numpy(x).to(DEV))
    yr = ol.forward(x, octx)
    assert np.array_equal(gl.xq.cpu().numpy(), ol.xf)
    assert np.array_equal(gl.wq.cpu().numpy(), ol.wf)
    _close(y.cpu().numpy(), yr, what="y")
    g = rng.normal(0, 0.05, size=yr.shape).astype(F32)
    dx = gl.backward(torch.from_numpy(g).to(DEV))
    dxr = ol.backward(g, octx)
    _close(gl.dW.cpu().numpy(), ol.dW, what="dW")
    if bias:
        _close(gl.db.cpu().numpy(), ol.db, what="db")
    _close(dx.cpu().numpy(), dxr, what="dX")
    ctx.update_range_op()
    assert ctx.ranges() == octx.new_ranges()


@pytest.mark.gpu
def test_conv_bits32_asserts_like_reference():
    """Conv2d_q(bits=32) quantises X at 33 bits, which the reference's assertion rejects (:21, :287)."""
    ctx = DfxpContext(seed=1)
    gl = D.Conv2d_q("c", 32, [3, 3, 4, 8], [1, 1, 1, 1], "SAME", ctx=ctx)
    with pytest.raises(AssertionError, match="invalid value for bits: 33"):
        gl.forward(torch.zeros((1, 4, 4, 4), device=DEV))


@pytest.mark.gpu
@pytest.mark.parametrize("bits,bias", [(32, False), (24, True)])
def test_dense_wide_bits_matches_oracle(bits, bias):
    rng = np.random.default_rng(bits)
    ctx = DfxpContext(seed=3)
    gl = D.Dense_q("fc", bits, 64, 10, use_bias=bias, weight_decay=2e-4, ctx=ctx)
    ol = onn.DenseQ("fc", bits, 64, 10, 2e-4, use_bias=bias)
    ol.W = gl.W.cpu().numpy().copy()
    x = rng.uniform(-2, 2, size=(33, 64)).astype(F32)
    octx = onn.Ctx(ctx.ranges(), 0, 3)
    y = gl.forward(torch.from_numpy(x).to(DEV))
    _close(y.cpu().numpy(), ol.forward(x, octx), what="y")
    g = rng.normal(0, 0.01, size=(33, 10)).astype(F32)
    dx = gl.backward(torch.from_numpy(g).to(DEV))
    dxr = ol.backward(g, octx)
    _close(gl.dW.cpu().numpy(), ol.dW, what="dW")
    _close(dx.cpu().numpy(), dxr, what="dX")
    if bias:
        _close(gl.db.cpu().numpy(), ol.db, what="db")
    ranges = dict(ctx.ranges())
    ctx.update_range_op()
    assert ctx.ranges() == octx.new_ranges()
    if bits == 32:  # the bypass registers no update_range op: nothing moves
        assert ctx.ranges() == ranges


@pytest.mark.gpu
@pytest.mark.parametrize("bits,shape", [(32, (8, 6, 6, 16)), (20, (16, 8, 8, 32))])
def test_batchnorm_wide_bits_matches_oracle(bits, shape):
    """BatchNorm_q (Normalization_q + Rescale_q) at 20 / 32 bits: training-mode forward and backward,
    dgamma / dbeta and the running averages within 1 ulp; then a testing-mode step."""
    rng = np.random.default_rng(bits + shape[0])
    C = shape[-1]
    ctx = DfxpContext(seed=12)
    gbn = D.BatchNorm_q("bn", bits, C, weight_decay=2e-4, ctx=ctx)
    obn = onn.BatchNormQ("bn", bits, C, 2e-4)
    gam = (1 + 0.2 * rng.standard_normal(C)).astype(F32)
    bet = (0.2 * rng.standard_normal(C)).astype(F32)
    gbn.layers[1].gamma.copy_(torch.from_numpy(gam))
    gbn.layers[1].beta.copy_(torch.from_numpy(bet))
    obn.layers[1].gamma, obn.layers[1].beta = gam.copy(), bet.copy()
    for step in range(2):
        testing = step == 1
        gbn.layers[0].train = obn.layers[0].train = not testing
        x = (rng.standard_normal(shape) * 1.3 + 0.4).astype(F32)
        octx = onn.Ctx(ctx.ranges(), step, 12)
        y = gbn.forward(torch.from_numpy(x).to(DEV))
        _close(y.cpu().numpy(), obn.forward(x, octx), rtol=1e-6, what="y")
        g = (rng.standard_normal(shape) * 0.03).astype(F32)
        dx = gbn.backward(torch.from_numpy(g).to(DEV))
        dxr = obn.backward(g, octx)
        _close(gbn.layers[1].dgamma.cpu().numpy(), obn.layers[1].dgamma, rtol=1e-6, what="dgamma")
        _close(gbn.layers[1].dbeta.cpu().numpy(), obn.layers[1].dbeta, what="dbeta")
        _close(dx.cpu().numpy(), dxr, rtol=1e-5, what="dX")
        _close(gbn.layers[0].X_mean_running.cpu().numpy(), obn.layers[0].mean_running, what="mean_running")
        _close(gbn.layers[0].X_var_running.cpu().numpy(), obn.layers[0].var_running, what="var_running")
        ctx.update_range_op()
        assert ctx.ranges() == octx.new_ranges()


@pytest.mark.gpu
def test_resnet20_20bit_step_matches_oracle():
    """CIFAR10_Resnet20(bits=20): the whole layer-wise network in float mode (every quantiser 20 / 21
    bits) -- logits, loss, every gradient and the exponent updates against the oracle."""
    from lbt_amd.models import CIFAR10_Resnet20
    ctx = DfxpContext(seed=4)
    gm = CIFAR10_Resnet20(20, weight_decay=2e-4, ctx=ctx)
    om = oresnet.build_resnet((3, 3, 3), 20, 2e-4)
    params = {o.name + {"W": "/W", "gamma": "/g", "beta": "/b"}[v]: getattr(o, v).cpu().numpy().copy()
              for o, v, _ in gm.param_slots()}
    oresnet.set_params(om, params)
    rng = np.random.default_rng(4)
    x = ((rng.integers(0, 256, size=(8, 32, 32, 3)) - 127.5) / 128).astype(F32)
    y = rng.integers(0, 10, size=8).astype(np.int32)
    logits = gm.forward(torch.from_numpy(x).to(DEV))
    loss = gm.compute_loss(torch.from_numpy(y).to(DEV))
    gm.backward()
    torch.cuda.synchronize()
    lref, _, grads, octx = oresnet.forward_backward(om, oresnet.init_ranges(om), x, y, 0, 4)
    zl = logits.cpu().numpy()
    assert np.abs(zl - octx.logits).max() <= 1e-4 * np.abs(octx.logits).max()
    assert abs(loss.item() - lref) <= 1e-5 * abs(lref)
    for o, v, gname in gm.param_slots():
        k = o.name + {"W": "/W", "gamma": "/g", "beta": "/b"}[v]
        a, b = getattr(o, gname).cpu().numpy(), grads[k]
        assert np.abs(a - b).max() <= 1e-4 * np.abs(b).max() + 1e-12, k
    ctx.update_range_op()
    assert ctx.ranges() == octx.new_ranges()


@pytest.mark.gpu
@pytest.mark.parametrize("kind,shape", [("conv", (4, 8, 8, 16, 32, 3, 1)), ("conv", (2, 8, 8, 64, 64, 1, 2)),
                                        ("dense", (33, 64, 10, 0, 0, 0, 0))])
def test_bias_with_16bit_gradients_matches_oracle(kind, shape):
    """Conv2d_q / Dense_q with use_bias=True and 16-bit gradient codes (config 4 with the
    batch_norm=False blocks of ResidualBlock_q, dynamic_fixed_point.py:778): db = the quantised
    gradient summed per channel (:303-304, :457) from the quantiser's exact channel sums; dW, db and
    dX bit-exact against the oracle, exponents identical."""
    rng = np.random.default_rng(sum(shape))
    ctx = DfxpContext(seed=17)
    if kind == "conv":
        N, H, Cin, Cout, k, s = shape[0], shape[1], shape[3], shape[4], shape[5], shape[6]
        gl = D.Conv2d_q("c", 8, [k, k, Cin, Cout], [1, s, s, 1], "SAME", use_bias=True, weight_decay=2e-4,
                        grad_bits=16, ctx=ctx)
        ol = onn.Conv2dQ("c", 8, [k, k, Cin, Cout], [1, s, s, 1], "SAME", 2e-4, grad_bits=16, use_bias=True)
        x = rng.uniform(-1.5, 1.5, size=(N, H, H, Cin)).astype(F32)
    else:
        N, Cin, Cout = shape[0], shape[1], shape[2]
        gl = D.Dense_q("fc", 8, Cin, Cout, use_bias=True, weight_decay=2e-4, grad_bits=16, ctx=ctx)
        ol = onn.DenseQ("fc", 8, Cin, Cout, 2e-4, use_bias=True, grad_bits=16)
        x = rng.uniform(-2, 2, size=(N, Cin)).astype(F32)
    ol.W = gl.W.cpu().numpy().copy()
    b = (0.1 * rng.standard_normal(Cout)).astype(F32)
    gl.b.copy_(torch.from_numpy(b))
    ol.b = b.copy()
    octx = onn.Ctx(ctx.ranges(), 0, 17)
    y = gl.forward(torch.from_numpy(x).to(DEV))
    yr = ol.forward(x, octx)
    assert np.array_equal(y.cpu().numpy(), yr)
    g = rng.normal(0, 0.01, size=yr.shape).astype(F32)
    dx = gl.backward(torch.from_numpy(g).to(DEV))
    dxr = ol.backward(g, octx)
    assert np.array_equal(gl.dW.cpu().numpy(), ol.dW)
    assert np.array_equal(gl.db.cpu().numpy(), ol.db)
    assert np.array_equal(dx.cpu().numpy(), dxr)
    ctx.update_range_op()
    assert ctx.ranges() == octx.new_ranges()
