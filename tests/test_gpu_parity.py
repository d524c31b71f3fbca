"""GPU parity: the HIP path (through the C-ABI) against the numpy oracle on the same seeded inputs.

Integer work (quantiser codes, overflow counters, exponent updates, every integer GEMM and the
dequantised fp32 results built from them, BN moments and backward sums) is required to be
BIT-EXACT. The only op that is not bit-exact is the softmax (expf/logf): loss and d loss / d
logits are compared with rtol 1e-5; the model backward is then checked bit-exact by feeding
the GPU's d loss / d logits into the oracle backward.
"""
import types

import numpy as np
import pytest
import torch

from lbt_amd import dynamic_fixed_point as D
from lbt_amd._lib import NSHARD, OUT_F32, OUT_I8, OUT_I16, OUT_U8OFF
from lbt_amd.dfxp import ops
from lbt_amd.runtime import DfxpContext, qid_of
from oracle import dfxp as odfxp
from oracle import nn as onn
from oracle import resnet as oresnet

pytestmark = pytest.mark.gpu
DEV = "cuda"


def decode(t, kind):
    a = t.cpu().numpy()
    if kind == OUT_U8OFF:
        return a.astype(np.int32) + 128
    return a.astype(np.int32) if kind != OUT_F32 else a


@pytest.mark.parametrize("shape,bits,I,stoch,kind,lo,hi", [
    ((128, 32, 32, 16), 9, 2, True, OUT_U8OFF, 0.0, 4.5),
    ((128, 32, 32, 16), 8, 2, True, OUT_I8, -5.0, 5.0),
    ((16, 16, 16, 32), 8, -3, True, OUT_I8, -0.2, 0.2),
    ((16, 8, 8, 64), 8, 2, False, OUT_I8, -5.0, 5.0),
    ((8, 32, 32, 3), 9, 0, True, OUT_I16, -1.0, 1.0),
    ((3, 7, 5), 8, 1, True, OUT_I8, -3.0, 3.0),
    ((64,), 8, 2, True, OUT_I8, -3.0, 3.0),
    ((128, 10), 8, -5, True, OUT_I8, -0.01, 0.01),
    ((4, 6, 6, 8), 4, 1, True, OUT_I8, -2.0, 2.0),
    ((4, 6, 6, 8), 12, 2, True, OUT_I16, -5.0, 5.0),
])
def test_quantize_codes_and_counts(shape, bits, I, stoch, kind, lo, hi):
    rng = np.random.default_rng(abs(hash((shape, bits, I))) % 2**32)
    x = rng.uniform(lo, hi, size=shape).astype(np.float32)
    ctx = DfxpContext(seed=1234)
    q = ctx.quantizer("t/X_range", bits, I, stochastic=stoch)
    out = ops.quantize(torch.from_numpy(x).to(DEV), q, kind)
    noise = odfxp.noise_for(shape, qid_of("t/X_range"), 0, 1234) if stoch else None
    ref = odfxp.quantize_int(x, bits, I, stoch, noise)
    got = decode(out, kind)
    if kind == OUT_F32:
        assert np.array_equal(got, odfxp.dequant(ref, odfxp.frac_bits(bits, I)))
    else:
        assert np.array_equal(got, ref)
    c = ctx.counts_view()[0].sum(0).cpu().tolist()
    assert tuple(c) == odfxp.overflow_counts(x, bits, I)


def test_quantize_channel_sums_and_range_update():
    rng = np.random.default_rng(3)
    x = rng.normal(0, 1.5, size=(32, 8, 8, 16)).astype(np.float32)
    ctx = DfxpContext(seed=9)
    q = ctx.quantizer("a/X_range", 8, 2)
    q2 = ctx.quantizer("b/X_range", 8, 2)   # fed nothing: must keep its exponent
    chsum = ops.new_sums(16, 2, DEV)
    codes = ops.quantize(torch.from_numpy(x).to(DEV), q, OUT_I8, chsum=chsum, C=16)
    ref = odfxp.quantize_int(x, 8, 2, True, odfxp.noise_for(x.shape, qid_of("a/X_range"), 0, 9))
    assert np.array_equal(codes.cpu().numpy(), ref)
    s = chsum.view(NSHARD, 32).sum(0).cpu().numpy()
    r = ref.reshape(-1, 16).astype(np.int64)
    assert np.array_equal(s[:16], r.sum(0)) and np.array_equal(s[16:], (r * r).sum(0))
    ctx.update_range_op()
    assert ctx.ranges() == {"a/X_range": odfxp.update_range(x, 0.0, 8, 2), "b/X_range": 2}
    assert int(ctx.step.item()) == 1
    assert int(ctx.counts.abs().sum().item()) == 0


@pytest.mark.parametrize("C", [4, 8, 12, 32, 64, 128, 256])
def test_quantize_channel_sums_every_lane_period(C):
    """Per-channel sums of the quantiser (quantize.hip: reduce-scatter over the wave's rows for a
    channel-quad period of 1..16 lanes, butterfly / per-lane atomics otherwise) on a ragged shape
    (inner = 21 C: the last wave of a row has dead lanes)."""
    rng = np.random.default_rng(C)
    x = rng.normal(0, 1.5, size=(5, 3, 7, C)).astype(np.float32)
    ctx = DfxpContext(seed=4)
    q = ctx.quantizer("p/X_range", 8, 2)
    chsum = ops.new_sums(C, 2, DEV)
    codes = ops.quantize(torch.from_numpy(x).to(DEV), q, OUT_I8, chsum=chsum, C=C)
    ref = odfxp.quantize_int(x, 8, 2, True, odfxp.noise_for(x.shape, qid_of("p/X_range"), 0, 4))
    assert np.array_equal(codes.cpu().numpy(), ref)
    s = chsum.view(NSHARD, 2 * C).sum(0).cpu().numpy()
    r = ref.reshape(-1, C).astype(np.int64)
    assert np.array_equal(s[:C], r.sum(0)) and np.array_equal(s[C:], (r * r).sum(0))


def test_counts_fold_and_folded_range_update():
    """The data-parallel controller path (fold -> [all-reduce] -> folded update) equals the
    sharded one; large counters survive the fp32 fold exactly."""
    from lbt_amd import distributed as Dd
    rng = np.random.default_rng(31)
    xs = [rng.normal(0, s, size=(64, 16, 16, 16)).astype(np.float32) for s in (0.5, 3.0, 40.0)]
    ref_ranges, folded_all = [], []
    for mode in ("sharded", "folded"):
        ctx = DfxpContext(seed=5)
        qs = [ctx.quantizer("s%d/X_range" % i, 8, 2) for i in range(3)]
        for x, q in zip(xs, qs):
            ops.quantize(torch.from_numpy(x).to(DEV), q, OUT_I8)
        if mode == "sharded":
            ctx.update_range_op()
            ref_ranges = ctx.ranges()
        else:
            folded = torch.full((4 * 3,), -1.0, device=DEV)
            ctx.fold_counts(folded)
            assert int(ctx.counts.abs().sum().item()) == 0
            got = Dd.unfold_host(folded.cpu()).tolist()
            assert got == [list(odfxp.overflow_counts(x, 8, 2)) for x in xs]
            ctx.update_range_folded_op(folded)
            assert ctx.ranges() == ref_ranges
            assert int(ctx.step.item()) == 1
    big = torch.tensor([[2 ** 30 + 777, 5]], dtype=torch.int64)
    f = Dd.fold_host(big).to(DEV)
    ctx = DfxpContext(seed=5)
    ctx.quantizer("big/X_range", 8, 2)
    ctx.nelem[0] = 2.0 ** 31
    ctx.update_range_folded_op(f)
    # r1 = (2^30+777)/2^31 > 0 -> I + 1
    assert ctx.ranges() == {"big/X_range": 3}


def test_division_by_reused_divisor_is_bitexact():
    """The BN kernels divide by sigma with the divisor-only part of the division hoisted
    (div_by / recip); it must equal '/' in every bit over the ranges the BN moments take."""
    from lbt_amd import _lib
    g = torch.Generator(device=DEV).manual_seed(0)
    n = 1 << 24
    y = torch.exp2(torch.empty(n, device=DEV).uniform_(-8, 12, generator=g))     # sigma = sqrt(var + eps)
    y = torch.where(torch.arange(n, device=DEV) % 7 == 0, y.view(torch.int32).bitwise_or(0x7FFFFF).view(torch.float32), y)
    x = torch.empty(n, device=DEV).uniform_(-1, 1, generator=g) * torch.exp2(torch.empty(n, device=DEV).uniform_(-40, 12,
                                                                                                          generator=g))
    x[::11] = 0.0
    x[3::17] = -0.0
    x[5::13] = torch.round(x[5::13] * 256) / 256                               # code-valued numerators (and -0)
    bad = torch.zeros(1, dtype=torch.int32, device=DEV)
    _lib.call("lbt_selftest_div", _lib.ptr(x), _lib.ptr(y), n, _lib.ptr(bad), None, None, _lib.stream())
    assert int(bad.item()) == 0


def test_tf_face_functions():
    rng = np.random.default_rng(4)
    x = rng.normal(0, 2, size=(16, 5, 5, 4)).astype(np.float32)
    ctx = DfxpContext(seed=2)
    q = ctx.quantizer("f/X_range", 8, 2)
    xt = torch.from_numpy(x).to(DEV)
    fq = D.weight_quantization(xt, 0, 8, q, stochastic=False).cpu().numpy()
    assert np.array_equal(fq, odfxp.dequant(odfxp.quantize_int(x, 8, 2, False), 5))
    r1, r2 = D.overflow_rate(xt, 8, q)
    e1, e2 = odfxp.overflow_rate(x, 8, 2)
    assert (r1, r2) == (float(e1), float(e2))
    D.update_range(xt, 0, 8, q)
    assert q.integer_bits == odfxp.update_range(x, 0.0, 8, 2)


def test_weight_packing():
    rng = np.random.default_rng(5)
    KH, KW, Cin, Cout = 3, 3, 32, 64
    w = rng.uniform(-0.1, 0.1, size=(KH, KW, Cin, Cout)).astype(np.float32)
    ctx = DfxpContext(seed=3)
    q = ctx.quantizer("c/W_range", 8, 2)
    ksf, ksd = ops.packed_slices(KH, KW, Cin), ops.packed_slices(KH, KW, Cout)
    hwio = torch.zeros((KH, KW, Cin, Cout), dtype=torch.int8, device=DEV)
    wf = torch.zeros((Cout, ksf * 16), dtype=torch.int8, device=DEV)
    wd = torch.zeros((Cin, ksd * 16), dtype=torch.int8, device=DEV)
    cs = torch.zeros(Cout, dtype=torch.int32, device=DEV)
    ops.quantize_weight(torch.from_numpy(w).to(DEV), q, hwio, wf, ksf, wd, ksd, cs)
    ref = odfxp.quantize_int(w, 8, 2, True, odfxp.noise_for(w.shape, qid_of("c/W_range"), 0, 3))
    assert np.array_equal(hwio.cpu().numpy(), ref)
    K = KH * KW * Cin
    assert np.array_equal(wf.cpu().numpy()[:, :K], ref.reshape(K, Cout).T)
    assert np.array_equal(wd.cpu().numpy()[:, :KH * KW * Cout],
                          ref.transpose(2, 0, 1, 3).reshape(Cin, KH * KW * Cout))
    assert np.array_equal(cs.cpu().numpy(), ref.reshape(K, Cout).sum(0))


def _copy_conv(gl, ol):
    ol.W = gl.W.cpu().numpy().copy()


# (N, H, Cin, Cout, k, s, nonneg)
CONV_CASES = [
    (8, 32, 16, 16, 3, 1, True),     # stage-1 block conv (MFMA, offset uint8)
    (8, 32, 16, 32, 3, 2, True),     # downsample conv, TF SAME (0,1) padding
    (8, 32, 16, 32, 1, 2, True),     # 1x1 stride-2 shortcut
    (8, 16, 32, 32, 3, 1, True),
    (8, 16, 32, 64, 3, 2, True),
    (8, 8, 64, 64, 3, 1, True),      # stage-3 block conv
    (8, 32, 3, 16, 3, 1, False),     # conv1: signed 9-bit image, fp16-MFMA stem path
    (128, 32, 3, 16, 3, 1, False),   # conv1 at the bench size
    (5, 7, 3, 32, 3, 2, False),      # stem: odd size, stride 2, two column tiles
    (3, 6, 2, 64, 3, 1, False),      # stem: K = 18, Cout = 64
    (4, 12, 16, 16, 3, 1, False),    # signed 9-bit input on a 16-channel conv -> VALU path
    (4, 9, 32, 16, 3, 2, True),      # odd spatial size
    (128, 32, 16, 16, 3, 1, True),   # full ResNet-20 stage-1 size (B=128)
]


@pytest.mark.parametrize("N,H,Cin,Cout,k,s,nonneg", CONV_CASES)
def test_conv_layer_bitexact(N, H, Cin, Cout, k, s, nonneg):
    rng = np.random.default_rng(N * 1000 + H * 10 + Cin + Cout + k + s)
    ctx = DfxpContext(seed=77)
    name = "blk"
    gl = D.Conv2d_q(name, 8, [k, k, Cin, Cout], [1, s, s, 1], "SAME", use_bias=False, weight_decay=2e-4,
                    input_nonnegative=nonneg, ctx=ctx)
    ol = onn.Conv2dQ(name, 8, [k, k, Cin, Cout], [1, s, s, 1], "SAME", 2e-4)
    _copy_conv(gl, ol)
    x = (rng.uniform(0, 3.5, size=(N, H, H, Cin)) if nonneg else rng.uniform(-1, 1, size=(N, H, H, Cin)))
    x = x.astype(np.float32)
    octx = onn.Ctx({r: 2 for r in ol.range_names()}, 0, 77)
    y = gl.forward(torch.from_numpy(x).to(DEV))
    yr = ol.forward(x, octx)
    assert np.array_equal(y.cpu().numpy(), yr)
    g = rng.normal(0, 0.05, size=yr.shape).astype(np.float32)
    dx = gl.backward(torch.from_numpy(g).to(DEV))
    dxr = ol.backward(g, octx)
    assert np.array_equal(gl.gradq.cpu().numpy(), octx.record[name + "/grad_range"])
    assert np.array_equal(gl.dW.cpu().numpy(), ol.dW)
    assert np.array_equal(dx.cpu().numpy(), dxr)
    ctx.update_range_op()
    assert ctx.ranges() == octx.new_ranges()


@pytest.mark.parametrize("N,H,Cin,Cout,s", [(8, 32, 3, 16, 1), (5, 9, 3, 32, 2), (2, 5, 1, 16, 1),
                                             (4, 8, 3, 64, 1), (4, 8, 3, 128, 1)])
def test_stem_kernels_equal_integer_gemm(N, H, Cin, Cout, s):
    """fp16-MFMA stem fwd / wgrad at the extreme codes of its contract (|x| <= 2048, int8 w / g)
    equal the exact integer convolution (int64 numpy) and the generic VALU kernels."""
    rng = np.random.default_rng(N + H + Cin + Cout)
    x = rng.integers(-2048, 2048, size=(N, H, H, Cin)).astype(np.int16)
    x.flat[:7] = -2048
    w = rng.integers(-128, 128, size=(3, 3, Cin, Cout)).astype(np.int8)
    w.flat[:5] = -128
    d = ops.conv_desc(N, H, H, Cin, Cout, 3, 3, s, s, "SAME")
    ctx = DfxpContext(seed=1)
    qx = ctx.quantizer("x/X_range", 12, 2)
    qw = ctx.quantizer("x/W_range", 8, 1)
    xt, wt = torch.from_numpy(x).to(DEV), torch.from_numpy(w).to(DEV)
    y_ref = onn.scale_int(onn.conv_fwd_int(x, w, (s, s), "SAME"), (12 - 2 - 1) + (8 - 1 - 1))
    y = torch.empty((N, d.Ho, d.Wo, Cout), dtype=torch.float32, device=DEV)
    ops.conv_stem_fwd(xt, wt, d, qx.desc, qw.desc, y=y)
    assert np.array_equal(y.cpu().numpy(), y_ref)
    if Cout <= 64:
        y2 = torch.empty_like(y)
        ops.conv_fwd_generic(xt, 1, wt, d, qx.desc, qw.desc, y2)
        assert torch.equal(y, y2)
        g = rng.integers(-128, 128, size=(N, d.Ho, d.Wo, Cout)).astype(np.int8)
        g.flat[:3] = -128
        ns = ops.stem_nsplit(d)
        slab = torch.zeros((ns, 9 * Cin, Cout), dtype=torch.int32, device=DEV)
        ops.conv_stem_wgrad(xt, torch.from_numpy(g).to(DEV), d, slab, ns)
        dw_ref = onn.conv_wgrad_int(x, g, (s, s), "SAME", (3, 3))
        assert np.array_equal(slab.cpu().numpy().astype(np.int64).sum(0), dw_ref.reshape(9 * Cin, Cout))


def test_dense_layer_bitexact():
    rng = np.random.default_rng(11)
    ctx = DfxpContext(seed=5)
    gl = D.Dense_q("softmax", 8, 64, 10, use_bias=False, weight_decay=2e-4, ctx=ctx)
    ol = onn.DenseQ("softmax", 8, 64, 10, 2e-4)
    ol.W = gl.W.cpu().numpy().copy()
    x = rng.uniform(0, 2, size=(128, 64)).astype(np.float32)
    octx = onn.Ctx({r: 2 for r in ol.range_names()}, 0, 5)
    y = gl.forward(torch.from_numpy(x).to(DEV))
    assert np.array_equal(y.cpu().numpy(), ol.forward(x, octx))
    g = rng.normal(0, 0.004, size=(128, 10)).astype(np.float32)
    dx = gl.backward(torch.from_numpy(g).to(DEV))
    dxr = ol.backward(g, octx)
    assert np.array_equal(gl.dW.cpu().numpy(), ol.dW)
    assert np.array_equal(dx.cpu().numpy(), dxr)


# channel counts 4 / 8 / 16 / 32 / 64 put 1 / 2 / 4 / 8 / 16 lanes between repeats of a channel quad
# (every DPP step of chan_scatter4); 128 and 12 take the butterfly fallback; the small ragged shapes
# leave workgroups with dead lanes
@pytest.mark.parametrize("shape", [(16, 32, 32, 16), (16, 8, 8, 64), (128, 16, 16, 32), (6, 5, 7, 4), (6, 5, 3, 8),
                                   (4, 6, 6, 128), (3, 5, 5, 12)])
def test_batchnorm_bitexact(shape):
    rng = np.random.default_rng(shape[0] + shape[-1])
    C = shape[-1]
    ctx = DfxpContext(seed=21)
    gbn = D.BatchNorm_q("bn", 8, C, weight_decay=2e-4, ctx=ctx)
    obn = onn.BatchNormQ("bn", 8, C, 2e-4)
    gam = (1 + 0.2 * rng.standard_normal(C)).astype(np.float32)
    bet = (0.2 * rng.standard_normal(C)).astype(np.float32)
    gbn.layers[1].gamma.copy_(torch.from_numpy(gam))
    gbn.layers[1].beta.copy_(torch.from_numpy(bet))
    obn.layers[1].gamma, obn.layers[1].beta = gam.copy(), bet.copy()
    x = (rng.standard_normal(shape) * 1.3 + 0.4).astype(np.float32)
    octx = onn.Ctx({r: 2 for r in obn.range_names()}, 0, 21)
    y = gbn.forward(torch.from_numpy(x).to(DEV))
    yr = obn.forward(x, octx)
    assert np.array_equal(y.cpu().numpy(), yr)
    g = (rng.standard_normal(shape) * 0.03).astype(np.float32)
    dx = gbn.backward(torch.from_numpy(g).to(DEV))
    dxr = obn.backward(g, octx)
    assert np.array_equal(gbn.layers[1].dgamma.cpu().numpy(), obn.layers[1].dgamma)
    assert np.array_equal(gbn.layers[1].dbeta.cpu().numpy(), obn.layers[1].dbeta)
    assert np.array_equal(dx.cpu().numpy(), dxr)
    ctx.update_range_op()
    assert ctx.ranges() == octx.new_ranges()


def _build_pair(batch_seed=0, wd=2e-4, seed=0, weight_bits=None):
    from lbt_amd.models import CIFAR10_Resnet20
    ctx = DfxpContext(seed=seed)
    gm = CIFAR10_Resnet20(8, weight_decay=wd, ctx=ctx, weight_bits=weight_bits)
    om = oresnet.build_resnet((3, 3, 3), 8, wd, weight_bits=weight_bits)
    return ctx, gm, om


def gpu_params(gm):
    out = {}
    for owner, var, _ in gm.param_slots():
        suffix = {"W": "/W", "gamma": "/g", "beta": "/b"}[var]
        out[owner.name + suffix] = getattr(owner, var).detach().cpu().numpy().copy()
    return out


def gpu_grads(gm):
    out = {}
    for owner, var, gname in gm.param_slots():
        suffix = {"W": "/W", "gamma": "/g", "beta": "/b"}[var]
        out[owner.name + suffix] = getattr(owner, gname).detach().cpu().numpy().copy()
    return out


def synthetic_batch(B, seed=0):
    rng = np.random.default_rng(seed)
    x = ((rng.integers(0, 256, size=(B, 32, 32, 3)) - 127.5) / 128).astype(np.float32)
    y = rng.integers(0, 10, size=B).astype(np.int32)
    return x, y


def test_resnet20_step_parity():
    ctx, gm, om = _build_pair()
    params = gpu_params(gm)
    oresnet.set_params(om, params)
    x, y = synthetic_batch(16, seed=1)
    xt, yt = torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV)
    octx = onn.Ctx(oresnet.init_ranges(om), 0, 0)
    logits = gm.forward(xt)
    lr = om.forward(x, octx)
    assert np.array_equal(logits.cpu().numpy(), lr), "forward must be bit-exact"
    loss = gm.compute_loss(yt)
    lref, dzr = onn.softmax_xent(lr, y)
    assert abs(loss.item() - lref) <= 1e-5 * abs(lref)
    dz = gm.dlogits.cpu().numpy()
    np.testing.assert_allclose(dz, dzr, rtol=1e-5, atol=1e-9)
    gm.backward()
    om.backward(dz, octx)   # same d loss / d logits -> the whole backward must be bit-exact
    gg, og = gpu_grads(gm), oresnet.get_grads(om)
    assert gg.keys() == og.keys()
    for k in gg:
        assert np.array_equal(gg[k], og[k]), k
    ctx.update_range_op()
    assert ctx.ranges() == octx.new_ranges()


def test_trainer_graph_replay_equals_eager():
    from lbt_amd.trainer import Trainer
    x, y = synthetic_batch(32, seed=2)
    xt, yt = torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV)
    res = []
    for use_graph in (False, True):
        ctx, gm, _ = _build_pair(seed=3)
        tr = Trainer(gm, lr=1e-2, momentum=0.9, batch_size=32, use_graph=use_graph)
        tr.init_model()
        losses = [tr.step(xt, yt).item() for _ in range(4)]
        torch.cuda.synchronize()
        res.append((losses, tr.flat.w.cpu().numpy(), ctx.ranges(), int(ctx.step.item())))
    (l0, w0, r0, s0), (l1, w1, r1, s1) = res
    assert l0 == l1 and r0 == r1 and s0 == s1 == 4
    assert np.array_equal(w0, w1)


def test_resnet20_trains_against_oracle_two_steps():
    """Two full optimiser steps of the layer-wise model: with the GPU's d loss / d logits injected
    into the oracle (the softmax's expf / logf is the one op that is not bit-exact) the weights,
    the momentum accumulators and the exponents after every step are BIT-IDENTICAL; the loss
    agrees to 1e-5."""
    from lbt_amd.trainer import Trainer
    ctx, gm, om = _build_pair(seed=4)
    state = dict(params=gpu_params(gm), accum=None, ranges=oresnet.init_ranges(om), step=0)
    state["accum"] = {k: np.zeros_like(v) for k, v in state["params"].items()}
    tr = Trainer(gm, lr=1e-2, momentum=0.9, batch_size=16, use_graph=False)
    for i in range(2):
        x, y = synthetic_batch(16, seed=10 + i)
        loss = tr.step(torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV)).item()
        dz = gm.dlogits.cpu().numpy()
        lref, state, octx = oresnet.train_step(om, state, x, y, lr=1e-2, momentum=0.9, seed=4, dz=dz)
        assert abs(loss - lref) <= 1e-5 * abs(lref), (i, loss, lref)
        np.testing.assert_allclose(dz, octx.dz, rtol=1e-5, atol=1e-9)
        gp = gpu_params(gm)
        for k in gp:
            assert np.array_equal(gp[k], state["params"][k]), (i, k)
        assert ctx.ranges() == state["ranges"], i


def _oracle_norms(om):
    return [l for l in oresnet._walk(om) if isinstance(l, onn.NormQ)]


def _gpu_norms(gm):
    from lbt_amd.dfxp.layers import Normalization_q
    return [l for l in gm._walk() if isinstance(l, Normalization_q)]


@pytest.mark.parametrize("weight_bits,B", [(None, 128), (4, 128), (None, 16), (None, 32), (None, 64), (4, 16)])
def test_fused_bench_workload_bitexact_vs_oracle(weight_bits, B):
    """The EXACT timed configuration (bench.py: FusedResNet, B=128, bench batches, HIP-graph replay)
    against the oracle for 3 optimiser steps. B=128 puts stage 1 at P = 131 072 pixels, so the
    one-launch conv backward (dgrad_wgrad_kernel) takes its >= 2-shard int32 wgrad branch. With the
    GPU's d loss / d logits injected, every weight, the exponents and every BN running mean /
    variance (dynamic_fixed_point.py:601-612) are bit-identical after each step; loss at 1e-5.
    weight_bits=4: configs[4]'s timed plan (bench.py --workload resnet20w4: packed 4-bit weight
    images, every fused kernel's W4 variant) against the oracle's 4-bit weight quantisers
    (dynamic_fixed_point.py:21-38 with bits=4). B=16 / 32: configs[2]'s per-GPU shards (global batch
    128 / 256 over 8 GPUs): the small-batch tile geometry (2-row tiles in every stage at B=16, 4-row
    stage-1 and 2-row stage-2 / 3 tiles at B=32, 2-row stage-3 tiles only at B=64; conv_mfma.hip
    tile_rows_for) and wgrad splits; (4, 16): the W4 variants of the 2-row tiles."""
    import bench
    from lbt_amd.fused import FusedResNet
    from lbt_amd.trainer import Trainer
    ctx, gm, om = _build_pair(seed=0, weight_bits=weight_bits)
    fm = FusedResNet(gm)
    state = dict(params=gpu_params(gm), accum=None, ranges=oresnet.init_ranges(om), step=0)
    state["accum"] = {k: np.zeros_like(v) for k, v in state["params"].items()}
    tr = Trainer(fm, lr=1e-2, momentum=0.9, batch_size=B, use_graph=True)
    xs, ys = bench.synthetic_batches(4, B, 1000, DEV)
    gn, on = _gpu_norms(gm), _oracle_norms(om)
    assert len(gn) == len(on) == 21
    for i in range(3):
        loss = tr.step(xs[i], ys[i]).item()
        torch.cuda.synchronize()
        dz = fm.dlogits.cpu().numpy()
        lref, state, octx = oresnet.train_step(om, state, xs[i].cpu().numpy(), ys[i].cpu().numpy(), lr=1e-2,
                                               momentum=0.9, seed=0, dz=dz)
        assert abs(loss - lref) <= 1e-5 * abs(lref), (i, loss, lref)
        np.testing.assert_allclose(dz, octx.dz, rtol=1e-5, atol=1e-9)
        gp = gpu_params(gm)
        for k in gp:
            assert np.array_equal(gp[k], state["params"][k]), (i, k)
        assert ctx.ranges() == state["ranges"], i
        for g, o in zip(gn, on):
            assert np.array_equal(g.X_mean_running.cpu().numpy(), o.mean_running), (i, g.name)
            assert np.array_equal(g.X_var_running.cpu().numpy(), o.var_running), (i, g.name)


@pytest.mark.parametrize("depth,blocks", [(32, (5, 5, 5)), (56, (9, 9, 9))])
def test_deeper_cifar_resnets_fused_vs_oracle(depth, blocks):
    """CIFAR10_Resnet32 / 56 (models.py CIFAR10_Resnet32-56, n = 5 / 9 ResidualBlock_q per stage) on the
    fused plan with HIP-graph replay against the oracle for 2 optimiser steps at B=32: weights, exponents
    and every BN running mean / variance bit-identical, loss at 1e-5 (d loss / d logits injected). Their
    30 / 54 block convs exceed one batched weight-gradient launch (24 jobs), so the stem-merged call
    (lbt_conv_wgrad_many_stem_i8) takes its two-call path here."""
    from lbt_amd import models
    from lbt_amd.fused import FusedResNet
    from lbt_amd.trainer import Trainer
    ctx = DfxpContext(seed=3)
    gm = getattr(models, "CIFAR10_Resnet%d" % depth)(8, weight_decay=2e-4, ctx=ctx)
    om = oresnet.build_resnet(blocks, 8, 2e-4)
    fm = FusedResNet(gm)
    state = dict(params=gpu_params(gm), accum=None, ranges=oresnet.init_ranges(om), step=0)
    state["accum"] = {k: np.zeros_like(v) for k, v in state["params"].items()}
    assert set(state["params"]) == set(oresnet.get_params(om))
    tr = Trainer(fm, lr=1e-2, momentum=0.9, batch_size=32, use_graph=True)
    gn, on = _gpu_norms(gm), _oracle_norms(om)
    assert len(gn) == len(on) == 2 * sum(blocks) + 3
    for i in range(2):
        x, y = synthetic_batch(32, seed=70 + i)
        loss = tr.step(torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV)).item()
        torch.cuda.synchronize()
        dz = fm.dlogits.cpu().numpy()
        lref, state, octx = oresnet.train_step(om, state, x, y, lr=1e-2, momentum=0.9, seed=3, dz=dz)
        assert abs(loss - lref) <= 1e-5 * abs(lref), (i, loss, lref)
        gp = gpu_params(gm)
        for k in gp:
            assert np.array_equal(gp[k], state["params"][k]), (i, k)
        assert ctx.ranges() == state["ranges"], i
        for g, o in zip(gn, on):
            assert np.array_equal(g.X_mean_running.cpu().numpy(), o.mean_running), (i, g.name)
            assert np.array_equal(g.X_var_running.cpu().numpy(), o.var_running), (i, g.name)


@pytest.mark.parametrize("scale", [1.0, 3.0])
def test_nonzero_target_overflow_rate_layers(scale):
    """target_overflow_rate = 0.01 (plumbed through every layer, dynamic_fixed_point.py:131,226,321,
    540,627; every model uses 0): conv + BN forward / backward codes and the range update against
    the oracle. Inputs are scaled so some quantisers overflow at rates between 0 and the target and
    above it -- the three branches of update_range (:83-94)."""
    rng = np.random.default_rng(int(scale * 10))
    t = 0.01
    ctx = DfxpContext(seed=31)
    conv = D.Conv2d_q("tc", 8, [3, 3, 16, 16], [1, 1, 1, 1], "SAME", use_bias=False, weight_decay=2e-4,
                      target_overflow_rate=t, input_nonnegative=True, ctx=ctx)
    bn = D.BatchNorm_q("tbn", 8, 16, weight_decay=2e-4, target_overflow_rate=t, ctx=ctx)
    oc = onn.Conv2dQ("tc", 8, [3, 3, 16, 16], [1, 1, 1, 1], "SAME", 2e-4)
    oc.W = conv.W.cpu().numpy().copy()
    ob = onn.BatchNormQ("tbn", 8, 16, 2e-4)
    # activations: ~1 % of the elements beyond the 9-bit range 2^(I) = 4 at I = 2
    x = np.abs(rng.normal(0, 1.2 * scale, size=(8, 16, 16, 16))).astype(np.float32)
    octx = onn.Ctx({r: 2 for r in oc.range_names() + ob.range_names()}, 0, 31, target=t)
    y = bn.forward(conv.forward(torch.from_numpy(x).to(DEV)))
    yr = ob.forward(oc.forward(x, octx), octx)
    assert np.array_equal(y.cpu().numpy(), yr)
    g = (rng.standard_normal(yr.shape) * 0.5 * scale).astype(np.float32)
    dx = conv.backward(bn.backward(torch.from_numpy(g).to(DEV)))
    dxr = oc.backward(ob.backward(g, octx), octx)
    assert np.array_equal(dx.cpu().numpy(), dxr)
    assert np.array_equal(conv.dW.cpu().numpy(), oc.dW)
    ctx.update_range_op()
    want = octx.new_ranges()
    assert ctx.ranges() == want
    # the non-zero target changes the outcome somewhere (else this test would not test it)
    z = {k: odfxp.update_range_from_counts(c1, c2, n, 0.0, b, 2) for k, (c1, c2, n, b) in octx.counts.items()}
    assert z != want


def test_torch_face_conv_matches_layer():
    from lbt_amd.dfxp import Conv2d_q, Linear_q, BatchNorm2d_q
    ctx = DfxpContext(seed=8)
    m = Conv2d_q(8, 16, 16, kernel_size=3, stride=1, padding=1, bias=False, ctx=ctx, name="tc",
                 input_nonnegative=True)
    ref = onn.Conv2dQ("tc", 8, [3, 3, 16, 16], [1, 1, 1, 1], "SAME", 0.0)
    ref.W = m.weight.detach().permute(2, 3, 1, 0).cpu().numpy().copy()
    rng = np.random.default_rng(8)
    x = rng.uniform(0, 2, size=(4, 16, 10, 10)).astype(np.float32)  # NCHW
    xt = torch.from_numpy(x).to(DEV).requires_grad_(True)
    y = m(xt)
    octx = onn.Ctx({r: 2 for r in ref.range_names()}, 0, 8)
    yr = ref.forward(x.transpose(0, 2, 3, 1).copy(), octx)
    assert np.array_equal(y.detach().permute(0, 2, 3, 1).cpu().numpy(), yr)
    g = rng.normal(0, 0.05, size=y.shape).astype(np.float32)
    y.backward(torch.from_numpy(g).to(DEV))
    dxr = ref.backward(g.transpose(0, 2, 3, 1).copy(), octx)
    assert np.array_equal(xt.grad.permute(0, 2, 3, 1).cpu().numpy(), dxr)
    assert np.array_equal(m.weight.grad.permute(2, 3, 1, 0).cpu().numpy(), ref.dW)


@pytest.mark.parametrize("shape", ["chain", "parallel"])
def test_torch_face_module_reuse_matches_oracle(shape):
    """One Conv2d_q called twice in a forward: chain ``conv(relu(conv(x)))`` or
    parallel ``conv(x1) + conv(x2)``. Each call's backward must read its own input codes although the
    second forward rewrote the layer's buffers (modules.py snapshots a displaced call's state). The
    oracle side is two Conv2dQ instances with the same name (same quantiser noise key) and weights;
    the outputs, the input gradients and the summed weight gradient are bit-identical. (The range
    update is not compared: the oracle keeps the last call's overflow counts per range name, the
    device adds every call's.)"""
    import torch.nn.functional as F
    from lbt_amd.dfxp import Conv2d_q
    ctx = DfxpContext(seed=9)
    m = Conv2d_q(8, 16, 16, kernel_size=3, stride=1, padding=1, bias=False, ctx=ctx, name="tr",
                 input_nonnegative=True)
    W = m.weight.detach().permute(2, 3, 1, 0).cpu().numpy().copy()
    refs = []
    for _ in range(2):
        o = onn.Conv2dQ("tr", 8, [3, 3, 16, 16], [1, 1, 1, 1], "SAME", 0.0)
        o.W = W.copy()
        refs.append(o)
    rng = np.random.default_rng(9)
    x1 = rng.uniform(0, 2, size=(4, 16, 10, 10)).astype(np.float32)
    x2 = rng.uniform(0, 1, size=(4, 16, 10, 10)).astype(np.float32)
    g = rng.normal(0, 0.05, size=(4, 16, 10, 10)).astype(np.float32)
    nhwc = lambda a: a.transpose(0, 2, 3, 1).copy()  # noqa: E731
    octx = onn.Ctx({r: 2 for r in refs[0].range_names()}, 0, 9)
    t1 = torch.from_numpy(x1).to(DEV).requires_grad_(True)
    if shape == "chain":
        h = m(t1)
        y = m(F.relu(h))
        y.backward(torch.from_numpy(g).to(DEV))
        zr = refs[0].forward(nhwc(x1), octx)
        ar = np.maximum(zr, 0).astype(np.float32)
        yr = refs[1].forward(ar, octx)
        gh = refs[1].backward(nhwc(g), octx)
        gh = np.where(zr > 0, gh, 0).astype(np.float32)
        dx1 = refs[0].backward(gh, octx)
        grads = [(t1, dx1)]
    else:
        t2 = torch.from_numpy(x2).to(DEV).requires_grad_(True)
        y = m(t1) + m(t2)
        y.backward(torch.from_numpy(g).to(DEV))
        ya = refs[0].forward(nhwc(x1), octx)
        yb = refs[1].forward(nhwc(x2), octx)
        yr = (ya + yb).astype(np.float32)
        dxb = refs[1].backward(nhwc(g), octx)
        dxa = refs[0].backward(nhwc(g), octx)
        grads = [(t1, dxa), (t2, dxb)]
    assert np.array_equal(y.detach().permute(0, 2, 3, 1).cpu().numpy(), yr)
    for t, ref in grads:
        assert np.array_equal(t.grad.permute(0, 2, 3, 1).cpu().numpy(), ref)
    dw = (refs[0].dW + refs[1].dW).astype(np.float32)
    assert np.array_equal(m.weight.grad.permute(2, 3, 1, 0).cpu().numpy(), dw)


def test_torch_face_custom_py_network_matches_oracle():
    """custom.py's own network (custom.py:10-12,15-50) on the torch face: conv5x5(1 -> 6, padding=1) ->
    ReLU -> MaxPool2d(2) -> conv5x5(6 -> 16) -> ReLU -> MaxPool2d(2) -> conv5x5(16 -> 120) -> ReLU ->
    flatten -> Linear_q(1080 -> 84) -> ReLU -> Linear_q(84 -> 10), MNIST-shaped input. (The reference
    feeds a 120-feature Linear_q from the 3x3x120 map; fc1 takes the 1080 features here.) The 5x5 convs
    have Cin = 1 / 6 / 16 (signed 9-bit inputs: the generic path) and Linear_q its default bias.
    Forward logits and every parameter / input gradient are bit-identical to the oracle layers
    composed the same way (torch's max pool / ReLU on both sides)."""
    import torch.nn.functional as F
    from lbt_amd.dfxp import Conv2d_q, Linear_q
    ctx = DfxpContext(seed=12)
    convs = [Conv2d_q(8, a, b, kernel_size=5, stride=1, padding=1, bias=False, ctx=ctx, name="c%d" % i)
             for i, (a, b) in enumerate(((1, 6), (6, 16), (16, 120)))]
    fc1 = Linear_q(8, 1080, 84, ctx=ctx, name="fc1")
    fc2 = Linear_q(8, 84, 10, ctx=ctx, name="fc2")
    with torch.no_grad():
        fc1.bias.copy_(torch.linspace(-0.05, 0.05, 84))
        fc2.bias.copy_(torch.linspace(-0.02, 0.03, 10))
    oconvs = []
    for i, c in enumerate(convs):
        o = onn.Conv2dQ("c%d" % i, 8, list(c.layer.ksize), [1, 1, 1, 1], 1, 0.0)
        o.W = c.weight.detach().permute(2, 3, 1, 0).cpu().numpy().copy()
        oconvs.append(o)
    ofc = []
    for name, f in (("fc1", fc1), ("fc2", fc2)):
        o = onn.DenseQ(name, 8, f.weight.shape[1], f.weight.shape[0], 0.0, use_bias=True)
        o.W = f.weight.detach().t().cpu().numpy().copy()
        o.b = f.bias.detach().cpu().numpy().copy()
        ofc.append(o)
    rng = np.random.default_rng(12)
    x = rng.uniform(-1, 1, size=(8, 1, 28, 28)).astype(np.float32)
    xt = torch.from_numpy(x).to(DEV).requires_grad_(True)
    h = xt
    for i, c in enumerate(convs):
        h = F.relu(c(h))
        if i < 2:
            h = F.max_pool2d(h, 2, 2)
    h.retain_grad()
    feat = h.permute(0, 2, 3, 1).reshape(8, -1)  # NHWC flatten (the oracle's order)
    out = fc2(F.relu(fc1(feat)))
    g = rng.normal(0, 0.05, size=(8, 10)).astype(np.float32)
    out.backward(torch.from_numpy(g).to(DEV))
    # oracle, same composition (NHWC)
    octx = onn.Ctx({r: 2 for o in oconvs + ofc for r in o.range_names()}, 0, 12)
    hs = [x.transpose(0, 2, 3, 1).copy()]
    pre, pooled = [], []
    for i, o in enumerate(oconvs):
        z = o.forward(hs[-1], octx)
        pre.append(z)
        a = np.maximum(z, 0).astype(np.float32)
        if i < 2:
            t = torch.from_numpy(a.transpose(0, 3, 1, 2).copy()).requires_grad_(True)
            p = F.max_pool2d(t, 2, 2)
            pooled.append(t)
            a = p.detach().numpy().transpose(0, 2, 3, 1).copy()
            pooled.append(p)
        hs.append(a)
    f = hs[-1].reshape(8, -1)
    z1 = ofc[0].forward(f, octx)
    a1 = np.maximum(z1, 0).astype(np.float32)
    z2 = ofc[1].forward(a1, octx)
    assert np.array_equal(out.detach().cpu().numpy(), z2)
    g1 = ofc[1].backward(g, octx)
    g1 = np.where(z1 > 0, g1, 0).astype(np.float32)
    gf = ofc[0].backward(g1, octx).reshape(hs[-1].shape)
    gh = gf
    for i in reversed(range(3)):
        if i < 2:
            t, p = pooled[2 * i], pooled[2 * i + 1]
            t.grad = None
            p.backward(torch.from_numpy(gh.transpose(0, 3, 1, 2).copy()))
            gh = t.grad.numpy().transpose(0, 2, 3, 1).copy()
        gh = np.where(pre[i] > 0, gh, 0).astype(np.float32)
        gh = oconvs[i].backward(gh, octx)
    assert np.array_equal(fc2.weight.grad.t().cpu().numpy(), ofc[1].dW)
    assert np.array_equal(fc2.bias.grad.cpu().numpy(), ofc[1].db)
    assert np.array_equal(fc1.weight.grad.t().cpu().numpy(), ofc[0].dW)
    assert np.array_equal(fc1.bias.grad.cpu().numpy(), ofc[0].db)
    for c, o in zip(convs, oconvs):
        assert np.array_equal(c.weight.grad.permute(2, 3, 1, 0).cpu().numpy(), o.dW)
    assert np.array_equal(xt.grad.permute(0, 2, 3, 1).cpu().numpy(), gh)
    ctx.update_range_op()
    assert ctx.ranges() == octx.new_ranges()


def test_torch_face_batchnorm2d_matches_oracle():
    """BatchNorm2d_q (custom.py:5; torch signature (bits, num_features)) on custom.py's conv-2 output
    geometry (16 channels, 11 x 11, NCHW): forward, the gamma / beta gradients, the input gradient and
    the running statistics are bit-identical to the oracle's BatchNormQ (Normalization_q +
    Rescale_q, dynamic_fixed_point.py:539-694)."""
    from lbt_amd.dfxp import BatchNorm2d_q
    ctx = DfxpContext(seed=13)
    bn = BatchNorm2d_q(8, 16, ctx=ctx, name="bn")
    with torch.no_grad():
        bn.weight.copy_(torch.linspace(0.7, 1.3, 16))
        bn.bias.copy_(torch.linspace(-0.2, 0.2, 16))
    ob = onn.BatchNormQ("bn", 8, 16, 0.0)
    ob.layers[1].gamma = bn.weight.detach().cpu().numpy().copy()
    ob.layers[1].beta = bn.bias.detach().cpu().numpy().copy()
    rng = np.random.default_rng(13)
    x = (rng.standard_normal((4, 16, 11, 11)) * 1.7 + 0.3).astype(np.float32)
    xt = torch.from_numpy(x).to(DEV).requires_grad_(True)
    y = bn(xt)
    octx = onn.Ctx({r: 2 for r in ob.range_names()}, 0, 13)
    yr = ob.forward(x.transpose(0, 2, 3, 1).copy(), octx)
    assert np.array_equal(y.detach().permute(0, 2, 3, 1).cpu().numpy(), yr)
    g = (rng.standard_normal(y.shape) * 0.1).astype(np.float32)
    y.backward(torch.from_numpy(g).to(DEV))
    dxr = ob.backward(g.transpose(0, 2, 3, 1).copy(), octx)
    assert np.array_equal(xt.grad.permute(0, 2, 3, 1).cpu().numpy(), dxr)
    assert np.array_equal(bn.weight.grad.cpu().numpy(), ob.layers[1].dgamma)
    assert np.array_equal(bn.bias.grad.cpu().numpy(), ob.layers[1].dbeta)
    assert np.array_equal(bn.norm.X_mean_running.cpu().numpy(), ob.layers[0].mean_running)
    assert np.array_equal(bn.norm.X_var_running.cpu().numpy(), ob.layers[0].var_running)
    ctx.update_range_op()
    assert ctx.ranges() == octx.new_ranges()


def test_bench_workload_loss_trajectory_matches_oracle():
    """The exact bench workload (B=128, bench.py batches, graph-captured Trainer): the first 3 steps'
    losses and exponents match the oracle's step-for-step (the reference semantics on this random-
    label synthetic data diverge after a few steps in BOTH implementations identically)."""
    import bench
    from lbt_amd.trainer import Trainer
    ctx, gm, om = _build_pair(seed=0)
    state = dict(params=gpu_params(gm), accum=None, ranges=oresnet.init_ranges(om), step=0)
    state["accum"] = {k: np.zeros_like(v) for k, v in state["params"].items()}
    tr = Trainer(gm, lr=1e-2, momentum=0.9, batch_size=128, use_graph=True)
    xs, ys = bench.synthetic_batches(4, 128, 1000, DEV)
    for i in range(3):
        loss = tr.step(xs[i], ys[i]).item()
        lref, state, _ = oresnet.train_step(om, state, xs[i].cpu().numpy(), ys[i].cpu().numpy(), lr=1e-2,
                                            momentum=0.9, seed=0)
        assert abs(loss - lref) <= 1e-5 * abs(lref), (i, loss, lref)
        assert ctx.ranges() == state["ranges"], i


def test_fused_executor_bitidentical_to_layerwise():
    """FusedResNet (the bench path) == the Layer_q model executed layer by layer, bit for bit:
    logits, loss, every gradient and every exponent update, then 3 graph-captured optimiser steps."""
    from lbt_amd.fused import FusedResNet
    from lbt_amd.models import CIFAR10_Resnet20
    from lbt_amd.trainer import Trainer
    x, y = synthetic_batch(32, seed=5)
    xt, yt = torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV)
    ctxA, ctxB = DfxpContext(seed=6), DfxpContext(seed=6)
    A = CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctxA)
    B = FusedResNet(CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctxB))
    la = A.forward(xt).cpu().numpy()
    lb = B.forward(xt).cpu().numpy()
    assert np.array_equal(la, lb)
    assert A.compute_loss(yt).item() == B.compute_loss(yt).item()
    A.backward()
    B.backward()
    ga, gb = gpu_grads(A), gpu_grads(B.model)
    for k in ga:
        assert np.array_equal(ga[k], gb[k]), k
    ctxA.update_range_op()
    ctxB.update_range_op()
    assert ctxA.ranges() == ctxB.ranges()
    # training: eager layer-wise vs graph-captured fused
    ctxA, ctxB = DfxpContext(seed=7), DfxpContext(seed=7)
    tA = Trainer(CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctxA), lr=1e-2, momentum=0.9, use_graph=False)
    tB = Trainer(FusedResNet(CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctxB)), lr=1e-2, momentum=0.9,
                 use_graph=True)
    for i in range(3):
        x, y = synthetic_batch(32, seed=20 + i)
        xt, yt = torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV)
        assert tA.step(xt, yt).item() == tB.step(xt, yt).item()
    torch.cuda.synchronize()
    assert np.array_equal(tA.flat.w.cpu().numpy(), tB.flat.w.cpu().numpy())
    assert ctxA.ranges() == ctxB.ranges()


@pytest.mark.parametrize("chain", ["1", "0"])
def test_fused_separate_calls_bn_state_equals_layerwise(chain, monkeypatch):
    """forward() / compute_loss() / backward() of the fused plan (the separate head launches) run the
    last block's end chain exactly once, with and without the head chain (it ran twice
    when LBT_HEAD_CHAIN=0, moving the BN running averages twice and double-counting the Rescale_q
    overflows): BN running statistics, gradients and the updated exponents equal the layer-wise model."""
    from lbt_amd.fused import FusedResNet
    from lbt_amd.models import CIFAR10_Resnet20
    monkeypatch.setenv("LBT_HEAD_CHAIN", chain)
    x, y = synthetic_batch(24, seed=15)
    xt, yt = torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV)
    ctxA, ctxB = DfxpContext(seed=16), DfxpContext(seed=16)
    A = CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctxA)
    B = FusedResNet(CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctxB))
    assert np.array_equal(A.forward(xt).cpu().numpy(), B.forward(xt).cpu().numpy())
    assert A.compute_loss(yt).item() == B.compute_loss(yt).item()
    A.backward()
    B.backward()
    names = [getattr(f, "kname", "") for f in B._fwd + B._hfwd]
    assert names.count("chain_fwd_kernel") == sum(1 for f in B._fwd if getattr(f, "kname", "") == "chain_fwd_kernel") \
        + (1 if chain == "1" else 0)
    ga, gb = gpu_grads(A), gpu_grads(B.model)
    for k in ga:
        assert np.array_equal(ga[k], gb[k]), k
    ra = [t.cpu().numpy() for t in _bn_running(A)]
    rb = [t.cpu().numpy() for t in _bn_running(B.model)]
    assert len(ra) == len(rb) > 0
    for u, v in zip(ra, rb):
        assert np.array_equal(u, v)
    ctxA.update_range_op()
    ctxB.update_range_op()
    assert ctxA.ranges() == ctxB.ranges()


def _bn_running(model):
    """Every Normalization_q's running mean / variance tensors, in model order."""
    from lbt_amd.trainer import Trainer
    return [t for l in Trainer._bn_layers(types.SimpleNamespace(model=model)) for t in (l.X_mean_running, l.X_var_running)]


@pytest.mark.parametrize("N,HW,C,K,table", [(128, 64, 64, 10, True), (300, 16, 32, 7, False), (5, 3, 256, 64, True), (700, 4, 8, 3, True)])
def test_head_kernel_equals_launch_sequence(N, HW, C, K, table):
    """lbt_head_fwd_bwd + lbt_step_reduce's head block == avgpool_fwd, quantize, dense fwd,
    softmax_xent, quantize, dense wgrad + reduce, dense dgrad, avgpool_bwd as separate launches:
    every output and counter bit for bit (with noise tables and with inline Philox; N > 256
    exercises the loss-term striding)."""
    import ctypes
    from lbt_amd import _lib
    rng = np.random.default_rng(N + C)
    x = torch.from_numpy(rng.uniform(0, 3, size=(N, HW, C)).astype(np.float32)).to(DEV)
    W = torch.from_numpy(rng.uniform(-0.5, 0.5, size=(C, K)).astype(np.float32)).to(DEV)
    labels = torch.from_numpy(rng.integers(0, K, size=N).astype(np.int32)).to(DEV)
    out = {}
    for mode in ("seq", "head"):
        ctx = DfxpContext(seed=77)
        qx = ctx.quantizer("d/X_range", 8, 2)
        qw = ctx.quantizer("d/W_range", 8, 1)
        qg = ctx.quantizer("d/grad_range", 8, -4)
        dx, dg = _lib.QDesc.from_buffer_copy(qx.desc), _lib.QDesc.from_buffer_copy(qg.desc)
        keep = []
        if table:
            for d_, q, n in ((dx, qx, C), (dg, qg, K)):
                t = torch.from_numpy(odfxp.noise_for((1, n), q.qid, 0, 77).reshape(-1).astype(np.float32)).to(DEV)
                keep.append(t)
                d_.noise = t.data_ptr()
        wq = torch.empty((C, K), dtype=torch.int8, device=DEV)
        _lib.call("lbt_dfxp_quantize", _lib.ptr(W), _lib.ptr(wq), OUT_I8, 1, C * K, qw.desc_nostats(), None, 0,
                  _lib.stream())
        pooled = torch.empty((N, C), device=DEV)
        pq = torch.empty((N, C), dtype=torch.int8, device=DEV)
        logits = torch.empty((N, K), device=DEV)
        loss = torch.empty(1, device=DEV)
        dz = torch.empty((N, K), device=DEV)
        gq = torch.empty((N, K), dtype=torch.int8, device=DEV)
        dW = torch.empty((C, K), device=DEV)
        gx = torch.empty((N, HW, C), device=DEV)
        wd2 = ops.f32(4e-4)
        st = _lib.stream()
        if mode == "seq":
            dd = _lib.ConvDesc(N, 1, 1, C, K, 1, 1, 1, 1, 0, 0, 0, 0, 1, 1)
            _lib.call("lbt_avgpool_fwd", _lib.ptr(x), _lib.ptr(pooled), N, HW, C, st)
            _lib.call("lbt_dfxp_quantize", _lib.ptr(pooled), _lib.ptr(pq), OUT_I8, N, C, dx, None, 0, st)
            _lib.call("lbt_conv_fwd_generic", _lib.ptr(pq), 0, _lib.ptr(wq), dd, dx, qw.desc, _lib.ptr(logits), st)
            _lib.call("lbt_softmax_xent", _lib.ptr(logits), _lib.ptr(labels), N, K, _lib.ptr(loss), _lib.ptr(dz), st)
            _lib.call("lbt_dfxp_quantize", _lib.ptr(dz), _lib.ptr(gq), OUT_I8, N, K, dg, None, 0, st)
            ns = ops.wgrad_nsplit(dd, generic=True)
            slab = torch.empty((ns, C, K), dtype=torch.int32, device=DEV)
            _lib.call("lbt_conv_wgrad_generic", _lib.ptr(pq), 0, _lib.ptr(gq), dd, _lib.ptr(slab), ns, st)
            _lib.call("lbt_conv_wgrad_reduce", _lib.ptr(slab), ns, C, K, 0, None, dx, dg, _lib.ptr(W), wd2,
                      _lib.ptr(dW), st)
            dp = torch.empty((N, C), device=DEV)
            _lib.call("lbt_conv_dgrad_generic", _lib.ptr(gq), _lib.ptr(wq), dd, dg, qw.desc, _lib.ptr(dp), None, st)
            _lib.call("lbt_avgpool_bwd", _lib.ptr(dp), _lib.ptr(gx), N, HW, C, st)
        else:
            lib = _lib.load()
            scratch = torch.empty(lib.lbt_head_scratch_bytes(N, C, K), dtype=torch.uint8, device=DEV)
            h = _lib.Head(x.data_ptr(), N, HW, C, K, pooled.data_ptr(), pq.data_ptr(), dx, wq.data_ptr(), qw.desc,
                          labels.data_ptr(), logits.data_ptr(), loss.data_ptr(), dz.data_ptr(), gq.data_ptr(), dg,
                          W.data_ptr(), wd2, dW.data_ptr(), gx.data_ptr(), scratch.data_ptr())
            _lib.call("lbt_head_fwd_bwd", ctypes.byref(h), st)
            # the batch reductions (Dense_q dW, loss) run in the step's final reduce launch
            _lib.call("lbt_step_reduce", None, 0, 0, None, 0, 0, ctypes.byref(h), st)
        torch.cuda.synchronize()
        out[mode] = dict(pooled=pooled, pq=pq, logits=logits, loss=loss, dz=dz, gq=gq, dW=dW, gx=gx,
                         counts=ctx.counts_view()[:3].sum(1))
    for k, v in out["seq"].items():
        assert torch.equal(v, out["head"][k]), k


@pytest.mark.parametrize("B,w4", [(32, False), (128, False), (32, True)])
def test_fused_conv_backward_equals_launch_pair(B, w4):
    """lbt_conv_bwd_fused_i8 (pass B + dgrad + pass A in one launch per stride-1 3x3 conv, each
    conv's wgrad deferred into the next such launch) and lbt_conv_fwd_fused_i8 (the BN chain that
    produces a conv's input run inside the conv launch) == the chain_bwd_b / dgrad_wgrad and
    chain_fwd / conv_fwd launches they replace: gradients, momentum, weights, exponents and BN running
    statistics bit-identical after two optimiser steps (eager, then graph replay)."""
    from lbt_amd.fused import FusedResNet
    from lbt_amd.models import CIFAR10_Resnet20
    from lbt_amd.trainer import Trainer
    outs = []
    for fb in (False, True):
        ctx = DfxpContext(seed=4)
        m = FusedResNet(CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctx, weight_bits=4 if w4 else None))
        m.fuse_bwd = m.fuse_fwd = fb
        tr = Trainer(m, lr=1e-2, momentum=0.9, batch_size=B, use_graph=fb)
        for i in range(2):
            x, y = synthetic_batch(B, seed=30 + i)
            tr.step(torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV))
        torch.cuda.synchronize()
        nf = sum(1 for f in m._bwd if getattr(f, "kname", "") == "conv_bwd_kernel")
        assert nf == (16 if fb else 0), nf
        nf = sum(1 for f in m._fwd if getattr(f, "kname", "") == "conv_fwd_fused_kernel")
        assert nf == (16 if fb else 0), nf
        bn = [t.cpu().numpy() for l in tr._bn_layers() for t in (l.X_mean_running, l.X_var_running)]
        outs.append((tr.flat.g.cpu().numpy(), tr.flat.a.cpu().numpy(), tr.flat.w.cpu().numpy(), ctx.ranges(), bn,
                     m.loss.item()))
    a, b = outs
    for i in range(3):
        assert np.array_equal(a[i], b[i]), i
    assert a[3] == b[3]
    for u, v in zip(a[4], b[4]):
        assert np.array_equal(u, v)
    assert a[5] == b[5]


@pytest.mark.parametrize("bwd2", [True, False])
@pytest.mark.parametrize("w4", [False, True])
def test_pair_launches_equal_single_launches(w4, bwd2, monkeypatch):
    """lbt_conv_fwd_pair_i8 (a projection block's 3x3/2 conv and 1x1/2 shortcut in one launch),
    lbt_bn_chain_bwd_b_pair (its shortcut-BN and first-BN pass B in one launch) and
    lbt_conv_dgrad2_chain_i8 (both convs' dgrads + the consumer's pass A in one launch) -- or, bwd2,
    lbt_conv_bwd2_fused_i8 (both pass-B chains, both dgrads and the pass A in ONE launch) and
    lbt_conv_fwd2_fused_i8 (the previous block's end chain, both strided convs and both quantising
    epilogues in ONE launch) == the single launches they replace: gradients, momentum, weights,
    exponents, BN running statistics and loss bit-identical after two graph-replayed optimiser steps
    at B=128."""
    monkeypatch.setenv("LBT_FUSE_BWD2", "1" if bwd2 else "0")
    monkeypatch.setenv("LBT_FUSE_FWD2", "1" if bwd2 else "0")
    from lbt_amd.fused import FusedResNet
    from lbt_amd.models import CIFAR10_Resnet20
    from lbt_amd.trainer import Trainer
    outs = []
    for pair in (False, True):
        ctx = DfxpContext(seed=6)
        m = FusedResNet(CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctx, weight_bits=4 if w4 else None))
        m.pair_launch = pair
        tr = Trainer(m, lr=1e-2, momentum=0.9, batch_size=128, use_graph=True)
        for i in range(2):
            x, y = synthetic_batch(128, seed=40 + i)
            tr.step(torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV))
        torch.cuda.synchronize()
        nf = sum(1 for f in m._fwd if getattr(f, "kname", "").startswith("conv_gemm2_kernel"))
        nb = sum(1 for f in m._bwd if getattr(f, "kname", "") == "chain_bwd_b2_kernel")
        nd = sum(1 for f in m._bwd if getattr(f, "kname", "").startswith("conv_dgrad2_kernel"))
        n2 = sum(1 for f in m._bwd if getattr(f, "kname", "") == "conv_bwd2_kernel")
        nf2 = sum(1 for f in m._fwd if getattr(f, "kname", "") == "conv_fwd2_kernel")
        want = ((0, 0, 0, 2, 2) if bwd2 else (2, 2, 2, 0, 0)) if pair else (0, 0, 0, 0, 0)
        assert (nf, nb, nd, n2, nf2) == want, (nf, nb, nd, n2, nf2)
        bn = [t.cpu().numpy() for l in tr._bn_layers() for t in (l.X_mean_running, l.X_var_running)]
        outs.append((tr.flat.g.cpu().numpy(), tr.flat.a.cpu().numpy(), tr.flat.w.cpu().numpy(), ctx.ranges(), bn,
                     m.loss.item()))
    a, b = outs
    for i in range(3):
        assert np.array_equal(a[i], b[i]), i
    assert a[3] == b[3]
    for u, v in zip(a[4], b[4]):
        assert np.array_equal(u, v)
    assert a[5] == b[5]


@pytest.mark.parametrize("B", [128, 32])
def test_stem_merge_equals_separate_launches(B, monkeypatch):
    """lbt_conv_wgrad_many_stem_i8 (the batched weight gradients with the stem's whole backward as the
    launch's last workgroups) == lbt_conv_wgrad_many_i8 followed by lbt_conv_stem_bwd: gradients,
    momentum, weights, exponents, BN running statistics and loss bit-identical after two
    graph-replayed optimiser steps (B=128 is the bench workload)."""
    from lbt_amd.fused import FusedResNet
    from lbt_amd.models import CIFAR10_Resnet20
    from lbt_amd.trainer import Trainer
    outs = []
    for merge in ("0", "1"):
        monkeypatch.setenv("LBT_STEM_MERGE", merge)
        ctx = DfxpContext(seed=9)
        m = FusedResNet(CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctx))
        tr = Trainer(m, lr=1e-2, momentum=0.9, batch_size=B, use_graph=True)
        for i in range(2):
            x, y = synthetic_batch(B, seed=60 + i)
            tr.step(torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV))
        torch.cuda.synchronize()
        names = [getattr(f, "kname", "") for f in m._bwd]
        want = (1, 0, 0) if merge == "1" else (0, 1, 1)
        got = (names.count("conv_wgrad_many_stem_kernel"), names.count("conv_wgrad_many_kernel"),
               names.count("stem_bwd_kernel"))
        assert got == want, (merge, got)
        bn = [t.cpu().numpy() for l in tr._bn_layers() for t in (l.X_mean_running, l.X_var_running)]
        outs.append((tr.flat.g.cpu().numpy(), tr.flat.a.cpu().numpy(), tr.flat.w.cpu().numpy(), ctx.ranges(), bn,
                     m.loss.item()))
    a, b = outs
    for i in range(3):
        assert np.array_equal(a[i], b[i]), i
    assert a[3] == b[3]
    for u, v in zip(a[4], b[4]):
        assert np.array_equal(u, v)
    assert a[5] == b[5]


@pytest.mark.parametrize("B", [128, 32])
def test_fused_update_and_head_chain_equal_separate_launches(B, monkeypatch):
    """The round-4 launch merges against the launches they replace, two graph-replayed optimiser steps
    then one eager one: the optimiser + update_range inside the step's last launch
    (lbt_step_reduce_update, LBT_FUSED_UPDATE) vs lbt_step_reduce + lbt_step_update, and the last
    block's end chain inside the fused head (lbt_head.chain, LBT_HEAD_CHAIN) vs lbt_bn_chain_fwd +
    the head on its output. Gradients, momentum, weights, exponents, noise step, BN running statistics
    and loss bit-identical."""
    from lbt_amd.fused import FusedResNet
    from lbt_amd.models import CIFAR10_Resnet20
    from lbt_amd.trainer import Trainer
    outs = []
    for upd, chain in (("1", "1"), ("0", "0"), ("1", "0"), ("0", "1")):
        monkeypatch.setenv("LBT_FUSED_UPDATE", upd)
        monkeypatch.setenv("LBT_HEAD_CHAIN", chain)
        ctx = DfxpContext(seed=11)
        m = FusedResNet(CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctx))
        tr = Trainer(m, lr=1e-2, momentum=0.9, batch_size=B, use_graph=True)
        for i in range(3):
            if i == 2:
                tr.use_graph = False
            x, y = synthetic_batch(B, seed=80 + i)
            tr.step(torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV))
        torch.cuda.synchronize()
        names = [getattr(f, "kname", "") for f in m._fwd]
        assert ("chain_fwd_kernel" in names) == (chain == "0"), (upd, chain)
        assert m.updates_in_step() == (upd == "1")
        bn = [t.cpu().numpy() for l in tr._bn_layers() for t in (l.X_mean_running, l.X_var_running)]
        outs.append((tr.flat.g.cpu().numpy(), tr.flat.a.cpu().numpy(), tr.flat.w.cpu().numpy(), ctx.ranges(), bn,
                     m.loss.item(), int(ctx.step.item())))
    ref = outs[0]
    for o in outs[1:]:
        for i in range(3):
            assert np.array_equal(ref[i], o[i]), i
        assert ref[3] == o[3]
        for u, v in zip(ref[4], o[4]):
            assert np.array_equal(u, v)
        assert ref[5] == o[5] and ref[6] == o[6] == 3


# (N, H, W, Cin, Cout, k, s): the staged 3x3 / stride-1 body (W | 64, whole-row chunks) and the
# per-tap body (strided / 1x1), mixed in one launch
WGRAD_MANY_CASES = [(8, 32, 32, 16, 16, 3, 1), (8, 16, 16, 32, 32, 3, 1), (8, 8, 8, 64, 64, 3, 1),
                    (8, 32, 32, 16, 32, 3, 2), (8, 32, 32, 16, 32, 1, 2), (4, 16, 16, 32, 64, 3, 2),
                    (2, 4, 64, 16, 32, 3, 1), (3, 12, 8, 32, 16, 3, 1), (128, 8, 8, 64, 64, 3, 1)]


def _wgrad_ref(x, g, d, fill):
    """Exact int64 sum_p X_tap (x) G of a TF-SAME conv (x: int8 NHWC codes, out-of-image taps = fill)."""
    N, H, W, Cin = x.shape
    _, Ho, Wo, Cout = g.shape
    xp = np.full((N, H + d.PT + d.PB + d.SH * 2, W + d.PL + d.PR + d.SW * 2, Cin), fill, np.int64)
    xp[:, d.PT:d.PT + H, d.PL:d.PL + W] = x
    out = np.zeros((d.KH, d.KW, Cin, Cout), np.int64)
    gg = g.reshape(-1, Cout).astype(np.int64)
    for kh in range(d.KH):
        for kw in range(d.KW):
            xt = xp[:, kh:kh + d.SH * Ho:d.SH, kw:kw + d.SW * Wo:d.SW][:, :Ho, :Wo].reshape(-1, Cin)
            out[kh, kw] = xt.T @ gg
    return out.reshape(-1, Cout)


def test_wgrad_many_equals_single_launches():
    """lbt_conv_wgrad_many_i8 (one launch, staged and per-tap bodies) == one lbt_conv_wgrad_i8 per
    conv == the exact integer sum, shard totals compared (int32 partials, exact)."""
    from lbt_amd._lib import WgradJob
    rng = np.random.default_rng(5)
    jobs, refs, singles, keep = [], [], [], []
    for (N, H, W, Cin, Cout, k, s) in WGRAD_MANY_CASES:
        d = ops.conv_desc(N, H, W, Cin, Cout, k, k, s, s, "SAME")
        x = rng.integers(-128, 128, size=(N, H, W, Cin), dtype=np.int8)
        g = rng.integers(-128, 128, size=(N, d.Ho, d.Wo, Cout), dtype=np.int8)
        xq, gq = torch.from_numpy(x).to(DEV), torch.from_numpy(g).to(DEV)
        ns = ops.wgrad_nsplit_batched(d)
        nh = ops.wgrad_nshard(d, ns)
        slab = torch.zeros((nh, k * k * Cin, Cout), dtype=torch.int32, device=DEV)
        keep += [xq, gq, slab]
        jobs.append(WgradJob(xq.data_ptr(), 1, gq.data_ptr(), d, slab.data_ptr(), ns, nh))
        refs.append((slab, _wgrad_ref(x, g, d, -128)))
        ns1 = ops.wgrad_nsplit(d)
        nh1 = ops.wgrad_nshard(d, ns1)
        slab1 = torch.zeros((nh1, k * k * Cin, Cout), dtype=torch.int32, device=DEV)
        ops.conv_wgrad_i8(xq, 1, gq, d, slab1, ns1, nh1)
        singles.append(slab1)
    arr = (WgradJob * len(jobs))(*jobs)
    ops.call("lbt_conv_wgrad_many_i8", arr, len(jobs), ops.stream())
    # more jobs than one launch carries (24): two launches, same sums
    for slab, _ in refs:
        slab.zero_()
    arr3 = (WgradJob * (3 * len(jobs)))(*(jobs * 3))
    ops.call("lbt_conv_wgrad_many_i8", arr3, 3 * len(jobs), ops.stream())
    torch.cuda.synchronize()
    for (slab, ref), slab1, case in zip(refs, singles, WGRAD_MANY_CASES):
        got = slab.cpu().numpy().astype(np.int64).sum(0)
        assert np.array_equal(got, 3 * ref), case
        assert np.array_equal(slab1.cpu().numpy().astype(np.int64).sum(0), ref), case
    bad = WgradJob(jobs[0].xq, 1, jobs[0].gq, jobs[0].d, None, jobs[0].nsplit, jobs[0].nshard)
    arrb = (WgradJob * 2)(jobs[0], bad)
    with pytest.raises(Exception):
        ops.call("lbt_conv_wgrad_many_i8", arrb, 2, ops.stream())
