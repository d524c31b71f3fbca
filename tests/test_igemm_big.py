"""configs[3]'s production GEMM: the 256-row LDS-DMA implicit GEMM (igemm.hip igemm_big_kernel), which
runs every large ResNet-50 forward and dgrad GEMM at the benched B=256.

The kernel is taken only by GEMMs with >= 200 256-row tiles; ``ops.igemm_forced`` (the C-ABI
lbt_igemm_set_tuning) lowers that threshold and picks the column tile and ring depth per call, so
these tests put every variant on small ragged shapes and compare it, bit for bit, with the generic
VALU kernels (conv_generic.hip), whose integer arithmetic restates tf.nn.conv2d and its input
gradient on the quantised codes (reference dynamic_fixed_point.py:287-305). The last test runs a
bottleneck model large enough to take the kernel with the default selection against the oracle.
"""
import numpy as np
import pytest
import torch

from oracle import nn as onn
from oracle import resnet as oresnet

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (stages, max_bn) pairs: every ring depth and column tile of the kernel
VARIANTS = [(2, 64), (3, 64), (4, 64), (2, 128), (3, 128), (4, 128), (2, 256)]


def _setup(N, H, Cin, Cout, k, s, seed):
    from lbt_amd.dfxp import ops
    from lbt_amd.runtime import DfxpContext
    rng = np.random.default_rng(seed)
    ctx = DfxpContext(seed=seed)
    qx, qw, qg = ctx.quantizer("t/X", 9, 2), ctx.quantizer("t/W", 8, 0), ctx.quantizer("t/g", 16, -3)
    d = ops.conv_desc(N, H, H, Cin, Cout, k, k, s, s, "SAME")
    W = torch.from_numpy(rng.uniform(-1, 1, size=(k, k, Cin, Cout)).astype(np.float32)).to(DEV)
    w_hwio = torch.empty((k, k, Cin, Cout), dtype=torch.int8, device=DEV)
    ksf, ksd = ops.packed_slices(k, k, Cin), ops.packed_slices(k, k, Cout)
    wf = torch.zeros((Cout, ksf * 16), dtype=torch.int8, device=DEV)
    wd = torch.zeros((Cin, ksd * 16), dtype=torch.int8, device=DEV)
    colsum = torch.zeros(Cout, dtype=torch.int32, device=DEV)
    ops.quantize_weight(W, qw, w_hwio=w_hwio, wf=wf, ksf=ksf, wd=wd, ksd=ksd, colsum=colsum)
    return rng, ctx, (qx, qw, qg), d, w_hwio, (wf, ksf), (wd, ksd), colsum


def _launches():
    from lbt_amd.dfxp import ops
    return ops.igemm_tuning()["launches"]


def test_tuning_roundtrip_and_validation():
    from lbt_amd import _lib
    from lbt_amd.dfxp import ops
    t0 = ops.igemm_tuning()
    with ops.igemm_forced(min_tiles=1, stages=3, max_bn=64):
        t = ops.igemm_tuning()
        assert (t["min_tiles"], t["stages"], t["max_bn"]) == (1, 3, 64)
    assert {k: v for k, v in ops.igemm_tuning().items() if k != "launches"} == \
        {k: v for k, v in t0.items() if k != "launches"}
    for bad in (dict(stages=5), dict(stages=1), dict(max_bn=32), dict(min_tiles=0)):
        with pytest.raises(_lib.LbtError):
            with ops.igemm_forced(**bad):
                pass


@pytest.mark.parametrize("N,H,Cin,Cout,k,s", [
    (3, 14, 64, 128, 3, 1),    # M = 588: two full 256-row tiles + 76 rows
    (2, 15, 128, 256, 1, 1),   # M = 450, 256 columns (the 256-column tile)
    (2, 15, 64, 64, 3, 2),     # strided fwd, M = 128: one partial tile
    (1, 9, 192, 128, 3, 1),    # 27 k-blocks (odd: the pipelined loop's tail), M = 81
])
@pytest.mark.parametrize("a_kind", [0, 1, 2])
def test_big_fwd_matches_generic(N, H, Cin, Cout, k, s, a_kind):
    """fwd, every ring depth / column tile: signed int8, offset int8 (sum_k W from the MFMA against
    ones, and from the caller's column sums), int16 codes (hi / lo' split)."""
    from lbt_amd import _lib
    from lbt_amd.dfxp import ops
    rng, ctx, (qx, qw, _), d, w_hwio, (wf, ksf), _, colsum = _setup(N, H, Cin, Cout, k, s, N * H + Cin + a_kind)
    if a_kind == 2:
        x = torch.from_numpy(rng.integers(-256, 256, size=(N, H, H, Cin)).astype(np.int16)).to(DEV)
        xg, signed9 = x, True
    else:
        x = torch.from_numpy(rng.integers(-128, 128, size=(N, H, H, Cin)).astype(np.int8)).to(DEV)
        xg, signed9 = (x.to(torch.int16) + 128, True) if a_kind == 1 else (x, False)
    ref = torch.empty((N, d.Ho, d.Wo, Cout), device=DEV)
    ops.conv_fwd_generic(xg, signed9, w_hwio, d, qx.desc, qw.desc, ref)
    for (stages, max_bn), halo in [(v, h) for v in VARIANTS for h in (0, 3)]:
        for cs in ((None, colsum) if a_kind == 1 else (None,)):
            y = torch.full_like(ref, float("nan"))
            n0 = _launches()
            with ops.igemm_forced(big=1, min_tiles=1, stages=stages, max_bn=max_bn, halo=halo):
                _lib.call("lbt_conv_fwd_igemm", _lib.ptr(x), a_kind, _lib.ptr(wf), ksf, _lib.ptr(cs), d, qx.desc,
                          qw.desc, _lib.ptr(y), _lib.stream())
            assert _launches() == n0 + 1, "the 256-row kernel did not run"
            assert torch.equal(y, ref), (stages, max_bn, halo, cs is not None)


@pytest.mark.parametrize("N,H,Cin,Cout,k", [
    (3, 14, 128, 64, 3),    # 3x3 dgrad, ncol = Cin = 128, M = 588
    (2, 15, 256, 128, 1),   # 1x1 dgrad, 256 output columns, M = 450
    (1, 9, 64, 192, 3),     # 27 k-blocks, M = 81
])
@pytest.mark.parametrize("g_i16", [0, 1])
@pytest.mark.parametrize("add", [False, True])
def test_big_dgrad_matches_generic(N, H, Cin, Cout, k, g_i16, add):
    """unit-stride dgrad (strided ones run as parity classes on the 128-row kernel), 8- and 16-bit
    gradient codes, with and without the residual addend, every ring depth / column tile."""
    from lbt_amd.dfxp import ops
    rng, ctx, (_, qw, qg), d, w_hwio, _, (wd, ksd), _ = _setup(N, H, Cin, Cout, k, 1, N * H + Cout + g_i16)
    if g_i16:
        g = torch.from_numpy(rng.integers(-32768, 32768, size=(N, d.Ho, d.Wo, Cout)).astype(np.int16)).to(DEV)
    else:
        g = torch.from_numpy(rng.integers(-128, 128, size=(N, d.Ho, d.Wo, Cout)).astype(np.int8)).to(DEV)
    addend = torch.from_numpy(rng.normal(size=(N, H, H, Cin)).astype(np.float32)).to(DEV) if add else None
    ref = torch.empty((N, H, H, Cin), device=DEV)
    (ops.conv_dgrad_generic16 if g_i16 else ops.conv_dgrad_generic)(g, w_hwio, d, qg.desc, qw.desc, ref)
    if add:
        ref = ref + addend
    for (stages, max_bn), halo in [(v, h) for v in VARIANTS for h in (0, 3)]:
        dx = torch.full_like(ref, float("nan"))
        n0 = _launches()
        with ops.igemm_forced(big=1, min_tiles=1, stages=stages, max_bn=max_bn, halo=halo):
            ops.conv_dgrad_igemm(g, g_i16, wd, ksd, d, qg.desc, qw.desc, dx, add_src=addend)
        assert _launches() == n0 + 1, "the 256-row kernel did not run"
        assert torch.equal(dx, ref), (stages, max_bn, halo)


@pytest.mark.parametrize("N,H,Cin,Cout,k", [(3, 14, 64, 128, 3), (2, 15, 128, 64, 1), (3, 14, 64, 256, 1)])
@pytest.mark.parametrize("a_kind", [0, 1])
@pytest.mark.parametrize("stochastic", [True, False])
def test_big_quantising_epilogue_matches_fwd_then_quantize(N, H, Cin, Cout, k, a_kind, stochastic):
    """lbt_conv_fwd_igemm_q on the 256-row kernel (Normalization_q's input quantiser on the MFMA
    accumulators, noise from the per-step table) == lbt_conv_fwd_igemm -> lbt_dfxp_quantize: the same
    int8 codes, overflow counters and exact channel sums (reference :291 then :584-588)."""
    from lbt_amd._lib import NSHARD, OUT_I8
    from lbt_amd.dfxp import ops
    rng, ctx, (qx, qw, _), d, w_hwio, (wf, ksf), _, _ = _setup(N, H, Cin, Cout, k, 1, N + H + Cout + a_kind)
    # a range that puts a few percent of the outputs past the clip (both counters non-zero)
    qo = ctx.quantizer("t/bnX", 8, 4, stochastic=stochastic)
    x = torch.from_numpy(rng.integers(-128, 128, size=(N, H, H, Cin)).astype(np.int8)).to(DEV)
    y = torch.empty((N, d.Ho, d.Wo, Cout), device=DEV)
    ops.conv_fwd_igemm(x, a_kind, wf, ksf, d, qx.desc, qw.desc, y)
    cs_ref = torch.zeros(NSHARD * 2 * Cout, dtype=torch.int64, device=DEV)
    ctx.counts.zero_()
    q_ref = ops.quantize(y, qo, OUT_I8, chsum=cs_ref, C=Cout)
    cnt_ref = ctx.counts_view()[qo.slot].sum(0).cpu()
    assert cnt_ref[0] > 0 and cnt_ref[1] > cnt_ref[0]
    # the quantising epilogue never takes the 256-column tile; fwdq_perm 1: the sample-blocked, LDS-staged
    # form (2 stages); 2 (the default): the same for these K > 64 shapes; 8: the persistent kernel on 8
    # workgroups, so every workgroup walks many tiles through its ring (3 and 4 stages); 0: quant_epilogue
    # on row-major tiles (every ring depth, halo on and off). The K = 64 shape (one k-block) takes the
    # persistent kernel at the default 2 as well.
    cases = [(v, h, 0) for v in VARIANTS[:-1] for h in (0, 3)] + [((2, mb), 0, 1) for mb in (64, 128)]
    cases += [((st, mb), 0, pp) for mb in (64, 128) for st, pp in ((2, 2), (3, 8), (4, 8))]
    for (stages, max_bn), halo, perm in cases:
        ctx.counts.zero_()
        cs = torch.zeros_like(cs_ref)
        yq = torch.full(q_ref.shape, 99, dtype=torch.int8, device=DEV)
        n0 = _launches()
        with ops.igemm_forced(big=1, min_tiles=1, stages=stages, max_bn=max_bn, halo=halo, fwdq_perm=perm):
            ops.conv_fwd_igemm_q(x, a_kind, wf, ksf, d, qx.desc, qw.desc, yq, qo, cs)
        assert _launches() == n0 + 1, "the 256-row kernel did not run"
        assert torch.equal(yq, q_ref), (stages, max_bn, halo, perm)
        assert torch.equal(ctx.counts_view()[qo.slot].sum(0).cpu(), cnt_ref), (stages, max_bn, halo, perm)
        assert torch.equal(cs.view(NSHARD, -1).sum(0), cs_ref.view(NSHARD, -1).sum(0)), (stages, max_bn, halo, perm)


@pytest.mark.parametrize("N,H,Cin,Cout,k", [
    (3, 14, 128, 64, 3),    # conv-2's dgrad shape (3x3), ncol = 128, M = 588 (ragged last tile)
    (2, 15, 64, 256, 1),    # conv-3's dgrad shape (1x1, K = 256), ncol = 64, M = 450
])
@pytest.mark.parametrize("stochastic", [True, False])
def test_big_dgrad_bna_matches_dgrad_then_pass_a(N, H, Cin, Cout, k, stochastic):
    """lbt_conv_dgrad_igemm_bna (ResidualBottleneck_q bn1 / bn2 pass A in the dgrad16 epilogue: ReLU mask
    from R, Rescale_q and Normalization_q gradient quantisers, noise from the per-step tables) ==
    lbt_conv_dgrad_igemm_ws -> lbt_bn_bwd_a_wide_masked(mask_r): the same G codes, channel sums and
    overflow counters, on every ring depth / column tile, and through the entry's own unfused fallback
    (reference Conv2d_q.backward :299-310, then ReLU_q, Rescale_q :686-691, Normalization_q :620-623)."""
    from lbt_amd._lib import NSHARD
    from lbt_amd.dfxp import ops
    rng, ctx, (_, qw, qg), d, _, _, (wd, ksd), _ = _setup(N, H, Cin, Cout, k, 1, N * H + Cin + int(stochastic))
    g = torch.from_numpy(rng.integers(-32768, 32768, size=(N, d.Ho, d.Wo, Cout)).astype(np.int16)).to(DEV)
    dx = torch.empty((N, H, H, Cin), device=DEV)
    ops.conv_dgrad_igemm(g, 1, wd, ksd, d, qg.desc, qw.desc, dx)
    # ranges that clip a few percent of both quantisers' inputs (every counter non-zero)
    top = int(np.ceil(np.log2(float(dx.abs().max())))) - 2
    qr = ctx.quantizer("t/rX", 8, 2)
    qrg = ctx.quantizer("t/rg", 16, top, stochastic=stochastic)
    qng = ctx.quantizer("t/ng", 16, top, stochastic=stochastic)
    R = torch.from_numpy(rng.integers(-128, 128, size=dx.shape).astype(np.int8)).to(DEV)
    qn = torch.from_numpy(rng.integers(-128, 128, size=dx.shape).astype(np.int8)).to(DEV)
    gb = torch.from_numpy(np.concatenate([rng.uniform(-2, 2, Cin), rng.uniform(-1, 1, Cin)]).astype(np.float32)).to(DEV)
    rows, inner = N * H * H, H * H * Cin

    def counts():
        v = ctx.counts_view()
        return torch.stack([v[qrg.slot].sum(0), v[qng.slot].sum(0)]).cpu()

    ctx.counts.zero_()
    G_ref = torch.empty(dx.shape, dtype=torch.int16, device=DEV)
    s_ref = torch.zeros(NSHARD * 4 * Cin, dtype=torch.int64, device=DEV)
    ops.bn_bwd_a_wide_masked(dx, None, True, qr.desc, gb, None, qrg.desc, R, qng.desc, qn, G_ref, s_ref, rows, inner,
                             Cin)
    c_ref = counts()
    assert (c_ref > 0).all(), c_ref
    s_ref = s_ref.view(NSHARD, -1).sum(0)
    # fwdq_perm 1 and 2 (the default): the LDS-staged pass-A epilogue; 8: the opt-in persistent kernel
    # on 8 workgroups (stochastic quantisers with tables; many tiles each)
    variants = [(1, st, mb, h, 1) for st, mb in VARIANTS if mb <= 128 for h in (0, 3)] + [(0, 2, 128, 0, 1)]
    variants += [(1, 2, 64, 0, 2), (1, 3, 64, 0, 8)]
    for big, stages, max_bn, halo, perm in variants:
        ctx.counts.zero_()
        G = torch.full_like(G_ref, 12345)
        sums = torch.zeros(NSHARD * 4 * Cin, dtype=torch.int64, device=DEV)
        scratch = torch.full_like(dx, float("nan"))
        n0 = _launches()
        with ops.igemm_forced(big=big, min_tiles=1, stages=stages, max_bn=max_bn, halo=halo, fwdq_perm=perm):
            ops.conv_dgrad_igemm_bna(g, wd, ksd, d, qg.desc, qw.desc, qr.desc, R, gb, qrg, qng, qn, G, sums, scratch,
                                     None)
        assert _launches() == n0 + big, "the 256-row kernel did not run"
        if big:
            assert torch.isnan(scratch).all(), "the fused path must not store dx"
        assert torch.equal(G, G_ref), (big, stages, max_bn, halo, perm)
        assert torch.equal(sums.view(NSHARD, -1).sum(0), s_ref), (big, stages, max_bn, halo, perm)
        assert torch.equal(counts(), c_ref), (big, stages, max_bn, halo, perm)


@pytest.mark.parametrize("N,H,Cin,Cout", [
    (3, 14, 256, 64),    # the next block's conv-1 (1x1, K = 64) into this block's 256-channel output, M = 588
    (2, 9, 128, 128),    # K = 128, ncol = 128, M = 162 (one partial tile)
])
@pytest.mark.parametrize("nbn,gmask", [(1, True), (2, False), (2, True)])
@pytest.mark.parametrize("stochastic", [True, False])
def test_big_dgrad_bn3_matches_dgrad_then_pass_a(N, H, Cin, Cout, nbn, gmask, stochastic):
    """lbt_conv_dgrad_igemm_bn3 (a bottleneck's entry: dx + g2, ReLU mask y_bits, the masked gradient
    optionally out, then pass A of bn3 and of the projection shortcut's BN in the dgrad16 epilogue) ==
    lbt_conv_dgrad_igemm_ws -> lbt_bn_bwd_a_wide_masked(g2, y_bits) per BN: the same G codes, masked
    gradient, channel sums and counters, on every ring depth / column tile and through the fallback
    (reference ResidualBlock_q.backward :865-869, ReLU_q, Rescale_q :686-691, Normalization_q :620-623)."""
    from lbt_amd._lib import NSHARD
    from lbt_amd.dfxp import ops
    rng, ctx, (_, qw, qg), d, _, _, (wd, ksd), _ = _setup(N, H, Cin, Cout, 1, 1,
                                                          N * H + Cin + nbn + 2 * int(gmask) + 4 * int(stochastic))
    g = torch.from_numpy(rng.integers(-32768, 32768, size=(N, H, H, Cout)).astype(np.int16)).to(DEV)
    shape = (N, H, H, Cin)
    dx = torch.empty(shape, device=DEV)
    ops.conv_dgrad_igemm(g, 1, wd, ksd, d, qg.desc, qw.desc, dx)
    g2 = torch.from_numpy(rng.normal(size=shape).astype(np.float32)).to(DEV) * dx.abs().mean()
    ybits = torch.from_numpy(rng.integers(0, 16, size=N * H * H * Cin // 4).astype(np.uint8)).to(DEV)
    top = int(np.ceil(np.log2(float((dx + g2).abs().max())))) - 2
    rows, inner = N * H * H, H * H * Cin
    bns = []
    for k in range(nbn):
        qrg = ctx.quantizer("t/rg%d" % k, 16, top - k, stochastic=stochastic)
        qng = ctx.quantizer("t/ng%d" % k, 16, top - k, stochastic=stochastic)
        R = torch.from_numpy(rng.integers(-128, 128, size=shape).astype(np.int8)).to(DEV)
        qn = torch.from_numpy(rng.integers(-128, 128, size=shape).astype(np.int8)).to(DEV)
        gam = torch.from_numpy(rng.uniform(-2, 2, 2 * Cin).astype(np.float32)).to(DEV)
        bns.append((R, gam, qrg, qng, qn))

    def counts():
        v = ctx.counts_view()
        return torch.stack([v[q.slot].sum(0) for b in bns for q in b[2:4]]).cpu()

    ctx.counts.zero_()
    ref_G, ref_s = [], []
    ref_m = torch.empty(shape, device=DEV) if gmask else None
    for k, (R, gam, qrg, qng, qn) in enumerate(bns):
        G = torch.empty(shape, dtype=torch.int16, device=DEV)
        sm = torch.zeros(NSHARD * 4 * Cin, dtype=torch.int64, device=DEV)
        ops.bn_bwd_a_wide_masked(dx, None, False, qrg.desc, gam, ref_m if k == 0 else None, qrg.desc, R, qng.desc, qn,
                                 G, sm, rows, inner, Cin, g2=g2, y_bits=ybits)
        ref_G.append(G)
        ref_s.append(sm.view(NSHARD, -1).sum(0))
    c_ref = counts()
    assert (c_ref > 0).all(), c_ref
    variants = [(1, st, mb) for st, mb in VARIANTS if mb <= 128] + [(0, 2, 128)]
    for big, stages, max_bn in variants:
        ctx.counts.zero_()
        outs = [(torch.full(shape, 12345, dtype=torch.int16, device=DEV),
                 torch.zeros(NSHARD * 4 * Cin, dtype=torch.int64, device=DEV)) for _ in bns]
        m = torch.full(shape, float("nan"), device=DEV) if gmask else None
        scratch = torch.full(shape, float("nan"), device=DEV)
        n0 = _launches()
        with ops.igemm_forced(big=big, min_tiles=1, stages=stages, max_bn=max_bn):
            ops.conv_dgrad_igemm_bn3(g, wd, ksd, d, qg.desc, qw.desc, g2, ybits, m,
                                     [b[:2] + b[2:4] + (b[4],) + o for b, o in zip(bns, outs)], scratch, None)
        assert _launches() == n0 + big, "the 256-row kernel did not run"
        if big:
            assert torch.isnan(scratch).all(), "the fused path must not store dx"
        for k in range(nbn):
            assert torch.equal(outs[k][0], ref_G[k]), (k, big, stages, max_bn)
            assert torch.equal(outs[k][1].view(NSHARD, -1).sum(0), ref_s[k]), (k, big, stages, max_bn)
        if gmask:
            assert torch.equal(m, ref_m), (big, stages, max_bn)
        assert torch.equal(counts(), c_ref), (big, stages, max_bn)


def test_bottleneck_takes_big_kernel_naturally_bitexact_vs_oracle():
    """A ResNet-50 configuration (one bottleneck per stage, width 64, 16-bit gradients, 224x224,
    B=17) whose stage-1 GEMMs have >= 200 256-row tiles, so the DEFAULT selection runs them on the
    256-row kernel (3x3 fwd with the quantising epilogue, 3x3 and 1x1 dgrad16): forward logits,
    every gradient and every exponent update bit-exact against the oracle."""
    from lbt_amd.dfxp import ops
    from lbt_amd.models import ImageNet_Resnet
    from lbt_amd.runtime import DfxpContext
    t = ops.igemm_tuning()
    assert t["big"] == 1 and t["min_tiles"] == 200, "run with the default selection"
    B, image, classes = 17, 224, 16
    ctx = DfxpContext(seed=1)
    gm = ImageNet_Resnet(8, (1, 1, 1, 1), grad_bits=16, width=64, classes=classes, image=image, ctx=ctx)
    om = oresnet.build_resnet50((1, 1, 1, 1), 64, classes, 8, 16)
    params = {}
    for owner, var, _ in gm.param_slots():
        params[owner.name + {"W": "/W", "gamma": "/g", "beta": "/b"}[var]] = getattr(owner, var).detach().cpu().numpy()
    oresnet.set_params(om, params)
    rng = np.random.default_rng(2)
    x = ((rng.integers(0, 256, size=(B, image, image, 3)) - 127.5) / 128).astype(np.float32)
    y = rng.integers(0, classes, size=B).astype(np.int32)
    octx = onn.Ctx(oresnet.init_ranges(om), 0, ctx.seed)
    n0 = _launches()
    logits = gm.forward(torch.from_numpy(x).to(DEV))
    gm.compute_loss(torch.from_numpy(y).to(DEV))
    dz = gm.dlogits.cpu().numpy()
    gm.backward()
    torch.cuda.synchronize()
    assert _launches() - n0 >= 3, "the default selection did not take the 256-row kernel"
    lr = om.forward(x, octx)
    assert np.array_equal(logits.cpu().numpy(), lr), "forward must be bit-exact"
    om.backward(dz, octx)
    og = oresnet.get_grads(om)
    for owner, var, gname in gm.param_slots():
        k = owner.name + {"W": "/W", "gamma": "/g", "beta": "/b"}[var]
        assert np.array_equal(getattr(owner, gname).detach().cpu().numpy(), og[k]), k
    ctx.update_range_op()
    assert ctx.ranges() == octx.new_ranges()
