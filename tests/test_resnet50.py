"""ResNet-50 (ResidualBottleneck_q, MaxPool_q) on ImageNet-shape inputs, with
8-bit and 16-bit gradient quantisers.

CPU: the oracle's MaxPoolQ against a direct loop restatement of tf.nn.max_pool and its gradient.
GPU: the HIP layer path against the oracle, bit-exact (forward logits, every gradient given the
same d loss / d logits, every exponent update), on reduced widths / depths so the numpy oracle
finishes in seconds; the full-size model through a training step (shape and finiteness checks).
"""
import contextlib
import os

import numpy as np
import pytest
import torch

from oracle import nn as onn
from oracle import resnet as oresnet

DEV = "cuda"
F32 = np.float32


@contextlib.contextmanager
def _env(name, value):
    """Set one environment variable for the block (launchers that read it per call)."""
    old = os.environ.get(name)
    os.environ[name] = value
    try:
        yield
    finally:
        if old is None:
            del os.environ[name]
        else:
            os.environ[name] = old


def _maxpool_loops(x, k, s, padding):
    N, H, W, C = x.shape
    Ho, Wo, pt, _, pl, _ = onn.conv_geometry(H, W, k, k, s, s, padding)
    y = np.zeros((N, Ho, Wo, C), F32)
    arg = np.zeros((N, Ho, Wo, C, 2), np.int64)
    for n in range(N):
        for oh in range(Ho):
            for ow in range(Wo):
                for c in range(C):
                    best, bi = -np.inf, None
                    for i in range(k):
                        for j in range(k):
                            ih, iw = oh * s + i - pt, ow * s + j - pl
                            if 0 <= ih < H and 0 <= iw < W and x[n, ih, iw, c] > best:
                                best, bi = x[n, ih, iw, c], (ih, iw)
                    y[n, oh, ow, c] = best
                    arg[n, oh, ow, c] = bi
    return y, arg


def test_oracle_maxpool_matches_loops():
    rng = np.random.default_rng(0)
    # ReLU-like input: many exact ties at 0 exercise the first-maximum rule
    x = np.maximum(rng.normal(size=(2, 7, 6, 3)), 0).astype(F32)
    g = rng.normal(size=(2, 4, 3, 3)).astype(F32)
    mp = onn.MaxPoolQ([1, 3, 3, 1], [1, 2, 2, 1], "SAME")
    y = mp.forward(x, None)
    yl, arg = _maxpool_loops(x, 3, 2, "SAME")
    assert np.array_equal(y, yl)
    dx = mp.backward(g, None)
    want = np.zeros_like(x)
    for n in range(2):
        for oh in range(4):
            for ow in range(3):
                for c in range(3):
                    ih, iw = arg[n, oh, ow, c]
                    want[n, ih, iw, c] = F32(want[n, ih, iw, c] + g[n, oh, ow, c])
    assert np.array_equal(dx, want)


def _pair(blocks, width, classes, image, grad_bits, seed=0):
    from lbt_amd.models import ImageNet_Resnet
    from lbt_amd.runtime import DfxpContext
    ctx = DfxpContext(seed=seed)
    gm = ImageNet_Resnet(8, blocks, grad_bits=grad_bits, width=width, classes=classes, image=image, ctx=ctx)
    om = oresnet.build_resnet50(blocks, width, classes, 8, grad_bits)
    return ctx, gm, om


def _params(gm):
    out = {}
    for owner, var, _ in gm.param_slots():
        out[owner.name + {"W": "/W", "gamma": "/g", "beta": "/b"}[var]] = getattr(owner, var).detach().cpu().numpy()
    return out


def _grads(gm):
    out = {}
    for owner, var, gname in gm.param_slots():
        out[owner.name + {"W": "/W", "gamma": "/g", "beta": "/b"}[var]] = getattr(owner, gname).detach().cpu().numpy()
    return out


def _batch(B, image, classes, seed):
    rng = np.random.default_rng(seed)
    x = ((rng.integers(0, 256, size=(B, image, image, 3)) - 127.5) / 128).astype(F32)
    return x, rng.integers(0, classes, size=B).astype(np.int32)


@pytest.mark.gpu
@pytest.mark.parametrize("grad_bits", [8, 16])
@pytest.mark.parametrize("blocks,width,image,classes", [((1, 1, 1, 1), 8, 32, 10), ((2, 1, 1, 1), 16, 40, 10),
                                                        ((1, 1, 1, 1), 8, 32, 16), ((2, 1, 1, 1), 64, 32, 16),
                                                        ((3, 2, 1, 1), 64, 40, 16), ((3, 4, 6, 3), 64, 56, 16),
                                                        ((3, 4, 6, 3), 64, 224, 1000)])
def test_resnet50_layers_bitexact_vs_oracle(blocks, width, image, classes, grad_bits):
    """classes=16: the fc runs on the int8-MFMA dense kernels (dense.hip), 10: the generic ones.
    width 64 with 16-bit gradients: every bottleneck runs fused (ResidualBottleneck_q._fusable).
    (3, 4, 6, 3) at width 64: the benched ResNet-50's depth and widths (stage 3's six-block chain, the
    2048-channel last stage), at 56x56 and at the benched 224x224 / 1000 classes (configs[3] itself, at
    B=4 instead of 256: the oracle takes seconds per image)."""
    from lbt_amd.dfxp.layers import ResidualBottleneck_q
    ctx, gm, om = _pair(blocks, width, classes, image, grad_bits, seed=1)
    assert gm.layers[-1].mfma == (classes % 8 == 0)
    blocks_ = [l for l in gm.layers if isinstance(l, ResidualBottleneck_q)]
    if width % 64 == 0:
        assert all(b._fusable() == (grad_bits > 8) for b in blocks_)
    oresnet.set_params(om, _params(gm))
    x, y = _batch(4, image, classes, seed=2)
    octx = onn.Ctx(oresnet.init_ranges(om), 0, ctx.seed)
    logits = gm.forward(torch.from_numpy(x).to(DEV))
    lr = om.forward(x, octx)
    assert np.array_equal(logits.cpu().numpy(), lr), "forward must be bit-exact"
    gm.compute_loss(torch.from_numpy(y).to(DEV))
    dz = gm.dlogits.cpu().numpy()
    gm.backward()
    om.backward(dz, octx)
    gg, og = _grads(gm), oresnet.get_grads(om)
    assert gg.keys() == og.keys()
    for k in gg:
        assert np.array_equal(gg[k], og[k]), k
    ctx.update_range_op()
    assert ctx.ranges() == octx.new_ranges()


@pytest.mark.gpu
@pytest.mark.parametrize("blocks,width,image,classes,grad_bits", [((1, 1, 1, 1), 8, 32, 10, 8),
                                                                  ((3, 2, 1, 1), 64, 40, 16, 16)])
def test_resnet50_deferred_reductions_bitexact(blocks, width, image, classes, grad_bits, monkeypatch):
    """The Trainer's backward scope (ops.deferred_reductions): every conv's slab reduce in one
    lbt_conv_wgrad_reduce64_many launch and every BN's dgamma / dbeta in one lbt_bn_param_grads_many
    launch at the end of the backward, equal to the oracle's."""
    from lbt_amd.dfxp import ops
    monkeypatch.setenv("LBT_BATCH_WREDUCE", "1")  # (off by default: measured slower, ops.py)
    ctx, gm, om = _pair(blocks, width, classes, image, grad_bits, seed=3)
    oresnet.set_params(om, _params(gm))
    x, y = _batch(4, image, classes, seed=4)
    octx = onn.Ctx(oresnet.init_ranges(om), 0, ctx.seed)
    gm.forward(torch.from_numpy(x).to(DEV))
    om.forward(x, octx)
    gm.compute_loss(torch.from_numpy(y).to(DEV))
    dz = gm.dlogits.cpu().numpy()
    for owner, _, gname in gm.param_slots():  # stale values must not survive
        getattr(owner, gname).fill_(float("nan"))
    with ops.deferred_reductions() as scope:
        gm.backward()
    assert scope.own_p and scope.own_r
    om.backward(dz, octx)
    gg, og = _grads(gm), oresnet.get_grads(om)
    for k in gg:
        assert np.array_equal(gg[k], og[k]), k


@pytest.mark.gpu
def test_resnet50_full_size_step():
    """The real ResNet-50 (224x224, 1000 classes, [3,4,6,3]) through one graph-captured training
    step with 16-bit gradients: finite loss, every gradient finite, exponents updated."""
    from lbt_amd.models import ImageNet_Resnet50
    from lbt_amd.runtime import DfxpContext
    from lbt_amd.trainer import Trainer
    ctx = DfxpContext(seed=0)
    m = ImageNet_Resnet50(8, grad_bits=16, weight_decay=1e-4, ctx=ctx)
    t = Trainer(m, lr=0.01, momentum=0.9, use_graph=True)
    x, y = _batch(2, 224, 1000, seed=3)
    for _ in range(2):
        loss = t.step(torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV))
    torch.cuda.synchronize()
    assert np.isfinite(loss.item())
    assert torch.isfinite(t.flat.g).all() and torch.isfinite(t.flat.w).all()
    assert int(ctx.step.item()) == 2


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,Cin,Cout,k,s,akind", [
    (2, 14, 64, 128, 3, 1, 2), (2, 15, 128, 64, 3, 2, 2), (3, 7, 256, 160, 1, 1, 0), (2, 8, 64, 2048, 1, 2, 1),
    (1, 9, 192, 48, 3, 2, 0)])
def test_igemm_matches_generic(N, H, Cin, Cout, k, s, akind):
    """The LDS-tiled MFMA implicit GEMM (fwd: int8 / offset int8 / int16 codes; dgrad: int8 and
    int16 gradient codes) == the generic VALU kernels, bit for bit, incl. ragged tiles and stride 2."""
    from lbt_amd import _lib
    from lbt_amd.dfxp import ops
    from lbt_amd.runtime import DfxpContext
    rng = np.random.default_rng(N * H + Cin)
    ctx = DfxpContext(seed=0)
    qx, qw, qg = ctx.quantizer("t/X", 9, 2), ctx.quantizer("t/W", 8, 0), ctx.quantizer("t/g", 16, -3)
    d = ops.conv_desc(N, H, H, Cin, Cout, k, k, s, s, "SAME")
    W = torch.from_numpy(rng.uniform(-1, 1, size=(k, k, Cin, Cout)).astype(np.float32)).to(DEV)
    w_hwio = torch.empty((k, k, Cin, Cout), dtype=torch.int8, device=DEV)
    ksf, ksd = ops.packed_slices(k, k, Cin), ops.packed_slices(k, k, Cout)
    wf = torch.zeros((Cout, ksf * 16), dtype=torch.int8, device=DEV)
    wd = torch.zeros((Cin, ksd * 16), dtype=torch.int8, device=DEV)
    ops.quantize_weight(W, qw, w_hwio=w_hwio, wf=wf, ksf=ksf, wd=wd, ksd=ksd)
    # forward
    if akind == 2:
        x = torch.from_numpy(rng.integers(-256, 256, size=(N, H, H, Cin)).astype(np.int16)).to(DEV)
    else:
        x = torch.from_numpy(rng.integers(-128, 128, size=(N, H, H, Cin)).astype(np.int8)).to(DEV)
    y1 = torch.empty((N, d.Ho, d.Wo, Cout), device=DEV)
    y2 = torch.empty_like(y1)
    ops.conv_fwd_igemm(x, akind, wf, ksf, d, qx.desc, qw.desc, y1)
    if akind == 1:  # offset codes q - 128: the generic kernel takes the codes themselves (int16)
        ops.conv_fwd_generic(x.to(torch.int16) + 128, True, w_hwio, d, qx.desc, qw.desc, y2)
    else:
        ops.conv_fwd_generic(x, akind == 2, w_hwio, d, qx.desc, qw.desc, y2)
    assert torch.equal(y1, y2)
    # input gradient, 8- and 16-bit codes (gathered side = Cout: multiples of 64 only)
    for g_i16 in ((0, 1) if Cout % 64 == 0 else ()):
        if g_i16:
            g = torch.from_numpy(rng.integers(-32768, 32768, size=(N, d.Ho, d.Wo, Cout)).astype(np.int16)).to(DEV)
        else:
            g = torch.from_numpy(rng.integers(-128, 128, size=(N, d.Ho, d.Wo, Cout)).astype(np.int8)).to(DEV)
        dx1 = torch.empty((N, H, H, Cin), device=DEV)
        dx2 = torch.empty_like(dx1)
        ops.conv_dgrad_igemm(g, g_i16, wd, ksd, d, qg.desc, qw.desc, dx1)
        if g_i16:
            ops.conv_dgrad_generic16(g, w_hwio, d, qg.desc, qw.desc, dx2)
        else:
            ops.conv_dgrad_generic(g, w_hwio, d, qg.desc, qw.desc, dx2)
        assert torch.equal(dx1, dx2), g_i16


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,Cin,Cout,k,s", [(2, 14, 64, 64, 3, 1), (2, 15, 128, 64, 3, 2), (3, 7, 64, 192, 1, 1),
                                              (1, 16, 64, 128, 1, 2)])
def test_wgrad_igemm_matches_generic(N, H, Cin, Cout, k, s):
    """Wide-layer MFMA weight gradient (offset int8 x; int8 and int16 g) == the generic kernels'
    exact integer sums."""
    from lbt_amd.dfxp import ops
    rng = np.random.default_rng(N + H + Cin + Cout)
    d = ops.conv_desc(N, H, H, Cin, Cout, k, k, s, s, "SAME")
    K = k * k * Cin
    x = rng.integers(0, 256, size=(N, H, H, Cin))
    x_off = torch.from_numpy((x - 128).astype(np.int8)).to(DEV)
    x16 = torch.from_numpy(x.astype(np.int16)).to(DEV)
    for g_i16 in (0, 1):
        if g_i16:
            g = torch.from_numpy(rng.integers(-32768, 32768, size=(N, d.Ho, d.Wo, Cout)).astype(np.int16)).to(DEV)
        else:
            g = torch.from_numpy(rng.integers(-128, 128, size=(N, d.Ho, d.Wo, Cout)).astype(np.int8)).to(DEV)
        nsplit = ops.wgrad_igemm_nsplit(d)
        slab = torch.zeros((2, K, Cout), dtype=torch.int64, device=DEV)
        ops.conv_wgrad_igemm(x_off, g, g_i16, d, slab, nsplit, min(2, nsplit))
        got = slab.sum(0)
        ns = ops.wgrad_nsplit(d, generic=True)
        if g_i16:
            ref = torch.zeros((ns, K, Cout), dtype=torch.int64, device=DEV)
            ops.conv_wgrad_generic16(x16, True, g, d, ref, ns)
        else:
            ref = torch.zeros((ns, K, Cout), dtype=torch.int32, device=DEV)
            ops.conv_wgrad_generic(x16, True, g, d, ref, ns)
        assert torch.equal(got, ref.to(torch.int64).sum(0)), g_i16
        ns2 = ops.wgrad_store_nsplit(d, g_i16)
        slab2 = torch.full((ns2, K, Cout), 3, dtype=torch.int64, device=DEV)  # every element overwritten
        ops.conv_wgrad_igemm_store(x_off, g, g_i16, d, slab2, ns2)
        assert torch.equal(slab2.sum(0), ref.to(torch.int64).sum(0)), ("store", g_i16)


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,Cout,k,s", [(2, 32, 64, 7, 2), (1, 40, 16, 7, 2), (2, 23, 48, 5, 1), (1, 224, 64, 7, 2),
                                          (3, 17, 32, 3, 2), (1, 230, 64, 7, 2), (1, 36, 128, 7, 2)])
def test_stem_wide_matches_generic(N, H, Cout, k, s):
    """The ImageNet conv1 on fp16 MFMA (stem_wide.hip: signed 9-bit image codes, K = k*k*3 patch
    elements; 8- and 16-bit gradient codes split hi/lo) == the generic VALU kernels' exact integer
    results, bit for bit, incl. ragged pixel tiles and SAME padding at both strides."""
    from lbt_amd.dfxp import ops
    from lbt_amd.runtime import DfxpContext
    rng = np.random.default_rng(N * H + Cout + k)
    ctx = DfxpContext(seed=0)
    qx, qw, qg = ctx.quantizer("t/X", 9, 2), ctx.quantizer("t/W", 8, 0), ctx.quantizer("t/g", 16, -3)
    d = ops.conv_desc(N, H, H, 3, Cout, k, k, s, s, "SAME")
    assert ops.stem_wide_ok(d, 9, 8)
    K = k * k * 3
    W = torch.from_numpy(rng.uniform(-1, 1, size=(k, k, 3, Cout)).astype(np.float32)).to(DEV)
    w_hwio = torch.empty((k, k, 3, Cout), dtype=torch.int8, device=DEV)
    ops.quantize_weight(W, qw, w_hwio=w_hwio)
    x = torch.from_numpy(rng.integers(-256, 256, size=(N, H, H, 3)).astype(np.int16)).to(DEV)
    y1 = torch.empty((N, d.Ho, d.Wo, Cout), device=DEV)
    y2 = torch.empty_like(y1)
    ops.conv_fwd_generic(x, True, w_hwio, d, qx.desc, qw.desc, y2)
    # the row-tile forward (LDS image rows, default) and the per-element gather kernel
    for tiles in ("1", "0"):
        with _env("LBT_STEM_WIDE_TILES", tiles):
            y1.fill_(float("nan"))
            ops.conv_stem_wide_fwd(x, w_hwio, d, qx.desc, qw.desc, y1)
        assert torch.equal(y1, y2), tiles
    for g_i16 in (0, 1):
        if g_i16:
            g = torch.from_numpy(rng.integers(-32768, 32768, size=(N, d.Ho, d.Wo, Cout)).astype(np.int16)).to(DEV)
        else:
            g = torch.from_numpy(rng.integers(-128, 128, size=(N, d.Ho, d.Wo, Cout)).astype(np.int8)).to(DEV)
        nr = ops.wgrad_nsplit(d, generic=True)
        if g_i16:
            ref = torch.zeros((nr, K, Cout), dtype=torch.int64, device=DEV)
            ops.conv_wgrad_generic16(x, True, g, d, ref, nr)
        else:
            ref = torch.zeros((nr, K, Cout), dtype=torch.int32, device=DEV)
            ops.conv_wgrad_generic(x, True, g, d, ref, nr)
        ns = ops.stem_wide_nsplit(d)
        # the row-chunk kernel (LDS window, default) and the per-element gather kernel (LBT_STEM_ROWS=0)
        for rows in ("1", "0"):
            old = os.environ.get("LBT_STEM_ROWS")
            os.environ["LBT_STEM_ROWS"] = rows
            try:
                slab = torch.full((ns, K, Cout), 7, dtype=torch.int64, device=DEV)  # fully overwritten
                ops.conv_stem_wide_wgrad(x, 9, g, d, slab, ns)
            finally:
                if old is None:
                    del os.environ["LBT_STEM_ROWS"]
                else:
                    os.environ["LBT_STEM_ROWS"] = old
            assert torch.equal(slab.sum(0), ref.to(torch.int64).sum(0)), (g_i16, rows)


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,C", [(2, 112, 64), (3, 17, 8)])
def test_maxpool_relu_mask_in_argmax(N, H, C):
    """lbt_maxpool_relu_fwd's argmax codes carry the ReLU mask (255: route nothing), so
    lbt_maxpool_relu_bwd without y == with y == relu_bwd(maxpool_bwd(g)) of the torch reference
    (3x3 / 2 SAME, a third of the inputs <= 0 and whole windows <= 0), bit for bit."""
    from lbt_amd.dfxp import ops
    rng = np.random.default_rng(N * H + C)
    d = ops.conv_desc(N, H, H, C, C, 3, 3, 2, 2, "SAME")
    xn = rng.standard_normal((N, H, H, C)).astype(np.float32) - 0.5
    xn[:, : H // 3] = -np.abs(xn[:, : H // 3])  # whole windows with max <= 0
    x = torch.from_numpy(xn).to(DEV).requires_grad_(True)
    y = torch.empty((N, d.Ho, d.Wo, C), device=DEV)
    amax = torch.empty((N, d.Ho, d.Wo, C), dtype=torch.uint8, device=DEV)
    ops.maxpool_relu_fwd(x.detach(), y, amax, d)
    assert int((amax == 255).sum()) > 0
    g = torch.from_numpy(rng.standard_normal((N, d.Ho, d.Wo, C)).astype(np.float32)).to(DEV)
    dx1, dx2 = torch.empty_like(x), torch.empty_like(x)
    ops.maxpool_relu_bwd(g, amax, y, dx1, d)
    ops.maxpool_relu_bwd(g, amax, None, dx2, d)
    assert torch.equal(dx1, dx2)
    # torch: relu then max pool (SAME 3x3/2 on even H pads bottom/right only; -inf padding)
    xr = torch.relu(x).permute(0, 3, 1, 2)
    pt, pb, pl, pr = d.PT, d.PB, d.PL, d.PR
    yr = torch.nn.functional.max_pool2d(torch.nn.functional.pad(xr, (pl, pr, pt, pb), value=-float("inf")), 3, 2)
    assert torch.equal(yr.permute(0, 2, 3, 1).detach(), y)
    # gradient routing against torch's relu + max-pool backward (fp32; an element that is the maximum of
    # several windows sums their gradients, possibly in another order: 1e-6)
    (yr.permute(0, 2, 3, 1) * g).sum().backward()
    assert torch.allclose(dx1, x.grad, rtol=1e-6, atol=1e-6)
    assert torch.all(dx1[x.detach() <= 0] == 0)


@pytest.mark.gpu
@pytest.mark.parametrize("N,IN,OUT", [(32, 2048, 1000), (3, 128, 40), (17, 64, 8)])
def test_dense_mfma_matches_generic(N, IN, OUT):
    """Dense_q on int8 MFMA (fwd; dgrad with int8 and hi/lo-split int16 gradient codes) and the
    fused-reduce VALU wgrad == the generic kernels + reduce, bit for bit."""
    from lbt_amd import _lib
    from lbt_amd.dfxp import ops
    from lbt_amd.runtime import DfxpContext
    rng = np.random.default_rng(N + IN + OUT)
    ctx = DfxpContext(seed=0)
    qx, qw, qg = ctx.quantizer("t/X", 8, 2), ctx.quantizer("t/W", 8, 0), ctx.quantizer("t/g", 16, -3)
    d = _lib.ConvDesc(N, 1, 1, IN, OUT, 1, 1, 1, 1, 0, 0, 0, 0, 1, 1)
    W = torch.from_numpy(rng.uniform(-1, 1, size=(IN, OUT)).astype(np.float32)).to(DEV)
    w_hwio = torch.empty((IN, OUT), dtype=torch.int8, device=DEV)
    ops.quantize_weight(W, qw, w_hwio=w_hwio)
    wf = torch.full((OUT, -(-IN // 64) * 64), 5, dtype=torch.int8, device=DEV)
    wd = torch.full((IN, -(-OUT // 64) * 64), 5, dtype=torch.int8, device=DEV)
    ops.dense_pack(w_hwio, wf, wd)
    x = torch.from_numpy(rng.integers(-128, 128, size=(N, IN)).astype(np.int8)).to(DEV)
    y1, y2 = torch.empty((N, OUT), device=DEV), torch.empty((N, OUT), device=DEV)
    ops.dense_gemm(x, wf, IN, qx.desc, qw.desc, y1)
    ops.conv_fwd_generic(x, False, w_hwio, d, qx.desc, qw.desc, y2)
    assert torch.equal(y1, y2)
    wd2 = ops.f32(2 * 1e-4)
    for g16 in (0, 1):
        if g16:
            g = torch.from_numpy(rng.integers(-32768, 32768, size=(N, OUT)).astype(np.int16)).to(DEV)
        else:
            g = torch.from_numpy(rng.integers(-128, 128, size=(N, OUT)).astype(np.int8)).to(DEV)
        dx1, dx2 = torch.empty((N, IN), device=DEV), torch.empty((N, IN), device=DEV)
        ops.dense_gemm(g, wd, OUT, qg.desc, qw.desc, dx1)
        (ops.conv_dgrad_generic16 if g16 else ops.conv_dgrad_generic)(g, w_hwio, d, qg.desc, qw.desc, dx2)
        assert torch.equal(dx1, dx2), g16
        dw1, dw2 = torch.empty_like(W), torch.empty_like(W)
        ops.dense_wgrad(x, g, qx.desc, qg.desc, W, wd2, dw1)
        ns = ops.wgrad_nsplit(d, generic=True)
        slab = torch.zeros((ns, IN, OUT), dtype=torch.int64 if g16 else torch.int32, device=DEV)
        if g16:
            ops.conv_wgrad_generic16(x, False, g, d, slab, ns)
            ops.conv_wgrad_reduce64(slab, ns, IN, OUT, qx.desc, qg.desc, W, wd2, dw2)
        else:
            ops.conv_wgrad_generic(x, False, g, d, slab, ns)
            ops.conv_wgrad_reduce(slab, ns, IN, OUT, 0, None, qx.desc, qg.desc, W, wd2, dw2)
        assert torch.equal(dw1, dw2), g16


@pytest.mark.gpu
@pytest.mark.parametrize("K", [1000, 1024, 1500])
def test_softmax_xent_wide(K):
    """The wide-K softmax-CE (one wave per row) against float64 numpy: loss and d loss / d z (K <= 1024:
    the row held in registers; 1500: the looped form). Bit-exactness against the oracle's softmax is
    test_resnet50_layers_bitexact_vs_oracle's 1000-class case."""
    from lbt_amd.dfxp import ops
    rng = np.random.default_rng(5)
    z = (rng.normal(size=(32, K)) * 4).astype(np.float32)
    y = rng.integers(0, K, size=32).astype(np.int32)
    loss = torch.empty(1, device=DEV)
    dz = torch.empty((32, K), device=DEV)
    ops.softmax_xent(torch.from_numpy(z).to(DEV), torch.from_numpy(y).to(DEV), loss, dz)
    zd = z.astype(np.float64)
    m = zd.max(1, keepdims=True)
    p = np.exp(zd - m) / np.exp(zd - m).sum(1, keepdims=True)
    want_loss = np.mean(-np.log(p[np.arange(32), y]))
    onehot = np.zeros_like(p)
    onehot[np.arange(32), y] = 1
    assert abs(loss.item() - want_loss) <= 1e-5 * abs(want_loss)
    assert np.allclose(dz.cpu().numpy(), (p - onehot) / 32, rtol=1e-5, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,Cin,Cout,k", [(2, 7, 512, 512, 3), (4, 7, 1024, 1024, 1), (1, 14, 256, 256, 3)])
def test_igemm_splitk_matches_generic(N, H, Cin, Cout, k):
    """Short-M / long-K wide GEMMs split K over workgroups (exact int32 partials + reduce): fwd with
    offset int8 codes, dgrad with int16 codes and the addend, bit-identical to the generic kernels."""
    from lbt_amd.dfxp import ops
    from lbt_amd.runtime import DfxpContext
    rng = np.random.default_rng(N * H + Cin + Cout)
    ctx = DfxpContext(seed=0)
    qx, qw, qg = ctx.quantizer("t/X", 9, 2), ctx.quantizer("t/W", 8, 0), ctx.quantizer("t/g", 16, -3)
    d = ops.conv_desc(N, H, H, Cin, Cout, k, k, 1, 1, "SAME")
    assert ops.igemm_workspace_bytes(d, 0, False) > 0 and ops.igemm_workspace_bytes(d, 1, True) > 0
    W = torch.from_numpy(rng.uniform(-1, 1, size=(k, k, Cin, Cout)).astype(np.float32)).to(DEV)
    w_hwio = torch.empty((k, k, Cin, Cout), dtype=torch.int8, device=DEV)
    ksf, ksd = ops.packed_slices(k, k, Cin), ops.packed_slices(k, k, Cout)
    wf = torch.zeros((Cout, ksf * 16), dtype=torch.int8, device=DEV)
    wd = torch.zeros((Cin, ksd * 16), dtype=torch.int8, device=DEV)
    ops.quantize_weight(W, qw, w_hwio=w_hwio, wf=wf, ksf=ksf, wd=wd, ksd=ksd)
    x = rng.integers(0, 256, size=(N, H, H, Cin))
    x_off = torch.from_numpy((x - 128).astype(np.int8)).to(DEV)
    ws = torch.empty(ops.igemm_workspace_bytes(d, 0, False) // 4, dtype=torch.int32, device=DEV)
    y1, y2 = torch.empty((N, H, H, Cout), device=DEV), torch.empty((N, H, H, Cout), device=DEV)
    ops.conv_fwd_igemm_ws(x_off, 1, wf, ksf, d, qx.desc, qw.desc, y1, ws)
    ops.conv_fwd_generic(torch.from_numpy(x.astype(np.int16)).to(DEV), True, w_hwio, d, qx.desc, qw.desc, y2)
    assert torch.equal(y1, y2)
    g = torch.from_numpy(rng.integers(-32768, 32768, size=(N, H, H, Cout)).astype(np.int16)).to(DEV)
    add = torch.from_numpy(rng.normal(size=(N, H, H, Cin)).astype(np.float32)).to(DEV)
    ws2 = torch.empty(ops.igemm_workspace_bytes(d, 1, True) // 4, dtype=torch.int32, device=DEV)
    dx1, dx2 = torch.empty((N, H, H, Cin), device=DEV), torch.empty((N, H, H, Cin), device=DEV)
    ops.conv_dgrad_igemm_ws(g, 1, wd, ksd, d, qg.desc, qw.desc, dx1, ws2, add_src=add)
    ops.conv_dgrad_generic16(g, w_hwio, d, qg.desc, qw.desc, dx2)
    assert torch.equal(dx1, dx2 + add)


@pytest.mark.gpu
def test_resnet50_fused_conv_quant_epilogue_bitexact(monkeypatch):
    """The opt-in quantising igemm epilogue (LBT_FUSE_CONV_QUANT=1: Normalization_q's input
    quantiser on the MFMA accumulators, in-register Philox exchange, exact channel sums) keeps
    the fused bottleneck bit-exact against the oracle."""
    monkeypatch.setenv("LBT_FUSE_CONV_QUANT", "1")
    test_resnet50_layers_bitexact_vs_oracle((1, 1, 1, 1), 64, 32, 16, 16)


@pytest.mark.gpu
def test_resnet50_fp32_ymask_path_bitexact(monkeypatch):
    """LBT_YBITS=0: the fused bottleneck's last pass A reads the fp32 block output as its ReLU mask
    instead of the chain's one-byte-per-channel-quad ybits; both forms bit-exact against the oracle
    (the default run of test_resnet50_layers_bitexact_vs_oracle covers ybits)."""
    monkeypatch.setenv("LBT_YBITS", "0")
    test_resnet50_layers_bitexact_vs_oracle((2, 1, 1, 1), 64, 32, 16, 16)
    test_resnet50_layers_bitexact_vs_oracle((2, 2, 1, 1), 64, 32, 16, 16)


@pytest.mark.gpu
def test_side_stream_schedule_bitidentical_under_graph_capture():
    """The backward's weight / BN-parameter gradients on a side stream (layers.SIDE_STREAM) at a size
    where the two streams really overlap (width 64, 16-bit gradients: every bottleneck fused; batch 16
    at 96x96), three graph-captured Trainer steps: gradients, weights and exponents are bit-identical
    to the one-stream schedule (a missing cross-stream dependency would show up here)."""
    from lbt_amd.dfxp import layers
    from lbt_amd.models import ImageNet_Resnet
    from lbt_amd.runtime import DfxpContext
    from lbt_amd.trainer import Trainer
    xs = [_batch(16, 96, 16, seed=10 + i) for i in range(3)]
    out = []
    saved = layers.SIDE_STREAM
    try:
        for side in (True, False):
            layers.SIDE_STREAM = side
            ctx = DfxpContext(seed=4)
            m = ImageNet_Resnet(8, (2, 1, 1, 1), grad_bits=16, width=64, classes=16, image=96, ctx=ctx)
            t = Trainer(m, lr=0.01, momentum=0.9, use_graph=True)
            for x, y in xs:
                t.step(torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV))
            torch.cuda.synchronize()
            out.append((t.flat.g.cpu().clone(), t.flat.w.cpu().clone(), ctx.exps.cpu().clone()))
    finally:
        layers.SIDE_STREAM = saved
    (ga, wa, ea), (gb, wb, eb) = out
    assert torch.equal(ga, gb) and torch.equal(wa, wb) and torch.equal(ea, eb)


@pytest.mark.gpu
def test_bottleneck_backward_called_directly_joins_side_stream():
    """The Layer_q contract: a fused bottleneck's backward called on its own (not inside
    Model.backward) returns with its dW / dgamma / dbeta finished on the caller's stream."""
    from lbt_amd.dfxp import layers
    from lbt_amd.runtime import DfxpContext
    ctx = DfxpContext(seed=6)
    blk = layers.ResidualBottleneck_q("blk", 8, 256, 64, 1, grad_bits=16, weight_decay=1e-4, ctx=ctx)
    assert blk._fusable()
    rng = np.random.default_rng(6)
    x = torch.from_numpy(np.maximum(rng.normal(size=(8, 28, 28, 256)), 0).astype(F32)).to(DEV)
    g = torch.from_numpy((rng.normal(size=(8, 28, 28, 256)) * 1e-3).astype(F32)).to(DEV)
    saved = layers.SIDE_STREAM
    res = []
    try:
        for side in (True, False):
            layers.SIDE_STREAM = side
            blk.forward(x)
            blk.backward(g)
            # read on the caller's stream with no synchronisation of our own
            c1 = blk.residual.layers[0]
            res.append((c1.dW.clone(), blk.residual.layers[1].layers[1].dgamma.clone()))
            torch.cuda.synchronize()
            ctx.counts.zero_()
    finally:
        layers.SIDE_STREAM = saved
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
