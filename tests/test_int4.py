"""SURVEY 8(f) rank 2 / BASELINE configs[4]: 4-bit weights, 8-bit activations and gradients.

The weight quantisers run at 4 bits (codes in [-8, 7]); the int8-MFMA conv kernels read the weight
images packed two codes per byte and unpack them in registers (gfx950 has no int4 MFMA). Checked
against the oracle with weight_bits = 4, bit-exact, through the whole ResNet-20 forward/backward.
"""
import numpy as np
import pytest
import torch

from oracle import nn as onn
from oracle import resnet as oresnet

DEV = "cuda"


@pytest.mark.gpu
def test_pack_int4_layout():
    from lbt_amd.dfxp import ops
    codes = torch.arange(-8, 8, dtype=torch.int8, device=DEV).repeat(4)
    packed = torch.empty(codes.numel() // 2, dtype=torch.uint8, device=DEV)
    ops.pack_int4(codes, packed)
    c = codes.cpu().numpy().astype(np.int64)
    want = ((c[0::2] & 15) | ((c[1::2] & 15) << 4)).astype(np.uint8)
    assert np.array_equal(packed.cpu().numpy(), want)


@pytest.mark.gpu
@pytest.mark.parametrize("B", [8, 32])
def test_resnet20_w4_bitexact_vs_oracle(B):
    from lbt_amd.models import CIFAR10_Resnet20
    from lbt_amd.runtime import DfxpContext
    ctx = DfxpContext(seed=4)
    gm = CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctx, weight_bits=4)
    assert all(c.w4 for c in _convs(gm) if c.mfma)
    om = oresnet.build_resnet((3, 3, 3), 8, 2e-4, weight_bits=4)
    params = {}
    for owner, var, _ in gm.param_slots():
        params[owner.name + {"W": "/W", "gamma": "/g", "beta": "/b"}[var]] = getattr(owner, var).cpu().numpy()
    oresnet.set_params(om, params)
    rng = np.random.default_rng(B)
    x = ((rng.integers(0, 256, size=(B, 32, 32, 3)) - 127.5) / 128).astype(np.float32)
    y = rng.integers(0, 10, size=B).astype(np.int32)
    octx = onn.Ctx(oresnet.init_ranges(om), 0, ctx.seed)
    logits = gm.forward(torch.from_numpy(x).to(DEV))
    assert np.array_equal(logits.cpu().numpy(), om.forward(x, octx))
    gm.compute_loss(torch.from_numpy(y).to(DEV))
    gm.backward()
    om.backward(gm.dlogits.cpu().numpy(), octx)
    og = oresnet.get_grads(om)
    for owner, var, gname in gm.param_slots():
        k = owner.name + {"W": "/W", "gamma": "/g", "beta": "/b"}[var]
        assert np.array_equal(getattr(owner, gname).cpu().numpy(), og[k]), k
    ctx.update_range_op()
    assert ctx.ranges() == octx.new_ranges()
    # the 4-bit weight codes really are 4-bit
    for c in _convs(gm):
        w = c.w_hwio.cpu().numpy()
        assert w.min() >= -8 and w.max() <= 7


def _convs(gm):
    from lbt_amd.dfxp.layers import Conv2d_q
    out = []

    def walk(layers):
        for l in layers:
            if isinstance(l, Conv2d_q):
                out.append(l)
            for attr in ("layers",):
                if hasattr(l, attr) and not isinstance(l, Conv2d_q):
                    walk(getattr(l, attr))
            for attr in ("residual", "shortcut"):
                if hasattr(l, attr):
                    walk(getattr(l, attr).layers)
    walk(gm.layers)
    return out


@pytest.mark.gpu
def test_fused_w4_equals_layerwise_w4():
    """The fused plan with 4-bit weights (packed arena, one pack launch, W4 GEMM entry points incl.
    the dgrad + BN pass-A fusion) == the layer-wise W4 model over 3 graph-captured steps."""
    from lbt_amd.fused import FusedResNet
    from lbt_amd.models import CIFAR10_Resnet20
    from lbt_amd.runtime import DfxpContext
    from lbt_amd.trainer import Trainer
    ctxA, ctxB = DfxpContext(seed=9), DfxpContext(seed=9)
    tA = Trainer(CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctxA, weight_bits=4), lr=1e-2, momentum=0.9,
                 use_graph=False)
    tB = Trainer(FusedResNet(CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctxB, weight_bits=4)), lr=1e-2,
                 momentum=0.9, use_graph=True)
    rng = np.random.default_rng(7)
    for _ in range(3):
        x = ((rng.integers(0, 256, size=(32, 32, 32, 3)) - 127.5) / 128).astype(np.float32)
        y = rng.integers(0, 10, size=32).astype(np.int32)
        xt, yt = torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV)
        assert tA.step(xt, yt).item() == tB.step(xt, yt).item()
    torch.cuda.synchronize()
    assert torch.equal(tA.flat.w, tB.flat.w)
    assert ctxA.ranges() == ctxB.ranges()
