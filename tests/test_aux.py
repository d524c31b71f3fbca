"""Components either side of the hot path: GradientBuffer_q, Dense_q's
pre_dense_func, preprocess_image, the test loop and the checkpoint.

CPU tests pin the oracle restatements (oracle/aux.py) with hand-worked known answers; the
@gpu tests check the HIP kernels (lbt_amd/csrc/aux.hip) and the Trainer against them.
"""
import numpy as np
import pytest
import torch

from oracle import aux as oaux
from oracle import dfxp as odfxp
from oracle import nn as onn

DEV = "cuda"
F32 = np.float32


# ---------------------------------------------------------------- oracle known answers (CPU)
def test_pre_dense_known_answers():
    eps = oaux.pre_dense_eps(8, 2)
    assert eps == F32(1 / 64)
    accu = np.full((1, 3), 0.001, F32)
    init = np.ones((1, 3), int)
    rem = np.zeros((1, 3), int)
    # step 1: |g| < eps -> start accumulating (accu = g); |g| >= eps -> pass through untouched
    g, accu, init, rem = oaux.pre_dense(np.array([[0.01, 0.02, -0.005]], F32), eps, accu, init, rem)
    assert g.tolist() == [[F32(0.01), F32(0.02), F32(-0.005)]]
    assert init.tolist() == [[0, 1, 0]] and rem.tolist() == [[0, 0, 0]]
    assert accu.tolist() == [[F32(0.01), F32(0.001), F32(-0.005)]]
    # step 2: accumulated 0.01 + 0.01 = 0.02 > eps -> released as the gradient, remainder kept
    g, accu, init, rem = oaux.pre_dense(np.array([[0.01, 0.0, -0.001]], F32), eps, accu, init, rem)
    a = F32(F32(0.01) + F32(0.01))
    assert g[0, 0] == a and init[0, 0] == 1 and rem[0, 0] == 1
    assert accu[0, 0] == F32(a - F32(np.floor(a / eps)) * eps)
    assert g[0, 1] == 0.0 and init[0, 1] == 0 and accu[0, 1] == 0.0  # |0| < eps: accumulation starts at g
    assert g[0, 2] == F32(-0.001) and accu[0, 2] == F32(F32(-0.005) + F32(-0.001)) and init[0, 2] == 0
    # step 3: a small gradient after a release resumes from the remainder (rem_flag)
    r = accu[0, 0]
    g, accu, init, rem = oaux.pre_dense(np.array([[0.001, 0.0, -0.02]], F32), eps, accu, init, rem)
    assert init[0, 0] == 0 and accu[0, 0] == F32(r + F32(0.001))
    b = F32(F32(-0.006) + F32(-0.02))
    assert g[0, 2] == b and accu[0, 2] == F32(b + F32(np.floor(-b / eps)) * eps) and init[0, 2] == 1


def test_augment_known_answer():
    x = np.arange(2 * 4 * 4, dtype=F32).reshape(2, 4, 4, 1)
    flip, oy, ox = oaux.augment_draws(2, 1, 5, 0)
    out = oaux.augment_flip_crop(x, 1, 5, 0)
    for n in range(2):
        img = x[n, :, ::-1] if flip[n] else x[n]
        for i in range(4):
            for j in range(4):
                si, sj = i + oy[n] - 1, j + ox[n] - 1
                want = img[si, sj, 0] if 0 <= si < 4 and 0 <= sj < 4 else 0.0
                assert out[n, i, j, 0] == want
    # pad 0: no crop offsets, only flips
    out0 = oaux.augment_flip_crop(x, 0, 9, 3)
    f0, _, _ = oaux.augment_draws(2, 0, 9, 3)
    for n in range(2):
        assert np.array_equal(out0[n], x[n, :, ::-1] if f0[n] else x[n])


def test_gradient_buffer_error_feedback():
    """Error feedback: sum of emitted gq + the residue == sum of incoming grads (no clipping)."""
    rng = np.random.default_rng(0)
    gb = oaux.GradientBufferQ("gb", 8, (6, 5))
    ctx = onn.Ctx({"gb/grad_range": 3}, 0, 11)
    sent = np.zeros((6, 5), np.float64)
    seen = np.zeros((6, 5), np.float64)
    for step in range(5):
        ctx.step = step
        g = rng.normal(0, 0.05, size=(4, 5)).astype(F32)  # batch 4 < buffer rows 6: zero-padded
        out = gb.backward(g, ctx)
        assert out.shape == (4, 5)
        seen[:4] += g
        sent[:4] += out
    resid = gb.buffer.astype(np.float64)
    # rows >= 4 never receive gradient: their residue is what they emitted, negated
    assert np.allclose(sent[:4] + resid[:4], seen[:4], atol=1e-6)
    assert np.all(np.abs(gb.buffer) <= 2.0 ** -odfxp.frac_bits(8, 3) + 1e-9)


# ---------------------------------------------------------------- HIP kernels (GPU)
@pytest.mark.gpu
def test_gradient_buffer_kernel_matches_oracle():
    from lbt_amd.dfxp.layers import GradientBuffer_q
    from lbt_amd.runtime import DfxpContext
    rng = np.random.default_rng(1)
    ctx = DfxpContext(seed=11)
    layer = GradientBuffer_q("gb", 8, (6, 5, 3), grad_range=1, ctx=ctx)
    ref = oaux.GradientBufferQ("gb", 8, (6, 5, 3))
    for step in range(3):
        octx = onn.Ctx(dict(ctx.ranges()), int(ctx.step.item()), 11)
        g = rng.normal(0, 0.3, size=(4, 5, 3)).astype(F32)
        want = ref.backward(g, octx)
        got = layer.backward(torch.from_numpy(g).to(DEV)).cpu().numpy()
        assert np.array_equal(got, want), step
        assert np.array_equal(layer.buffer.cpu().numpy(), ref.buffer), step
        c1, c2, _, _ = octx.counts["gb/grad_range"]
        assert tuple(ctx.counts_view()[0].sum(0).cpu().tolist()) == (c1, c2)
        ctx.update_range_op()
        assert ctx.ranges()["gb/grad_range"] == octx.new_ranges()["gb/grad_range"]


@pytest.mark.gpu
def test_gradient_buffer_bits32_bypass():
    from lbt_amd.dfxp.layers import GradientBuffer_q
    from lbt_amd.runtime import DfxpContext
    ctx = DfxpContext(seed=1)
    layer = GradientBuffer_q("gb32", 32, (3, 4), ctx=ctx)
    g = torch.randn(2, 4, device=DEV)
    assert torch.equal(layer.backward(g), g)
    assert float(layer.buffer.abs().sum().item()) == 0.0


@pytest.mark.gpu
def test_pre_dense_kernel_matches_oracle():
    from lbt_amd.dfxp.layers import Dense_q
    from lbt_amd.runtime import DfxpContext
    ctx = DfxpContext(seed=3)
    d = Dense_q("dense", 8, 64, 10, use_bias=False, grad_range=2, ctx=ctx)
    rng = np.random.default_rng(2)
    eps = oaux.pre_dense_eps(8, 2)
    accu = np.full((64, 10), 0.001, F32)
    init = np.ones((64, 10), int)
    rem = np.zeros((64, 10), int)
    for step in range(6):
        g = (rng.normal(0, 0.01, size=(32, 10)) * (rng.random((32, 10)) < 0.7)).astype(F32)
        want, accu, init, rem = oaux.pre_dense(g, eps, accu, init, rem)
        got = d.pre_dense_func(torch.from_numpy(g).to(DEV)).cpu().numpy()
        assert np.array_equal(got, want), step
        assert np.array_equal(d._pd_accu.cpu().numpy(), accu), step
        assert np.array_equal(d._pd_init.cpu().numpy(), init) and np.array_equal(d._pd_rem.cpu().numpy(), rem)


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,W,C,pad", [(128, 32, 32, 3, 4), (3, 5, 7, 2, 2), (4, 8, 8, 1, 0)])
def test_augment_kernel_matches_oracle(N, H, W, C, pad):
    from lbt_amd.dfxp import ops
    x = np.random.default_rng(N).normal(size=(N, H, W, C)).astype(F32)
    got = ops.augment_flip_crop(torch.from_numpy(x).to(DEV), pad, 1234, 77).cpu().numpy()
    assert np.array_equal(got, oaux.augment_flip_crop(x, pad, 1234, 77))


def _trainer(seed, fused=True):
    from lbt_amd.fused import FusedResNet
    from lbt_amd.models import CIFAR10_Resnet20
    from lbt_amd.runtime import DfxpContext
    from lbt_amd.trainer import Trainer
    ctx = DfxpContext(seed=seed)
    m = CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctx)
    return Trainer(FusedResNet(m) if fused else m, lr=1e-2, momentum=0.9, use_graph=True)


def _batch(B, seed):
    rng = np.random.default_rng(seed)
    x = ((rng.integers(0, 256, size=(B, 32, 32, 3)) - 127.5) / 128).astype(F32)
    return x, rng.integers(0, 10, size=B).astype(np.int32)


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [True, False])
def test_evaluate_and_checkpoint_round_trip(tmp_path, fused):
    """The test loop leaves training untouched (counters, captured graph) and a checkpoint
    restores the exact training state: continuing from it gives bit-identical steps."""
    t = _trainer(5, fused)
    xs = [_batch(32, 40 + i) for i in range(4)]
    for x, y in xs[:2]:
        t.step(torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV))
    counts = t.ctx.counts.clone()
    xte, yte = _batch(96, 99)
    acc, loss = t.evaluate(xte, yte, batch_size=40)  # ragged last batch
    assert 0.0 <= acc <= 1.0 and np.isfinite(loss)
    assert torch.equal(counts, t.ctx.counts)
    path = t.save_model(str(tmp_path / "ckpt"))
    t2 = _trainer(5, fused)
    t2.load_model(path)
    assert torch.equal(t.flat.w, t2.flat.w) and torch.equal(t.flat.a, t2.flat.a)
    assert torch.equal(t.ctx.exps, t2.ctx.exps) and torch.equal(t.ctx.step, t2.ctx.step)
    for x, y in xs[2:]:
        la = t.step(torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV)).item()
        lb = t2.step(torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV)).item()
        assert la == lb
    torch.cuda.synchronize()
    assert torch.equal(t.flat.w, t2.flat.w)
    assert t.ctx.ranges() == t2.ctx.ranges()
