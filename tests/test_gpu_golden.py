"""The HIP path against the FROZEN oracle fixtures (tests/golden/*.npz, tools/gen_golden.py).

Unlike tests/test_gpu_parity.py, nothing here runs the oracle: the kernels (through the C-ABI) are
compared with committed numbers, so the oracle and the kernels cannot drift together.
Bit-exact for codes, counters, exponents, logits, gradients, weights and BN running averages; the
softmax (expf / logf, the one op of the step that is not) at rtol 1e-5, and the fixtures' own
d loss / d logits are injected where a test goes on to compare the backward bit for bit.
"""
import os

import numpy as np
import pytest
import torch

import golden_cases as G
from lbt_amd._lib import OUT_F32, OUT_I8, OUT_I16, OUT_U8OFF
from lbt_amd.dfxp import ops
from lbt_amd.models import CIFAR10_Resnet20
from lbt_amd.runtime import DfxpContext

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KIND = {"i8": OUT_I8, "u8off": OUT_U8OFF, "i16": OUT_I16, "f32": OUT_F32}


@pytest.fixture(scope="module")
def quant():
    return np.load(os.path.join(GOLD, "dfxp_quant.npz"))


@pytest.fixture(scope="module", params=["resnet20_b128", "resnet20_b128_gr6"])
def step(request):
    """The bench workload's frozen trajectory with the reference's default ranges, and in the timed
    configuration (gradient quantisers from I = -6, bench.py --grad-range's default)."""
    return np.load(os.path.join(GOLD, request.param + ".npz"))


def _model(ctx, step):
    kw = {}
    if "init_ranges" in step.files:
        kw["grad_range"] = G.BENCH_GRAD_RANGE
    gm = CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctx, **kw)
    if "init_ranges" in step.files:
        r = ctx.ranges()
        assert [r[str(k)] for k in step["range_names"]] == step["init_ranges"].tolist()
    return gm


@pytest.mark.parametrize("i", range(len(G.QUANT_CASES)))
def test_quantiser_kernel_matches_fixture(quant, i):
    """lbt_dfxp_quantize (codes, overflow counters) + lbt_dfxp_range_update against the frozen codes."""
    name, shape, bits, I, stoch, kind, lo, hi = G.QUANT_CASES[i]
    x = G.quant_input(i)
    assert G.digest(x) == str(quant["q%02d_input_sha" % i])
    ctx = DfxpContext(seed=G.QUANT_SEED)
    q = ctx.quantizer(name, bits, I, stochastic=stoch)
    out = ops.quantize(torch.from_numpy(x).to(DEV), q, KIND[kind]).cpu().numpy()
    if kind == "u8off":
        codes = out.astype(np.int64) + 128
    elif kind == "f32":  # dequantised values q * 2^-e: back to the codes (exact)
        codes = np.rint(out.astype(np.float64) * 2.0 ** (bits - I - 1)).astype(np.int64)
    else:
        codes = out.astype(np.int64)
    assert np.array_equal(codes.reshape(-1)[:64], quant["q%02d_codes_head" % i])
    assert G.digest(codes) == str(quant["q%02d_codes_sha" % i])
    c = ctx.counts_view()[0].sum(0).cpu().tolist()
    assert list(c) + [x.size] == quant["q%02d_counts" % i].tolist()
    ctx.update_range_op()
    assert ctx.ranges()[name] == int(quant["q%02d_new_I" % i])


def _load_params(gm, step):
    """The fixtures' initial parameters into a build model (checked against their digests)."""
    names = [str(k) for k in step["param_names"]]
    from oracle import resnet as R  # the oracle's parameter shapes / names only
    params = G.init_params(R.build_resnet((3, 3, 3), 8, 2e-4))
    assert [G.digest(params[k]) for k in names] == [str(s) for s in step["init_params_sha"]]
    seen = set()
    for owner, var, _ in gm.param_slots():
        k = owner.name + {"W": "/W", "gamma": "/g", "beta": "/b"}[var]
        t = getattr(owner, var)
        t.copy_(torch.from_numpy(params[k]).reshape(t.shape).to(t.device))
        seen.add(k)
    assert seen == set(names)
    return names


def _grads(gm):
    return {o.name + {"W": "/W", "gamma": "/g", "beta": "/b"}[v]: getattr(o, g).detach().cpu().numpy()
            for o, v, g in gm.param_slots()}


def _params(gm):
    return {o.name + {"W": "/W", "gamma": "/g", "beta": "/b"}[v]: getattr(o, v).detach().cpu().numpy()
            for o, v, _ in gm.param_slots()}


def _bn_digests(model):
    from lbt_amd.dfxp.layers import Normalization_q
    out = []

    def walk(l):
        if isinstance(l, Normalization_q):
            out.append(G.digest(np.concatenate([l.X_mean_running.cpu().numpy(), l.X_var_running.cpu().numpy()])))
        for sub in getattr(l, "layers", []) or []:
            walk(sub)
        for attr in ("residual", "shortcut"):
            if hasattr(l, attr):
                walk(getattr(l, attr))
    for l in model.layers:
        walk(l)
    return out


@pytest.mark.parametrize("fused", [False, True])
def test_bench_step_matches_fixture(step, fused):
    """Step 1 of the bench workload (B=128) on the layer-wise model and on the fused plan (its separate
    forward / compute_loss / backward launches): logits bit-exact, loss / dz at 1e-5, then with the
    fixture's dz injected every gradient, the updated exponents and the BN running averages bit-exact."""
    xs, ys = G.bench_batches()
    ctx = DfxpContext(seed=0)
    gm = _model(ctx, step)
    names = _load_params(gm, step)
    m = gm
    if fused:
        from lbt_amd.fused import FusedResNet
        m = FusedResNet(gm)
    x, y = torch.from_numpy(xs[0]).to(DEV), torch.from_numpy(ys[0]).to(torch.int32).to(DEV)
    logits = m.forward(x).cpu().numpy()
    assert np.array_equal(logits, step["step1_logits"])
    loss = m.compute_loss(y).item()
    assert abs(loss - float(step["step1_loss"])) <= 1e-5 * abs(float(step["step1_loss"]))
    np.testing.assert_allclose(m.dlogits.cpu().numpy(), step["step1_dz"], rtol=1e-5, atol=1e-9)
    m.dlogits.copy_(torch.from_numpy(step["step1_dz"]).to(DEV))
    m.backward()
    torch.cuda.synchronize()
    g = _grads(gm)
    assert [G.digest(g[k]) for k in names] == [str(s) for s in step["step1_grad_sha"]]
    assert _bn_digests(gm) == [str(s) for s in step["step1_bn_sha"]]
    ctx.update_range_op()
    rn = [str(k) for k in step["range_names"]]
    r = ctx.ranges()
    assert [r[k] for k in rn] == step["traj_ranges"][0].tolist()


def test_fused_plan_20_step_trajectory_matches_fixture(step, monkeypatch):
    """20 optimiser steps of the bench workload on the fused plan's conv / BN kernels (the timed
    configuration's launches, with the head as separate launches so the fixture's d loss / d logits
    can be injected each step): the exponents of all 192 quantisers after EVERY step, and the weights
    and BN running averages after the 20th, bit-identical to the frozen oracle trajectory; the loss of
    every step at 1e-5 -- along a trajectory whose loss runs from 2.6 to 8 000 (the reference's default
    ranges)."""
    from lbt_amd.fused import FusedResNet
    from lbt_amd.trainer import Trainer
    xs, ys = G.bench_batches()
    ctx = DfxpContext(seed=0)
    gm = _model(ctx, step)
    names = _load_params(gm, step)
    fm = FusedResNet(gm)
    cur = {"i": 0}

    def fwd_bwd(X, labels, update=False):  # train_fwd_bwd with the fixture's dz between loss and backward
        fm.forward(X)
        fm.compute_loss(labels)
        fm.dlogits.copy_(dzs[cur["i"]])
        fm.backward()
        return False
    monkeypatch.setattr(fm, "train_fwd_bwd", fwd_bwd)
    tr = Trainer(fm, lr=1e-2, momentum=0.9, batch_size=G.STEP_B, use_graph=False)
    tr.init_model()
    dzs = torch.from_numpy(step["traj_dz"]).to(DEV)
    X = [torch.from_numpy(x).to(DEV) for x in xs]
    Y = [torch.from_numpy(y).to(torch.int32).to(DEV) for y in ys]
    rn = [str(k) for k in step["range_names"]]
    for i in range(G.TRAJ_STEPS):
        cur["i"] = i
        loss = tr.step(X[i % 4], Y[i % 4]).item()
        torch.cuda.synchronize()
        want = float(step["traj_loss"][i])
        assert abs(loss - want) <= 1e-5 * abs(want), (i, loss, want)
        r = ctx.ranges()
        assert [r[k] for k in rn] == step["traj_ranges"][i].tolist(), i
    p = _params(gm)
    assert [G.digest(p[k]) for k in names] == [str(s) for s in step["traj_params_sha"]]
    assert _bn_digests(gm) == [str(s) for s in step["traj_bn_sha"]]


def test_timed_plan_trajectory_exponents_match_fixture(step):
    """The bench's own timed step (fused head, HIP-graph replay, no injection -- the GPU's softmax
    feeds the backward): the exponents after every one of the first 20 steps equal the frozen oracle
    trajectory's; the loss at 1e-4 relative (the softmax's last-ulp differences are carried through
    the stochastic rounding of the gradient codes from step 1 on)."""
    from lbt_amd.fused import FusedResNet
    from lbt_amd.trainer import Trainer
    xs, ys = G.bench_batches()
    ctx = DfxpContext(seed=0)
    gm = _model(ctx, step)
    _load_params(gm, step)
    tr = Trainer(FusedResNet(gm), lr=1e-2, momentum=0.9, batch_size=G.STEP_B, use_graph=True)
    tr.init_model()
    X = [torch.from_numpy(x).to(DEV) for x in xs]
    Y = [torch.from_numpy(y).to(torch.int32).to(DEV) for y in ys]
    rn = [str(k) for k in step["range_names"]]
    mism = []
    for i in range(G.TRAJ_STEPS):
        loss = tr.step(X[i % 4], Y[i % 4]).item()
        r = ctx.ranges()
        mism.append(sum(r[k] != v for k, v in zip(rn, step["traj_ranges"][i].tolist())))
        want = float(step["traj_loss"][i])
        assert abs(loss - want) <= 1e-4 * abs(want), (i, loss, want, mism)
    assert sum(mism) == 0, mism


@pytest.mark.parametrize("fused", [False, True])
def test_b16_step_matches_fixture(fused):
    """Step 1 at B = 16 (one rank's images of configs[2]'s 8 x 16 partition, as a batch of its own) in
    the timed configuration, on the batch-adaptive geometry (4-row stage-1 tiles, doubled weight-
    gradient splits, the 4-way head split): logits bit-exact, loss / dz at 1e-5, then with the
    fixture's dz injected every gradient, the updated weights and exponents bit-exact."""
    step = np.load(os.path.join(GOLD, "resnet20_b128_gr6.npz"))
    xs, ys = G.bench_batches()
    ctx = DfxpContext(seed=0)
    gm = _model(ctx, step)
    names = _load_params(gm, step)
    m = gm
    if fused:
        from lbt_amd.fused import FusedResNet
        m = FusedResNet(gm)
    x = torch.from_numpy(xs[0][:G.B16]).to(DEV)
    y = torch.from_numpy(ys[0][:G.B16]).to(torch.int32).to(DEV)
    assert np.array_equal(m.forward(x).cpu().numpy(), step["b16_logits"])
    loss = m.compute_loss(y).item()
    assert abs(loss - float(step["b16_loss"])) <= 1e-5 * abs(float(step["b16_loss"]))
    np.testing.assert_allclose(m.dlogits.cpu().numpy(), step["b16_dz"], rtol=1e-5, atol=1e-9)
    m.dlogits.copy_(torch.from_numpy(step["b16_dz"]).to(DEV))
    m.backward()
    torch.cuda.synchronize()
    g = _grads(gm)
    assert [G.digest(g[k]) for k in names] == [str(s) for s in step["b16_grad_sha"]]
    ctx.update_range_op()
    r = ctx.ranges()
    assert [r[str(k)] for k in step["range_names"]] == step["b16_ranges"].tolist()
