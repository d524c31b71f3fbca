"""CPU tests of the oracle: pinned against the golden KATs, and its layer maths checked against
an independent float64 autodiff of the reference formulas (test infrastructure only)."""
import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F
from hypothesis import given, settings
from hypothesis import strategies as st

from oracle import dfxp, nn, philox, resnet

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_philox_random123_kat():
    kat = json.load(open(os.path.join(GOLDEN, "kat_philox.json")))
    for v in kat["vectors"]:
        c, k = v["ctr"], v["key"]
        out = philox.philox4x32_10(*[np.uint32(x) for x in c], k[0], k[1])
        assert [int(o) for o in out] == v["out"]


def test_uniform_noise_properties():
    u = philox.uniform_noise(1 << 16, qid=7, step=3, seed=11)
    assert u.dtype == np.float32 and u.min() >= 0 and u.max() < 1
    assert abs(float(u.mean()) - 0.5) < 0.01
    assert not np.array_equal(u, philox.uniform_noise(1 << 16, qid=8, step=3, seed=11))
    assert not np.array_equal(u, philox.uniform_noise(1 << 16, qid=7, step=4, seed=11))
    # noise index i depends only on i (prefix property used by the GPU kernels)
    assert np.array_equal(u[:1001], philox.uniform_noise(1001, qid=7, step=3, seed=11))


def test_dfxp_nearest_kat():
    kat = json.load(open(os.path.join(GOLDEN, "kat_dfxp.json")))
    for v in kat["nearest"]:
        q = dfxp.quantize_int(np.array(v["x"], np.float32), v["bits"], v["I"], stochastic=False)
        assert q.tolist() == v["q"], v["why"]


def test_dfxp_stochastic_kat():
    kat = json.load(open(os.path.join(GOLDEN, "kat_dfxp.json")))
    for v in kat["stochastic"]:
        for u, qe in zip(v["u"], v["q"]):
            q = dfxp.quantize_int(np.array([v["x"]], np.float32), v["bits"], v["I"], True, np.float32(u))
            assert int(q[0]) == qe, v["why"]


def test_dfxp_update_range_kat():
    kat = json.load(open(os.path.join(GOLDEN, "kat_dfxp.json")))
    for v in kat["update_range"]:
        x = np.array(v["x"], np.float32)
        if "ovf" in v:
            r1, r2 = dfxp.overflow_rate(x, v["bits"], v["I"])
            assert r1 == np.float32(v["ovf"])
            if "ovf2" in v:
                assert r2 == np.float32(v["ovf2"])
        assert dfxp.update_range(x, v["target"], v["bits"], v["I"]) == v["I_new"], v["why"]


def test_exponent_guard():
    assert dfxp.clamp_I(8, -100) == 8 - 1 - 30
    with pytest.raises(ValueError):
        dfxp.frac_bits(8, 8)


@settings(max_examples=60, deadline=None)
@given(bits=st.integers(3, 12), I=st.integers(-4, 2), seed=st.integers(0, 2**31 - 1))
def test_quantizer_properties(bits, I, seed):
    I = min(I, bits - 1)
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal(257) * 2.0 ** (I - 1)).astype(np.float32)
    u = rng.random(257).astype(np.float32)
    L = 2 ** (bits - 1)
    for stoch in (False, True):
        q = dfxp.quantize_int(x, bits, I, stoch, u if stoch else None)
        assert q.min() >= -L and q.max() <= L - 1
        # idempotence: re-quantising the dequantised value (nearest) returns the same codes
        xr = dfxp.dequant(q, dfxp.frac_bits(bits, I))
        assert np.array_equal(dfxp.quantize_int(xr, bits, I, False), q)
    # stochastic rounding is floor or ceil of x*m
    xm = x * np.float32(2.0 ** dfxp.frac_bits(bits, I))
    qs = dfxp.quantize_int(x, bits, I, True, u)
    inside = (xm > -L) & (xm < L - 1)
    assert np.all((qs[inside] == np.floor(xm[inside])) | (qs[inside] == np.floor(xm[inside]) + 1))


@settings(max_examples=40, deadline=None)
@given(seed=st.integers(0, 2**31 - 1), scale=st.floats(0.01, 100.0))
def test_update_range_monotone(seed, scale):
    """More overflow never makes the controller shrink the range more."""
    x = (np.random.default_rng(seed).standard_normal(100) * scale).astype(np.float32)
    I0 = 2
    a = dfxp.update_range(x, 0.0, 8, I0)
    b = dfxp.update_range((x * 4).astype(np.float32), 0.0, 8, I0)
    assert b >= a


def _tf_same_pad_nchw(x, k, s):
    H = x.shape[2]
    _, pt, pb = nn.tf_same_pads(H, k, s)
    return F.pad(x, (pt, pb, pt, pb))


@pytest.mark.parametrize("H,Cin,Cout,k,s", [(8, 3, 4, 3, 1), (8, 4, 8, 3, 2), (7, 2, 3, 3, 2), (8, 4, 8, 1, 2),
                                          (6, 3, 5, 3, 1)])
def test_oracle_int_conv_vs_torch(H, Cin, Cout, k, s):
    """oracle conv fwd / dgrad / wgrad (TF SAME) == float64 torch conv2d + autograd."""
    rng = np.random.default_rng(H * 100 + Cin * 10 + k + s)
    x = rng.integers(-256, 256, size=(2, H, H, Cin))
    w = rng.integers(-128, 128, size=(k, k, Cin, Cout))
    y = nn.conv_fwd_int(x, w, (s, s), "SAME")
    xt = torch.tensor(x, dtype=torch.float64).permute(0, 3, 1, 2).requires_grad_(True)
    wt = torch.tensor(w, dtype=torch.float64).permute(3, 2, 0, 1).requires_grad_(True)
    yt = F.conv2d(_tf_same_pad_nchw(xt, k, s), wt, stride=s)
    assert np.array_equal(y, yt.detach().permute(0, 2, 3, 1).numpy().astype(np.int64))
    g = rng.integers(-128, 128, size=y.shape)
    yt.backward(torch.tensor(g, dtype=torch.float64).permute(0, 3, 1, 2))
    dx = nn.conv_dgrad_int(g, w, (s, s), "SAME", x.shape)
    dw = nn.conv_wgrad_int(x, g, (s, s), "SAME", (k, k))
    assert np.array_equal(dx, xt.grad.permute(0, 2, 3, 1).numpy().astype(np.int64))
    assert np.array_equal(dw, wt.grad.permute(2, 3, 1, 0).numpy().astype(np.int64))


def test_tf_same_padding_is_asymmetric_for_stride2():
    assert nn.tf_same_pads(32, 3, 2) == (16, 0, 1)
    assert nn.tf_same_pads(32, 3, 1) == (32, 1, 1)
    assert nn.tf_same_pads(32, 1, 2) == (16, 0, 0)


def _ctx(names, I=2, step=0, seed=5):
    return nn.Ctx({n: I for n in names}, step, seed)


def test_oracle_bn_matches_autodiff():
    """NormQ/RescaleQ (integer-sum formulas) == float64 autodiff of the reference graph
    (dynamic_fixed_point.py:588-623,683-691) with STE quantisers."""
    rng = np.random.default_rng(0)
    X = (rng.standard_normal((4, 5, 5, 8)) * 0.7 + 0.2).astype(np.float32)
    g = (rng.standard_normal(X.shape) * 0.05).astype(np.float32)
    norm = nn.NormQ("bn-norm", 8, 8)
    resc = nn.RescaleQ("bn-rescale", 8, 8, weight_decay=1e-3)
    resc.gamma = (1 + 0.1 * rng.standard_normal(8)).astype(np.float32)
    resc.beta = (0.1 * rng.standard_normal(8)).astype(np.float32)
    ctx = _ctx(norm.range_names() + resc.range_names())
    y = resc.forward(norm.forward(X, ctx), ctx)
    dx = norm.backward(resc.backward(g, ctx), ctx)
    # float64 reference graph on the same quantised values
    s = 2.0 ** -norm.e
    xq = torch.tensor(norm.q * s, dtype=torch.float64, requires_grad=True)
    mean = xq.mean(dim=(0, 1, 2))
    var = ((xq - mean.detach()) ** 2).mean(dim=(0, 1, 2))
    xh = (xq - mean) / torch.sqrt(var + 1e-5)
    assert np.allclose(norm.xhat, xh.detach().numpy(), rtol=1e-5, atol=1e-5)
    # rescale on its own quantised input
    R = torch.tensor(resc.R * 2.0 ** -resc.er, dtype=torch.float64)
    gam = torch.tensor(resc.gq_f, dtype=torch.float64, requires_grad=True)
    yr = R * gam
    assert np.allclose(y, (yr + torch.tensor(y - yr.detach().numpy())).detach().numpy())
    G2 = torch.tensor(ctx.record["bn-rescale/grad_range"] * 2.0 ** -dfxp.frac_bits(8, 2), dtype=torch.float64)
    yr.backward(G2)
    dgam_ref = gam.grad.numpy() + 2e-3 * resc.gamma.astype(np.float64)
    assert np.allclose(resc.dgamma, dgam_ref, rtol=1e-6, atol=1e-7)
    assert np.allclose(resc.dbeta, G2.sum(dim=(0, 1, 2)).numpy(), rtol=1e-6, atol=1e-7)
    # normalisation backward with the quantised incoming gradient
    Gn = torch.tensor(ctx.record["bn-norm/grad_range"] * 2.0 ** -dfxp.frac_bits(8, 2), dtype=torch.float64)
    xh.backward(Gn)
    assert np.allclose(dx, xq.grad.numpy(), rtol=1e-4, atol=1e-6)


def test_oracle_resnet20_step_smoke():
    model = resnet.build_resnet((3, 3, 3), 8, 2e-4)
    rng = np.random.default_rng(0)
    params = {}
    for name, owner in model.params():
        if name.endswith("/W"):
            shp = owner.ksize if hasattr(owner, "ksize") else (owner.in_units, owner.units)
            fan = np.prod(shp[:-1])
            params[name] = rng.uniform(-np.sqrt(3 / fan), np.sqrt(3 / fan), size=shp).astype(np.float32)
        elif name.endswith("/g"):
            params[name] = np.ones(owner.C, np.float32)
        else:
            params[name] = np.zeros(owner.C, np.float32)
    assert sum(v.size for v in params.values()) == 272474 - 10  # 272 464 params
    state = dict(params=params, accum={k: np.zeros_like(v) for k, v in params.items()},
                 ranges=resnet.init_ranges(model), step=0)
    assert len(state["ranges"]) == 192  # 192 quantisers per step
    x = ((rng.integers(0, 256, size=(4, 32, 32, 3)) - 127.5) / 128).astype(np.float32)
    y = rng.integers(0, 10, size=4)
    loss, new_state, ctx = resnet.train_step(model, state, x, y, seed=0)
    assert np.isfinite(loss) and 1.0 < loss < 4.0
    assert len(ctx.counts) == 192
    assert new_state["step"] == 1
    assert any(new_state["ranges"][k] != 2 for k in new_state["ranges"])
