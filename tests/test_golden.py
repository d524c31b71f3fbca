"""The oracle pinned to its frozen fixtures (tests/golden/*.npz, tools/gen_golden.py).

CPU only. A change to the oracle that moves any quantiser code, overflow counter, range update, logit,
gradient, BN running average or exponent of the bench workload's first steps fails here, whatever the
kernels do -- the GPU suite compares the HIP path with the same files (tests/test_gpu_golden.py)."""
import os

import numpy as np
import pytest

import golden_cases as G
from oracle import dfxp
from oracle import nn as onn
from oracle import resnet as R

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def quant():
    return np.load(os.path.join(GOLD, "dfxp_quant.npz"))


@pytest.fixture(scope="module")
def step():
    return np.load(os.path.join(GOLD, "resnet20_b128.npz"))


@pytest.mark.parametrize("i", range(len(G.QUANT_CASES)))
def test_oracle_quantiser_matches_fixture(quant, i):
    name, shape, bits, I, stoch, kind, lo, hi = G.QUANT_CASES[i]
    x = G.quant_input(i)
    assert G.digest(x) == str(quant["q%02d_input_sha" % i]), "input generator drifted"
    noise = dfxp.noise_for(shape, dfxp.qid_of(name), 0, G.QUANT_SEED) if stoch else None
    q = dfxp.quantize_int(x, bits, I, stoch, noise)
    assert np.array_equal(q.reshape(-1)[:64], quant["q%02d_codes_head" % i])
    assert G.digest(q) == str(quant["q%02d_codes_sha" % i])
    c1, c2 = dfxp.overflow_counts(x, bits, I)
    assert [c1, c2, x.size] == quant["q%02d_counts" % i].tolist()
    assert dfxp.update_range_from_counts(c1, c2, x.size, 0.0, bits, I) == int(quant["q%02d_new_I" % i])


def test_fixture_cases_cover_every_controller_branch(quant):
    """The fixture set exercises update_range's three branches (:83-94): I + 1, I - 1 and unchanged."""
    moves = {int(quant["q%02d_new_I" % i]) - G.QUANT_CASES[i][3] for i in range(len(G.QUANT_CASES))}
    assert moves == {-1, 0, 1}


def test_oracle_bench_step_matches_fixture(step):
    """Step 1 of the bench workload (B=128) in full, and step 2's loss and exponents."""
    model = R.build_resnet((3, 3, 3), 8, 2e-4)
    params = G.init_params(model)
    names = [str(k) for k in step["param_names"]]
    rnames = [str(k) for k in step["range_names"]]
    assert names == sorted(params) and rnames == sorted(R.init_ranges(model))
    assert [G.digest(params[k]) for k in names] == [str(s) for s in step["init_params_sha"]]
    xs, ys = G.bench_batches()
    assert [G.digest(x) for x in xs] == [str(s) for s in step["batch_x_sha"]], "bench batch generator drifted"
    assert [G.digest(y) for y in ys] == [str(s) for s in step["batch_y_sha"]]
    state = dict(params=params, accum={k: np.zeros_like(v) for k, v in params.items()},
                 ranges=R.init_ranges(model), step=0)
    loss, state, ctx = R.train_step(model, state, xs[0], ys[0], lr=1e-2, momentum=0.9, seed=0)
    assert np.array_equal(ctx.logits, step["step1_logits"])
    assert np.array_equal(ctx.dz, step["step1_dz"])
    assert loss == float(step["step1_loss"])
    grads = R.get_grads(model)
    assert [G.digest(grads[k]) for k in names] == [str(s) for s in step["step1_grad_sha"]]
    assert [G.digest(state["params"][k]) for k in names] == [str(s) for s in step["step1_params_sha"]]
    bn = [G.digest(np.concatenate([l.mean_running, l.var_running])) for l in R._walk(model) if isinstance(l, onn.NormQ)]
    assert bn == [str(s) for s in step["step1_bn_sha"]]
    cn = [str(k) for k in step["step1_codes_names"]]
    assert [G.digest(ctx.record[k]) for k in cn] == [str(s) for s in step["step1_codes_sha"]]
    assert [state["ranges"][k] for k in rnames] == step["traj_ranges"][0].tolist()
    loss2, state, _ = R.train_step(model, state, xs[1], ys[1], lr=1e-2, momentum=0.9, seed=0)
    assert loss2 == float(step["traj_loss"][1])
    assert [state["ranges"][k] for k in rnames] == step["traj_ranges"][1].tolist()


@pytest.fixture(scope="module")
def step_gr6():
    return np.load(os.path.join(GOLD, "resnet20_b128_gr6.npz"))


def test_oracle_timed_config_matches_fixture(step_gr6):
    """The timed configuration (bench.py --grad-range -6: gradient quantisers from I = -6): step 1 in
    full, step 2's loss and exponents; and the B = 16 step 1 (one rank's share of configs[2])."""
    f = step_gr6
    model = R.build_resnet((3, 3, 3), 8, 2e-4)
    params = G.init_params(model)
    names = [str(k) for k in f["param_names"]]
    rnames = [str(k) for k in f["range_names"]]
    assert [G.digest(params[k]) for k in names] == [str(s) for s in f["init_params_sha"]]
    ranges0 = G.init_ranges(model, G.BENCH_GRAD_RANGE)
    assert [ranges0[k] for k in rnames] == f["init_ranges"].tolist()
    assert sum(k.endswith("grad_range") for k in rnames) == int((f["init_ranges"] == -6).sum()) > 0
    xs, ys = G.bench_batches()
    assert [G.digest(x) for x in xs] == [str(s) for s in f["batch_x_sha"]], "bench batch generator drifted"
    state = dict(params=params, accum={k: np.zeros_like(v) for k, v in params.items()}, ranges=dict(ranges0), step=0)
    loss, state, ctx = R.train_step(model, state, xs[0], ys[0], lr=1e-2, momentum=0.9, seed=0)
    assert np.array_equal(ctx.logits, f["step1_logits"]) and np.array_equal(ctx.dz, f["step1_dz"])
    assert loss == float(f["step1_loss"])
    grads = R.get_grads(model)
    assert [G.digest(grads[k]) for k in names] == [str(s) for s in f["step1_grad_sha"]]
    assert [G.digest(state["params"][k]) for k in names] == [str(s) for s in f["step1_params_sha"]]
    cn = [str(k) for k in f["step1_codes_names"]]
    assert [G.digest(ctx.record[k]) for k in cn] == [str(s) for s in f["step1_codes_sha"]]
    assert [state["ranges"][k] for k in rnames] == f["traj_ranges"][0].tolist()
    bn = [G.digest(np.concatenate([l.mean_running, l.var_running])) for l in R._walk(model) if isinstance(l, onn.NormQ)]
    assert bn == [str(s) for s in f["step1_bn_sha"]]
    loss2, state, _ = R.train_step(model, state, xs[1], ys[1], lr=1e-2, momentum=0.9, seed=0)
    assert loss2 == float(f["traj_loss"][1])
    assert [state["ranges"][k] for k in rnames] == f["traj_ranges"][1].tolist()
    # B = 16, a fresh model (its own BN running averages)
    model = R.build_resnet((3, 3, 3), 8, 2e-4)
    params = G.init_params(model)
    state = dict(params=params, accum={k: np.zeros_like(v) for k, v in params.items()}, ranges=dict(ranges0), step=0)
    loss, state, ctx = R.train_step(model, state, xs[0][:G.B16], ys[0][:G.B16], lr=1e-2, momentum=0.9, seed=0)
    assert np.array_equal(ctx.logits, f["b16_logits"]) and loss == float(f["b16_loss"])
    grads = R.get_grads(model)
    assert [G.digest(grads[k]) for k in names] == [str(s) for s in f["b16_grad_sha"]]
    assert [state["ranges"][k] for k in rnames] == f["b16_ranges"].tolist()
