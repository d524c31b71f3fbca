"""Freeze the oracle: write tests/golden/dfxp_quant.npz and tests/golden/resnet20_b128.npz.

    python tools/gen_golden.py [quant] [b128] [gr6]     (about a minute each on 8 cores)

Test infrastructure. The reference (TensorFlow 1.x) cannot run here
and holds no fixtures, so these are the oracle's outputs frozen at a reviewed commit: the quantiser
codes / overflow counters / range updates of every ResNet-20 tensor class (dynamic_fixed_point.py:4-94),
and one full B=128 ResNet-20 step plus a 20-step trajectory of the bench workload (models.py:7-54,
371-455, trainer.py:79-84,144-162), once with the reference's default ranges and once in the timed
configuration (gradient quantisers from I = -6, bench.py --grad-range; plus a B = 16 step 1).
tests/test_golden.py pins the oracle to them on the CPU;
tests/test_gpu_golden.py checks the HIP path against them directly on the MI355X.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import golden_cases as G  # noqa: E402
from oracle import dfxp  # noqa: E402
from oracle import nn as onn  # noqa: E402
from oracle import resnet as R  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def quant_fixtures():
    out = {}
    for i, (name, shape, bits, I, stoch, kind, lo, hi) in enumerate(G.QUANT_CASES):
        x = G.quant_input(i)
        noise = dfxp.noise_for(shape, dfxp.qid_of(name), 0, G.QUANT_SEED) if stoch else None
        q = dfxp.quantize_int(x, bits, I, stoch, noise)
        c1, c2 = dfxp.overflow_counts(x, bits, I)
        newI = dfxp.update_range_from_counts(c1, c2, x.size, 0.0, bits, I)
        out["q%02d_input_sha" % i] = np.array(G.digest(x))
        out["q%02d_codes_sha" % i] = np.array(G.digest(q))
        out["q%02d_codes_head" % i] = q.reshape(-1)[:64].astype(np.int32)
        out["q%02d_counts" % i] = np.array([c1, c2, x.size], np.int64)
        out["q%02d_new_I" % i] = np.array(newI, np.int32)
        print("q%02d %-45s c1 %7d c2 %7d  I %d -> %d" % (i, name, c1, c2, I, newI))
    return out


def bn_state(model):
    return [(l.mean_running.copy(), l.var_running.copy()) for l in R._walk(model) if isinstance(l, onn.NormQ)]


def step_fixtures(grad_range=None):
    """grad_range None: the reference's default ranges (every *_range at I = 2); an int: the gradient
    quantisers start there (bench.py's timed configuration: --grad-range -6, G.init_ranges)."""
    model = R.build_resnet((3, 3, 3), 8, 2e-4)
    params = G.init_params(model)
    names = sorted(params)
    rnames = sorted(R.init_ranges(model))
    xs, ys = G.bench_batches()
    out = {"param_names": np.array(names), "range_names": np.array(rnames),
           "init_params_sha": np.array([G.digest(params[k]) for k in names]),
           "batch_x_sha": np.array([G.digest(x) for x in xs]), "batch_y_sha": np.array([G.digest(y) for y in ys])}
    ranges0 = G.init_ranges(model, grad_range)
    out["init_ranges"] = np.array([ranges0[k] for k in rnames], np.int32)
    if grad_range is not None:
        out.update(b16_fixtures(model, names, rnames, ranges0, xs, ys))
    state = dict(params=params, accum={k: np.zeros_like(v) for k, v in params.items()},
                 ranges=dict(ranges0), step=0)
    losses, ranges, dzs = [], [], []
    for i in range(G.TRAJ_STEPS):
        loss, state, ctx = R.train_step(model, state, xs[i % 4], ys[i % 4], lr=1e-2, momentum=0.9, seed=0)
        losses.append(loss)
        dzs.append(ctx.dz.astype(np.float32))
        ranges.append([state["ranges"][k] for k in rnames])
        if i == 0:  # the first step in full: logits, d loss / d logits, every gradient, BN running stats
            grads = R.get_grads(model)
            out["step1_logits"] = ctx.logits.astype(np.float32)
            out["step1_dz"] = ctx.dz.astype(np.float32)
            out["step1_loss"] = np.array(loss, np.float64)
            out["step1_grad_sha"] = np.array([G.digest(grads[k]) for k in names])
            out["step1_grad_sum"] = np.array([float(grads[k].astype(np.float64).sum()) for k in names])
            out["step1_params_sha"] = np.array([G.digest(state["params"][k]) for k in names])
            bn = bn_state(model)
            out["step1_bn_sha"] = np.array([G.digest(np.concatenate([m, v])) for m, v in bn])
            out["step1_codes_sha"] = np.array([G.digest(ctx.record[k]) for k in rnames if k in ctx.record])
            out["step1_codes_names"] = np.array([k for k in rnames if k in ctx.record])
        print("step %2d loss %.6f" % (i + 1, loss), flush=True)
    out["traj_loss"] = np.array(losses, np.float64)
    out["traj_dz"] = np.array(dzs, np.float32)  # each step's d loss / d logits (the GPU tests inject them)
    out["traj_ranges"] = np.array(ranges, np.int32)
    out["traj_params_sha"] = np.array([G.digest(state["params"][k]) for k in names])
    out["traj_bn_sha"] = np.array([G.digest(np.concatenate([m, v])) for m, v in bn_state(model)])
    return out


def b16_fixtures(model, names, rnames, ranges0, xs, ys):
    """Step 1 on the first G.B16 images of the first bench batch (one rank's share of configs[2]'s
    8 x 16 partition, run as its own batch): logits, loss, dz, every gradient, the new exponents."""
    model = R.build_resnet((3, 3, 3), 8, 2e-4)  # its own BN running averages
    params = G.init_params(model)
    state = dict(params=params, accum={k: np.zeros_like(v) for k, v in params.items()}, ranges=dict(ranges0),
                 step=0)
    loss, state, ctx = R.train_step(model, state, xs[0][:G.B16], ys[0][:G.B16], lr=1e-2, momentum=0.9, seed=0)
    grads = R.get_grads(model)
    print("b16 step 1 loss %.6f" % loss, flush=True)
    return {"b16_logits": ctx.logits.astype(np.float32), "b16_dz": ctx.dz.astype(np.float32),
            "b16_loss": np.array(loss, np.float64),
            "b16_grad_sha": np.array([G.digest(grads[k]) for k in names]),
            "b16_params_sha": np.array([G.digest(state["params"][k]) for k in names]),
            "b16_ranges": np.array([state["ranges"][k] for k in rnames], np.int32)}


def main():
    os.makedirs(OUT, exist_ok=True)
    which = sys.argv[1:] or ["quant", "b128", "gr6"]
    if "quant" in which:
        np.savez_compressed(os.path.join(OUT, "dfxp_quant.npz"), **quant_fixtures())
    if "b128" in which:
        np.savez_compressed(os.path.join(OUT, "resnet20_b128.npz"), **step_fixtures())
    if "gr6" in which:  # the timed configuration (bench.py --grad-range -6, its default)
        np.savez_compressed(os.path.join(OUT, "resnet20_b128_gr6.npz"), **step_fixtures(G.BENCH_GRAD_RANGE))


if __name__ == "__main__":
    main()
