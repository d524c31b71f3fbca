"""CPU pins of the data-parallel oracle (oracle.resnet.dp_train_step) that the GPU world-2 tests
check the Trainer against: with one shard it IS the single-process step; with two shards the
global-batch loss splits exactly into the shards' shares and the exponents follow the summed counts."""
import numpy as np

from oracle import nn as onn
from oracle import resnet as oresnet


def _init(model, seed=0):
    rng = np.random.default_rng(seed)
    params = {}
    for name, owner in model.params():
        if name.endswith("/W"):
            shp = owner.ksize if hasattr(owner, "ksize") else (owner.in_units, owner.units)
            lim = np.sqrt(3 / np.prod(shp[:-1]))
            params[name] = rng.uniform(-lim, lim, size=shp).astype(np.float32)
        elif name.endswith("/g"):
            params[name] = (1 + 0.1 * rng.standard_normal(owner.C)).astype(np.float32)
        else:
            params[name] = (0.1 * rng.standard_normal(owner.C)).astype(np.float32)
    return dict(params=params, accum={k: np.zeros_like(v) for k, v in params.items()}, ranges=oresnet.init_ranges(model),
                step=0)


def _batch(B, seed):
    rng = np.random.default_rng(seed)
    return ((rng.integers(0, 256, size=(B, 32, 32, 3)) - 127.5) / 128).astype(np.float32), rng.integers(0, 10, size=B)


def test_dp_oracle_one_shard_is_the_single_process_step():
    m = oresnet.build_resnet((1, 1, 1), 8, 2e-4)
    st = _init(m)
    x, y = _batch(6, 1)
    la, sa, _ = oresnet.train_step(m, st, x, y)
    lb, sb, _ = oresnet.dp_train_step(m, st, [(x, y)])
    assert la == lb
    assert sa["ranges"] == sb["ranges"]
    for k in sa["params"]:
        assert np.array_equal(sa["params"][k], sb["params"][k]), k
        assert np.array_equal(sa["accum"][k], sb["accum"][k]), k


def test_dp_oracle_two_shards_loss_split_and_counts():
    m = oresnet.build_resnet((1, 1, 1), 8, 2e-4)
    st = _init(m, 3)
    x, y = _batch(8, 2)
    loss, new, ctxs = oresnet.dp_train_step(m, st, [(x[:4], y[:4]), (x[4:], y[4:])])
    parts = [onn.softmax_xent(c.logits, yy, norm=8)[0] for c, yy in zip(ctxs, (y[:4], y[4:]))]
    assert abs(loss - sum(parts)) < 1e-12
    # the global-batch normalisation: each shard's dz is (p - onehot) / 8
    for c, yy in zip(ctxs, (y[:4], y[4:])):
        z = c.logits
        p = np.exp(z - z.max(1, keepdims=True))
        p = p / p.sum(1, keepdims=True)
        p[np.arange(4), yy] -= 1
        np.testing.assert_allclose(c.dz, p / 8, rtol=1e-5, atol=1e-8)
    # exponents from the summed counts over the summed element counts
    from oracle import dfxp
    for name, I in new["ranges"].items():
        c = [cx.counts[name] for cx in ctxs]
        want = dfxp.update_range_from_counts(c[0][0] + c[1][0], c[0][1] + c[1][1], c[0][2] + c[1][2], 0.0, c[0][3],
                                             st["ranges"][name])
        assert I == want, name
