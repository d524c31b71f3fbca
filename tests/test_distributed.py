"""Data-parallel path on CPU: world_size-2 gloo processes run the REAL exchange of the trainer
(lbt_amd.distributed: one all-reduce of [grads | folded counters]) on oracle gradients / overflow counters of their batch shards."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lbt_amd import distributed as D
        from oracle import dfxp, nn
        from oracle import resnet as R
        rng = np.random.default_rng(0)          # identical weights on every rank
        model = R.build_resnet((1, 1, 1), 8, 2e-4)
        params = {}
        for name, owner in model.params():
            if name.endswith("/W"):
                shp = owner.ksize if hasattr(owner, "ksize") else (owner.in_units, owner.units)
                lim = np.sqrt(3 / np.prod(shp[:-1]))
                params[name] = rng.uniform(-lim, lim, size=shp).astype(np.float32)
            elif name.endswith("/g"):
                params[name] = np.ones(owner.C, np.float32)
            else:
                params[name] = np.zeros(owner.C, np.float32)
        R.set_params(model, params)
        xr = np.random.default_rng(100 + rank)  # each rank its own batch shard
        x = ((xr.integers(0, 256, size=(4, 32, 32, 3)) - 127.5) / 128).astype(np.float32)
        y = xr.integers(0, 10, size=4)
        ranges = R.init_ranges(model)
        _, _, grads, ctx = R.forward_backward(model, ranges, x, y, step=0, seed=0)
        names = sorted(grads)
        flat = torch.from_numpy(np.concatenate([grads[k].ravel() for k in names]).astype(np.float32))
        qn = sorted(ctx.counts)
        counts = torch.tensor([c for k in qn for c in ctx.counts[k][:2]], dtype=torch.int32)
        local = (flat.clone(), counts.clone())
        # the trainer's layout: grads are the comm head, folded counters the tail
        comm = D.make_comm_buffer(flat.numel(), len(qn), "cpu")
        n = flat.numel()
        comm[:n].copy_(flat)
        comm[n:].copy_(D.fold_host(counts))
        # large counters (2**30-element tensors overflowing) must also survive exactly
        big = torch.tensor([[2 ** 29 + 12345 + rank, 2 ** 28 + 4095]], dtype=torch.int64)
        bigc = D.fold_host(big)
        D.allreduce_comm(comm)
        D.allreduce_comm(bigc)
        flat = comm[:n]
        counts = D.unfold_host(comm[n:]).view(-1).to(torch.int32)
        assert D.unfold_host(bigc).tolist() == [[2 ** 30 + 24690 + 1, 2 ** 29 + 8190]]
        c = counts.view(-1, 2).tolist()
        new_I = {k: dfxp.update_range_from_counts(c[i][0], c[i][1], ctx.counts[k][2] * world, 0.0,
                                                  ctx.counts[k][3], ranges[k]) for i, k in enumerate(qn)}
        out_q.put((rank, local[0].numpy(), local[1].numpy(), flat.numpy(), counts.numpy(), new_I))
    finally:
        dist.destroy_process_group()


def test_dp_exchange_two_ranks_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, g0, c0, G0, C0, I0), (_, g1, c1, G1, C1, I1) = res
    # every rank holds the exact sums
    assert np.array_equal(G0, G1) and np.array_equal(C0, C1)
    assert np.array_equal(C0, c0 + c1)                        # integer counters: exact
    np.testing.assert_allclose(G0, g0 + g1, rtol=1e-6, atol=1e-12)
    assert not np.array_equal(g0, g1)                          # shards really differ
    # identical DFXP exponents on both ranks, from the global counts
    assert I0 == I1


def _xworker(rank, world, port, out_q):
    """The exact exchange's layout on CPU: each rank packs its shard's integer gradient numerators,
    overflow counts and loss share into the int64 buffer of lbt_amd.distributed.make_exchange, one
    gloo all-reduce sums them, and the dequantised result must equal the oracle's global step."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lbt_amd import distributed as D
        from oracle import resnet as R
        model = R.build_resnet((1, 1, 1), 8, 2e-4)
        rng = np.random.default_rng(0)
        params = {}
        for name, owner in model.params():
            if name.endswith("/W"):
                shp = owner.ksize if hasattr(owner, "ksize") else (owner.in_units, owner.units)
                params[name] = rng.uniform(-0.3, 0.3, size=shp).astype(np.float32)
            elif name.endswith("/g"):
                params[name] = np.ones(owner.C, np.float32)
            else:
                params[name] = np.zeros(owner.C, np.float32)
        state = dict(params=params, accum={k: np.zeros_like(v) for k, v in params.items()},
                     ranges=R.init_ranges(model), step=0)
        xr = np.random.default_rng(7)
        X = ((xr.integers(0, 256, size=(2 * world, 32, 32, 3)) - 127.5) / 128).astype(np.float32)
        Y = xr.integers(0, 10, size=2 * world)
        shards = [(X[2 * r:2 * r + 2], Y[2 * r:2 * r + 2]) for r in range(world)]
        R.set_params(model, params)
        loss, _, _, ctx = R.forward_backward(model, state["ranges"], *shards[rank], step=0, seed=0, norm=2 * world)
        num = R._numerators(model)
        keys = sorted(num)
        names = sorted(ctx.counts)
        n = sum(num[k][1].size for k in keys)
        buf, x = D.make_exchange(n, len(names), "cpu")
        off = 0
        for k in keys:
            v = num[k][1].ravel()
            buf[off:off + v.size] = torch.from_numpy(v.astype(np.int64))
            off += v.size
        for i, k in enumerate(names):
            buf[x.cnt_off + 2 * i] = ctx.counts[k][0]
            buf[x.cnt_off + 2 * i + 1] = ctx.counts[k][1]
        buf[x.loss_off] = int(round(loss * 2 ** 32))
        D.allreduce_comm(buf)
        want_loss, want, _ = R.dp_train_step(model, state, shards)
        got = {}
        off = 0
        for k in keys:
            kind, S, sc, owner = num[k]
            tot = buf[off:off + S.size].numpy().reshape(S.shape)
            off += S.size
            if kind == "w":
                got[k] = (R.nn.scale_int(tot, sc) + (np.float32(2 * owner.wd) * params[k]).astype(np.float32)).astype(np.float32)
            elif kind == "g":
                got[k] = ((tot.astype(np.float64) * sc).astype(np.float32) + (np.float32(2 * owner.wd) * params[k]).astype(np.float32)).astype(np.float32)
            else:
                got[k] = (tot.astype(np.float64) * sc).astype(np.float32)
        new_p, _ = R.sgd_momentum(params, got, state["accum"], 1e-2, 0.9)
        ok = all(np.array_equal(new_p[k], want["params"][k]) for k in keys)
        counts = {k: (int(buf[x.cnt_off + 2 * i]), int(buf[x.cnt_off + 2 * i + 1])) for i, k in enumerate(names)}
        out_q.put((rank, ok, counts, float(buf[x.loss_off]) / 2 ** 32, want_loss))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_exact_int64_exchange_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_xworker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, ok, counts, loss, want_loss in res:
        assert ok                                   # exact: bit-identical to the oracle's global step
        assert counts == res[0][2]                  # every rank sees the same global counts
        assert abs(loss - want_loss) < 1e-6


def test_exchange_sink_slots_follow_the_flat_gradient_layout():
    """ops.set_exchange_sink: a gradient view of the flat fp32 buffer maps to the int64 slots at the
    same element offsets (the exact layer-wise exchange); a tensor outside the buffer is refused."""
    from lbt_amd.dfxp import ops
    g = torch.zeros(100, dtype=torch.float32)
    x = torch.zeros(100 + 7, dtype=torch.int64)
    ops.set_exchange_sink(g, 100, x, loss_off=106, world=4)
    try:
        assert ops._num(g[10:30]).value == x.data_ptr() + 8 * 10
        assert ops._num(g).value == x.data_ptr()
        assert ops._XSINK["loss"] == x.data_ptr() + 8 * 106 and ops._XSINK["world"] == 4
        with pytest.raises(RuntimeError):
            ops._num(torch.zeros(4))
        with pytest.raises(RuntimeError):
            ops._num(torch.zeros(200)[:101])
    finally:
        ops.set_exchange_sink()
    assert ops._num(g) is None


def _bench_params(model, seed=0):
    """bench.py cpu_baseline's initialisation: uniform(+-sqrt(3 / fan_in)) weights, gamma 1, beta 0."""
    rng = np.random.default_rng(seed)
    params = {}
    for name, owner in model.params():
        if name.endswith("/W"):
            shp = owner.ksize if hasattr(owner, "ksize") else (owner.in_units, owner.units)
            lim = np.sqrt(3 / float(np.prod(shp[:-1])))
            params[name] = rng.uniform(-lim, lim, size=shp).astype(np.float32)
        elif name.endswith("/g"):
            params[name] = np.ones(owner.C, np.float32)
        else:
            params[name] = np.zeros(owner.C, np.float32)
    return params


def _global_batch(B, seed=7):
    xr = np.random.default_rng(seed)
    X = ((xr.integers(0, 256, size=(B, 32, 32, 3)) - 127.5) / 128).astype(np.float32)
    return X, xr.integers(0, 10, size=B)


def _sworker(rank, world, port, per, out_q):
    """configs[2]'s partition on CPU: the ResNet-20 step of a global batch of world * per images, rank r
    taking images [r*per, (r+1)*per) (bench.py --global-batch), in SyncBN mode: every Normalization_q's
    exact integer statistics go through ONE int64 gloo all-reduce in the build's sharded layout
    (NSHARD x [S1 | S2] per channel, what FusedResNet(sync_bn=True)._allreduce sums), then the step's exact
    exchange (lbt_amd.distributed.make_exchange) and the dequantised update on every rank."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from threadpoolctl import threadpool_limits
    threadpool_limits(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lbt_amd import distributed as D
        from lbt_amd._lib import NSHARD
        from oracle import nn
        from oracle import resnet as R
        model = R.build_resnet((3, 3, 3), 8, 2e-4)
        params = _bench_params(model)
        R.set_params(model, params)
        ranges = R.init_ranges(model)
        X, Y = _global_batch(world * per)
        x, y = X[rank * per:(rank + 1) * per], Y[rank * per:(rank + 1) * per]
        ncoll = [0]

        def sync(a, b, n):
            C = a.shape[0]
            t = torch.zeros(NSHARD, 2 * C, dtype=torch.int64)
            k = (rank * 5 + ncoll[0]) % NSHARD  # a rank's sums land in some shard slot, as workgroup ids do
            t[k, :C] = torch.from_numpy(a.astype(np.int64))
            t[k, C:] = torch.from_numpy(b.astype(np.int64))
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            ncoll[0] += 1
            t = t.sum(0).numpy()
            return t[:C], t[C:], n * world  # every rank holds per * H * W elements per channel
        nn.SYNC = sync
        try:
            loss, _, _, ctx = R.forward_backward(model, ranges, x, y, step=0, seed=0, norm=world * per)
        finally:
            nn.SYNC = None
        num = R._numerators(model)
        keys = sorted(num)
        names = sorted(ctx.counts)
        n = sum(num[k][1].size for k in keys)
        buf, xc = D.make_exchange(n, len(names), "cpu")
        off = 0
        for k in keys:
            v = num[k][1].ravel()
            buf[off:off + v.size] = torch.from_numpy(v.astype(np.int64))
            off += v.size
        for i, k in enumerate(names):
            buf[xc.cnt_off + 2 * i] = ctx.counts[k][0]
            buf[xc.cnt_off + 2 * i + 1] = ctx.counts[k][1]
        buf[xc.loss_off] = int(round(loss * 2 ** 32))
        D.allreduce_comm(buf)
        got, off = {}, 0
        for k in keys:
            kind, S, sc, owner = num[k]
            tot = buf[off:off + S.size].numpy().reshape(S.shape)
            off += S.size
            if kind == "w":
                got[k] = (R.nn.scale_int(tot, sc) + (np.float32(2 * owner.wd) * params[k]).astype(np.float32)).astype(np.float32)
            elif kind == "g":
                got[k] = ((tot.astype(np.float64) * sc).astype(np.float32)
                          + (np.float32(2 * owner.wd) * params[k]).astype(np.float32)).astype(np.float32)
            else:
                got[k] = (tot.astype(np.float64) * sc).astype(np.float32)
        zero = {k: np.zeros_like(v) for k, v in params.items()}
        new_p, _ = R.sgd_momentum(params, got, zero, 1e-2, 0.9)
        new_r = dict(ranges)
        for i, k in enumerate(names):
            c1, c2 = int(buf[xc.cnt_off + 2 * i]), int(buf[xc.cnt_off + 2 * i + 1])
            new_r[k] = R.dfxp.update_range_from_counts(c1, c2, ctx.counts[k][2] * world, 0.0, ctx.counts[k][3], ranges[k])
        bn = [(l.mean_running, l.var_running) for l in R._walk(model) if isinstance(l, nn.NormQ)]
        out_q.put((rank, new_p, new_r, bn, float(buf[xc.loss_off]) / 2 ** 32, ncoll[0]))
    finally:
        dist.destroy_process_group()


def test_syncbn_partition_world8_equals_one_process_gloo():
    """configs[2] (ResNet-20, global batch 128 over 8 ranks = 16 images each) with the reference's
    whole-batch BatchNorm statistics (dynamic_fixed_point.py:588, trainer.py:34): 8 gloo ranks, each
    with its shard, the SyncBN statistics all-reduces and the exact int64 gradient exchange, end the step
    with weights, exponents and BN running averages BIT-IDENTICAL to one process stepping on all 128
    images (oracle.resnet.train_step); the loss (2^-32 fixed point in the exchange) to 1e-6."""
    from threadpoolctl import threadpool_limits
    from oracle import nn
    from oracle import resnet as R
    world, per = 8, 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sworker, args=(r, world, port, per, q)) for r in range(world)]
    for p in procs:
        p.start()
    # meanwhile: the single-process step on the whole batch
    model = R.build_resnet((3, 3, 3), 8, 2e-4)
    params = _bench_params(model)
    state = dict(params=params, accum={k: np.zeros_like(v) for k, v in params.items()},
                 ranges=R.init_ranges(model), step=0)
    X, Y = _global_batch(world * per)
    with threadpool_limits(1):
        want_loss, want, _ = R.train_step(model, state, X, Y, lr=1e-2, momentum=0.9, seed=0)
    want_bn = [(l.mean_running, l.var_running) for l in R._walk(model) if isinstance(l, nn.NormQ)]
    res = sorted([q.get(timeout=600) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(want_bn) == 21
    for rank, new_p, new_r, bn, loss, ncoll in res:
        assert ncoll == 2 * 21  # every Normalization_q: its forward moments and its backward sums
        for k in want["params"]:
            assert np.array_equal(new_p[k], want["params"][k]), (rank, k)
        assert new_r == want["ranges"], rank
        for (m, v), (wm, wv) in zip(bn, want_bn):
            assert np.array_equal(m, wm) and np.array_equal(v, wv), rank
        assert abs(loss - want_loss) < 1e-6, (rank, loss, want_loss)
