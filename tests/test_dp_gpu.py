"""The Trainer's data-parallel path on the MI355X (VERDICT r1 "next" 1 and 5).

Two or eight ranks are spawned as fresh processes; all use the gloo backend and share cuda:0 (a
one-GPU rehearsal of the RCCL path: the same Trainer code -- captured graphs, lbt_step_reduce_x,
the int64 all-reduce, lbt_step_finish, lbt_dfxp_range_update_x -- only the collective's transport
differs). Every rank takes 16 images of a global batch of B = 16 * world images; world 8 at B = 128
is BASELINE configs[2]'s partition of the bench batch.

* per-rank BatchNorm (standard DDP, the bench's mode), graph-captured: after every step the weights,
  the dequantised gradients and the exponents equal the ORACLE's world-shard step
  (oracle.resnet.dp_train_step: per-shard forward / backward with the global-batch loss, integer
  numerators and overflow counts summed, one dequantisation) BIT FOR BIT, given each rank's
  d loss / d logits (the softmax is the one op that is not bit-exact; the loss is compared at 1e-5).
* SyncBN (FusedResNet(sync_bn=True)): every rank's weights, exponents and BN running statistics
  equal a SINGLE process training on the whole batch B bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
STEPS = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _state(tr, ctx, m):
    bn = [(n.X_mean_running.cpu().numpy().copy(), n.X_var_running.cpu().numpy().copy()) for n in _norms(m)]
    return dict(loss=float(m.loss.item()), dz=m.dlogits.cpu().numpy().copy(), w=tr.flat.w.cpu().numpy().copy(),
                g=tr.flat.g.cpu().numpy().copy(), ranges=ctx.ranges(), bn=bn)


def _norms(m):
    from lbt_amd.dfxp.layers import Normalization_q
    out = []

    def walk(layer):
        if isinstance(layer, Normalization_q):
            out.append(layer)
        for attr in ("layers", "residual", "shortcut"):
            sub = getattr(layer, attr, None)
            if sub is not None:
                for s in (sub if isinstance(sub, (list, tuple)) else [sub]):
                    walk(s)
    for layer in m.model.layers:
        walk(layer)
    return out


def _batches(B):
    import bench
    xs, ys = bench.synthetic_batches(STEPS, B, 1000, "cpu")
    return xs, ys


def _make(world, sync, B, force=False, exchange=None):
    from lbt_amd.fused import FusedResNet
    from lbt_amd.models import CIFAR10_Resnet20
    from lbt_amd.runtime import DfxpContext
    from lbt_amd.trainer import Trainer
    ctx = DfxpContext(device="cuda:0", seed=0, world_size=world)
    m = FusedResNet(CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctx), sync_bn=sync, force_sync_bn=force)
    return ctx, m, Trainer(m, lr=1e-2, momentum=0.9, batch_size=B // world, use_graph=True, exchange=exchange)


def _worker(rank, world, port, sync, B, out_q, backend="gloo", force=False):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        ctx, m, tr = _make(world, sync, B, force=force, exchange=True if force else None)
        if force:  # the captured-collective path must be the one that ran
            assert tr.dp and tr.capture_comm and m.sync_bn == sync, (tr.dp, tr.capture_comm, m.sync_bn)
        xs, ys = _batches(B)
        b = B // world
        xr = [x[rank * b:(rank + 1) * b].contiguous().cuda() for x in xs]  # kept alive: graphs read them
        yr = [y[rank * b:(rank + 1) * b].contiguous().cuda() for y in ys]
        rec = []
        for i in range(STEPS):
            tr.step(xr[i], yr[i])
            torch.cuda.synchronize()
            rec.append(_state(tr, ctx, m))
        if force:  # one graph per step: the exchange (and SyncBN's sums) captured inside it
            assert tr._graphs is not None and tr._graphs[1] is None
        out_q.put((rank, rec))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        out_q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _run_ranks(sync, B, world=2, backend="gloo", force=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sync, B, q, backend, force)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0, p.exitcode
    for r, rec in res:
        assert not isinstance(rec, str), rec
    return [rec for _, rec in res]


def _gpu_params(m):
    out = {}
    for owner, var, _ in m.param_slots():
        out[owner.name + {"W": "/W", "gamma": "/g", "beta": "/b"}[var]] = getattr(owner, var).detach().cpu().numpy().copy()
    return out


def _flat_to_dict(m, flat_vals, offsets):
    out = {}
    for owner, var, off, sz in offsets:
        key = owner.name + {"W": "/W", "gamma": "/g", "beta": "/b"}[var]
        out[key] = flat_vals[off:off + sz].reshape(getattr(owner, var).shape)
    return out


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 8])
def test_dp_ranks_local_bn_match_oracle_shard_step(world):
    """world 2 (B = 32) and world 8 (B = 128, configs[2]'s partition: 16 images per rank of the bench's
    batches): every rank's weights / gradients / exponents after every step equal the oracle's
    world-shard step bit for bit."""
    from oracle import resnet as oresnet
    B = 16 * world
    recs = _run_ranks(False, B, world=world)
    for s in zip(*recs):  # identical model on every rank
        for o in s[1:]:
            assert np.array_equal(s[0]["w"], o["w"]) and s[0]["ranges"] == o["ranges"]
            assert np.array_equal(s[0]["g"], o["g"])
    # the oracle's shard step, fed each rank's d loss / d logits
    _, m, tr = _make(1, False, B)  # same seed -> same initial parameters, and the flat layout
    om = oresnet.build_resnet((3, 3, 3), 8, 2e-4)
    params = _gpu_params(m)
    state = dict(params=params, accum={k: np.zeros_like(v) for k, v in params.items()},
                 ranges=oresnet.init_ranges(om), step=0)
    xs, ys = _batches(B)
    b = B // world
    for i in range(STEPS):
        shards = [(xs[i][r * b:(r + 1) * b].numpy(), ys[i][r * b:(r + 1) * b].numpy()) for r in range(world)]
        loss, new_state, ctxs = oresnet.dp_train_step(om, state, shards, seed=0, dzs=[rec[i]["dz"] for rec in recs])
        # each rank's dz is its rows of the global-batch softmax gradient (rtol: expf / logf)
        for r, c in enumerate(ctxs):
            np.testing.assert_allclose(recs[r][i]["dz"], c.dz, rtol=1e-5, atol=1e-9)
        assert abs(recs[0][i]["loss"] - loss) <= 1e-5 * abs(loss), (i, recs[0][i]["loss"], loss)
        got_w = _flat_to_dict(m, recs[0][i]["w"], tr.flat.offsets)
        for k in new_state["params"]:
            assert np.array_equal(got_w[k], new_state["params"][k]), (i, k)
        assert recs[0][i]["ranges"] == new_state["ranges"], i
        state = new_state


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 8])
def test_dp_ranks_syncbn_equal_single_process_batch(world):
    """SyncBN over world ranks of 16 images == ONE process on the whole batch (world 8: configs[2]'s
    8 x 16 partition of the reference's B = 128 step, trainer.py:34,144-162, with the whole-batch
    moments of dynamic_fixed_point.py:588): weights, gradients, exponents, BN running statistics
    bit for bit after every step, and each rank's dz rows are the single process's."""
    B = 16 * world
    recs = _run_ranks(True, B, world=world)
    ctx, m, tr = _make(1, False, B)
    xs, ys = _batches(B)
    xg = [x.cuda() for x in xs]
    yg = [y.cuda() for y in ys]
    for i in range(STEPS):
        tr.step(xg[i], yg[i])
        torch.cuda.synchronize()
        ref = _state(tr, ctx, m)
        for s in (rec[i] for rec in recs):
            assert np.array_equal(s["w"], ref["w"]), i
            assert np.array_equal(s["g"], ref["g"]), i
            assert s["ranges"] == ref["ranges"], i
            for (ma, va), (mb, vb) in zip(s["bn"], ref["bn"]):
                assert np.array_equal(ma, mb) and np.array_equal(va, vb), i
        assert np.array_equal(np.concatenate([rec[i]["dz"] for rec in recs]), ref["dz"]), i


@pytest.mark.parametrize("sync", [False, True])
def test_captured_rccl_collectives_world1_equal_plain_step(sync):
    """The nccl (= RCCL) path with its collectives CAPTURED in the step's HIP graph (Trainer
    capture_comm): one rank, so every all-reduce is the identity and the step -- exchange buffer,
    lbt_step_finish, range update from the exchanged counters, and with SyncBN the 42 statistics
    all-reduces inside the graph -- must equal the plain single-process step bit for bit. (Two RCCL
    ranks cannot share one GPU; the N-rank sums themselves are covered by the gloo tests above.)"""
    B = 32
    (r0,) = _run_ranks(sync, B, world=1, backend="nccl", force=True)
    ctx, m, tr = _make(1, False, B)
    xs, ys = _batches(B)
    xg = [x.cuda() for x in xs]
    yg = [y.cuda() for y in ys]
    for i in range(STEPS):
        tr.step(xg[i], yg[i])
        torch.cuda.synchronize()
        ref = _state(tr, ctx, m)
        s = r0[i]
        assert np.array_equal(s["w"], ref["w"]), i
        assert np.array_equal(s["g"], ref["g"]), i
        assert s["ranges"] == ref["ranges"], i
        assert abs(s["loss"] - ref["loss"]) <= 1e-6 * abs(ref["loss"]), i  # 2^-32 fixed-point loss sum
        for (ma, va), (mb, vb) in zip(s["bn"], ref["bn"]):
            assert np.array_equal(ma, mb) and np.array_equal(va, vb), i
