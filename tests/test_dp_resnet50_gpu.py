"""Exact data parallelism of the layer-wise ResNet-50 (configs[3] at N GPUs).

The layer-wise models exchange the INTEGER numerators of every gradient (ops.set_exchange_sink: the
wgrad / dense / BN-parameter reductions write S where they would write dequant(S) + 2*wd*W,
dynamic_fixed_point.py:302,457-460,689-691), the overflow counters and the loss sum in one int64
all-reduce, then dequantise once (lbt_step_finish) -- so a step on N ranks equals the oracle's
N-shard step (oracle.resnet.dp_train_step) bit for bit, whatever order the collective sums in.

Two spawned ranks share cuda:0 over gloo (the one-GPU rehearsal of the RCCL path: same Trainer code,
only the transport differs), on reduced bottleneck configs the numpy oracle finishes in seconds:
8- and 16-bit gradients, the generic and the int8-MFMA fc, and full-width 64 (every block on the
fused bottleneck schedule with 16-bit gradients).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
STEPS = 2
B = 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches(image, classes):
    rng = np.random.default_rng(5)
    xs = [((rng.integers(0, 256, size=(B, image, image, 3)) - 127.5) / 128).astype(np.float32) for _ in range(STEPS)]
    ys = [rng.integers(0, classes, size=B).astype(np.int32) for _ in range(STEPS)]
    return xs, ys


def _make(world, cfg):
    from lbt_amd.models import ImageNet_Resnet
    from lbt_amd.runtime import DfxpContext
    from lbt_amd.trainer import Trainer
    blocks, width, image, classes, grad_bits = cfg
    ctx = DfxpContext(device="cuda:0", seed=1, world_size=world)
    gm = ImageNet_Resnet(8, blocks, grad_bits=grad_bits, width=width, classes=classes, image=image,
                         weight_decay=1e-4, ctx=ctx)
    return ctx, gm, Trainer(gm, lr=1e-2, momentum=0.9, batch_size=B // world, use_graph=True)


def _worker(rank, world, port, cfg, out_q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx, gm, tr = _make(world, cfg)
        assert tr.dp and tr._lw_exact and tr.comm is None, "the exact layer-wise exchange must be the one in use"
        xs, ys = _batches(cfg[2], cfg[3])
        b = B // world
        xr = [torch.from_numpy(x[rank * b:(rank + 1) * b].copy()).cuda() for x in xs]
        yr = [torch.from_numpy(y[rank * b:(rank + 1) * b].copy()).cuda() for y in ys]
        rec = []
        for i in range(STEPS):
            tr.step(xr[i], yr[i])
            torch.cuda.synchronize()
            rec.append(dict(loss=float(gm.loss.item()), dz=gm.dlogits.cpu().numpy().copy(),
                            w=tr.flat.w.cpu().numpy().copy(), g=tr.flat.g.cpu().numpy().copy(), ranges=ctx.ranges()))
        out_q.put((rank, rec))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        out_q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _run(cfg, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0, p.exitcode
    for _, rec in res:
        assert not isinstance(rec, str), rec
    return [rec for _, rec in res]


def _flat_to_dict(flat_vals, offsets):
    out = {}
    for owner, var, off, sz in offsets:
        out[owner.name + {"W": "/W", "gamma": "/g", "beta": "/b"}[var]] = flat_vals[off:off + sz].reshape(
            getattr(owner, var).shape)
    return out


@pytest.mark.parametrize("cfg", [((1, 1, 1, 1), 8, 32, 10, 8), ((1, 1, 1, 1), 8, 32, 16, 16),
                                 ((1, 1, 1, 1), 64, 32, 16, 16)])
def test_resnet50_two_ranks_equal_oracle_two_shard_step(cfg):
    from oracle import resnet as oresnet
    blocks, width, image, classes, grad_bits = cfg
    r0, r1 = _run(cfg)
    for s0, s1 in zip(r0, r1):  # one model on both ranks
        assert np.array_equal(s0["w"], s1["w"]) and np.array_equal(s0["g"], s1["g"]) and s0["ranges"] == s1["ranges"]
    _, gm, tr = _make(1, cfg)  # same seed: the same initial parameters and flat layout
    om = oresnet.build_resnet50(blocks, width, classes, 8, grad_bits, weight_decay=1e-4)
    params = {}
    for owner, var, _ in gm.param_slots():
        params[owner.name + {"W": "/W", "gamma": "/g", "beta": "/b"}[var]] = getattr(owner, var).detach().cpu().numpy()
    state = dict(params=params, accum={k: np.zeros_like(v) for k, v in params.items()},
                 ranges=oresnet.init_ranges(om), step=0)
    xs, ys = _batches(image, classes)
    b = B // 2
    for i in range(STEPS):
        shards = [(xs[i][r * b:(r + 1) * b], ys[i][r * b:(r + 1) * b]) for r in range(2)]
        loss, new_state, ctxs = oresnet.dp_train_step(om, state, shards, seed=1, dzs=[r0[i]["dz"], r1[i]["dz"]])
        for r, c in enumerate(ctxs):  # each rank's rows of the GLOBAL-batch softmax gradient
            np.testing.assert_allclose((r0, r1)[r][i]["dz"], c.dz, rtol=1e-5, atol=1e-9)
        assert abs(r0[i]["loss"] - loss) <= 1e-5 * abs(loss), (i, r0[i]["loss"], loss)
        got = _flat_to_dict(r0[i]["w"], tr.flat.offsets)
        for k in new_state["params"]:
            assert np.array_equal(got[k], new_state["params"][k]), (i, k)
        assert r0[i]["ranges"] == new_state["ranges"], i
        state = new_state
