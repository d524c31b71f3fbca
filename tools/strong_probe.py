"""Strong-scaling pieces of configs[2] on ONE GPU.

  python tools/strong_probe.py [--steps K] [--out FILE]

1. the fused ResNet-20 plan's step time at per-GPU batches 16 / 32 / 64 / 128 (no collectives) --
   the per-rank compute of an 8-way strong run of global batch 128 / 256 / 512 / 1024;
2. at world size 1 over RCCL (nccl backend, one rank): the same step with the exact gradient
   exchange captured in the graph (one int64 all-reduce), and with SyncBN's statistics
   all-reduces as well (42 more collectives) -- what the collectives cost on the critical path
   when the transport is free (a one-rank all-reduce moves no bytes over xGMI).
Prints one JSON object (and writes it to --out).
"""
import argparse
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(trainer, xs, ys, steps, warmup=20):
    for i in range(warmup):
        trainer.step(xs[i % len(xs)], ys[i % len(ys)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        trainer.step(xs[i % len(xs)], ys[i % len(ys)])
    torch.cuda.synchronize()
    return 1000.0 * (time.perf_counter() - t0) / steps


def _run(B, steps, sync=False, exchange=None, comm=False):
    import bench
    from lbt_amd.fused import FusedResNet
    from lbt_amd.models import CIFAR10_Resnet20
    from lbt_amd.runtime import DfxpContext
    from lbt_amd.trainer import Trainer
    ctx = DfxpContext(device="cuda:0", seed=0, world_size=1)
    m = FusedResNet(CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctx), sync_bn=sync, force_sync_bn=sync)
    tr = Trainer(m, lr=1e-2, momentum=0.9, batch_size=B, use_graph=True, exchange=exchange)
    if comm:
        assert tr.dp and tr.capture_comm and m.sync_bn == sync
    xs, ys = bench.synthetic_batches(4, B, 1000, "cuda:0")
    ms = _time(tr, xs, ys, steps)
    return {"per_gpu_batch": B, "ms_per_step": round(ms, 4), "samples_per_s": round(B / ms * 1000.0, 1),
            "launches": getattr(m, "n_launches", None)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    res = {"plain": [], "rccl_world1_exchange": [], "rccl_world1_syncbn": []}
    for B in (16, 32, 64, 128):
        res["plain"].append(_run(B, a.steps))
        print(json.dumps(res["plain"][-1]), flush=True)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(s.getsockname()[1])
    s.close()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        for B in (16, 128):
            res["rccl_world1_exchange"].append(_run(B, a.steps, exchange=True, comm=True))
            print(json.dumps(res["rccl_world1_exchange"][-1]), flush=True)
            res["rccl_world1_syncbn"].append(_run(B, a.steps, sync=True, exchange=True, comm=True))
            print(json.dumps(res["rccl_world1_syncbn"][-1]), flush=True)
    finally:
        dist.destroy_process_group()
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
