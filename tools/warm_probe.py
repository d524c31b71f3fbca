"""How the timed window's length and position move ms/step (the driver times --steps 20 --warmup 5).

Builds the bench's ResNet-20 fused trainer exactly as bench.py does, then times consecutive windows of
K steps (barrier-free, synchronize on both sides, perf_counter) from the first step after capture, and
prints one JSON line per window: the window index, steps, ms/step. Run: python tools/warm_probe.py
[--windows 40] [--k 20]."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=40)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--batch", type=int, default=128)
    args = ap.parse_args()
    from lbt_amd.fused import FusedResNet
    from lbt_amd.models import CIFAR10_Resnet20
    from lbt_amd.runtime import DfxpContext
    from lbt_amd.trainer import Trainer
    dev = torch.device("cuda", 0)
    ctx = DfxpContext(device=dev, seed=0, world_size=1)
    model = FusedResNet(CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctx, grad_range=-6))
    xs, ys = bench.synthetic_batches(4, args.batch, seed=1000, device=dev)
    tr = Trainer(model, lr=1e-2, momentum=0.9, batch_size=args.batch, use_graph=True)
    tr.init_model()
    for x, y in zip(xs, ys):
        tr.prepare(x, y)
    torch.cuda.synchronize()
    i = 0
    for w in range(args.windows):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.k):
            tr.step(xs[i % 4], ys[i % 4])
            i += 1
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(json.dumps({"window": w, "steps_before": i - args.k, "k": args.k,
                          "ms_per_step": round(1e3 * el / args.k, 4)}), flush=True)
    # host cost of one replay call with the GPU busy (the step's submit path)
    t0 = time.perf_counter()
    for _ in range(200):
        tr.step(xs[i % 4], ys[i % 4])
        i += 1
    host = (time.perf_counter() - t0) / 200
    torch.cuda.synchronize()
    print(json.dumps({"host_submit_us_per_step": round(1e6 * host, 2)}), flush=True)


if __name__ == "__main__":
    main()
