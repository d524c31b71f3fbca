"""Per-process spread of the timed step (diagnostics): python tools/process_spread.py [--reps 5] [--steps 100].
Builds the bench's ResNet-20 fused trainer as bench.py does and times `reps` consecutive regions of `steps`
steps (synchronize on both sides) in ONE process; prints one JSON line. Run it in several processes to
separate a slow process (placement) from a slow moment (clocks)."""
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
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--steps", type=int, default=100)
    args = ap.parse_args()
    from lbt_amd.fused import FusedResNet
    from lbt_amd.models import CIFAR10_Resnet20
    from lbt_amd.runtime import DfxpContext
    from lbt_amd.trainer import Trainer
    dev = torch.device("cuda", 0)
    ctx = DfxpContext(device=dev, seed=0, world_size=1)
    model = FusedResNet(CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctx, grad_range=-6))
    xs, ys = bench.synthetic_batches(4, 128, seed=1000, device=dev)
    tr = Trainer(model, lr=1e-2, momentum=0.9, batch_size=128, use_graph=True)
    tr.init_model()
    for x, y in zip(xs, ys):
        tr.prepare(x, y)
    out, i = [], 0
    for _ in range(20):
        tr.step(xs[i % 4], ys[i % 4])
        i += 1
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            tr.step(xs[i % 4], ys[i % 4])
            i += 1
        torch.cuda.synchronize()
        out.append(round(1e3 * (time.perf_counter() - t0) / args.steps, 4))
    print(json.dumps({"ms_per_step": out, "x_ptr": hex(xs[0].data_ptr())}), flush=True)


if __name__ == "__main__":
    main()
