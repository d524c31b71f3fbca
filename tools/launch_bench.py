"""Per-launch device time of the fused ResNet-20 step, each launch timed in isolation (diagnostics).

    python tools/launch_bench.py [--batch B] [--reps R] [--filter SUBSTR]

Every prebuilt launch of the plan (forward, fused head, backward, tail) is captured R times into a
HIP graph and replayed between two events: per-launch time without event or host gaps (the
launch's inputs are what the previous step left, so caches are warm as in the replayed step).
The parameters / exponents / counters / BN running statistics are restored afterwards.
Environment switches of the plan (LBT_FUSE_WGRAD=0 ...) select what is timed.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from lbt_amd.fused import FusedResNet  # noqa: E402
from lbt_amd.models import CIFAR10_Resnet20  # noqa: E402
from lbt_amd.roofline import graph_launches, time_launches  # noqa: E402
from lbt_amd.runtime import DfxpContext  # noqa: E402
from lbt_amd.trainer import Trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--filter", default="")
    ap.add_argument("--w4", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = DfxpContext(device=dev, seed=0)
    model = FusedResNet(CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctx, weight_bits=4 if a.w4 else None))
    xs, ys = bench.synthetic_batches(1, a.batch, seed=1000, device=dev)
    tr = Trainer(model, lr=1e-2, momentum=0.9, batch_size=a.batch, use_graph=True)
    tr.init_model()
    for _ in range(3):
        tr.step(xs[0], ys[0])
    torch.cuda.synchronize()
    launches = [f for f in graph_launches(model) if a.filter in getattr(f, "kname", "")]
    res = time_launches(tr, launches, reps=a.reps)
    tot = 0.0
    for i, (f, us) in enumerate(zip(launches, res)):
        tot += us
        print("%3d %8.2f  %s" % (i, us, f.kname))
    print("sum %.1f us over %d launches" % (tot, len(launches)))
    # the whole step, graph-replayed back to back (what bench.py times)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        tr.step(xs[0], ys[0])
    e1.record()
    e1.synchronize()
    print("step %.1f us (graph replay, 50 steps)" % (1000.0 * e0.elapsed_time(e1) / 50))


if __name__ == "__main__":
    main()
