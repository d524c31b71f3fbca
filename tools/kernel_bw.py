"""Per-launch algorithmic bandwidth of one eager training step (diagnostics).

    python tools/kernel_bw.py [--workload resnet50|resnet20] [--batch B] [--detail KERNEL ...]

Every wrapped launch is bracketed by HIP events (lbt_amd.dfxp.ops.PROFILE, as bench.py's roofline);
prints per kernel: launches, us/step, average GB/s of algorithmic bytes; --detail lists each launch
of the named kernels (bytes, us, GB/s) in issue order.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from lbt_amd.dfxp import ops  # noqa: E402
from lbt_amd.runtime import DfxpContext  # noqa: E402
from lbt_amd.trainer import Trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="resnet50")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--detail", nargs="*", default=[])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = DfxpContext(device=dev, seed=0)
    if a.workload == "resnet50":
        from lbt_amd.models import ImageNet_Resnet50
        B = a.batch or 256
        model = ImageNet_Resnet50(8, grad_bits=16, weight_decay=1e-4, ctx=ctx)
        xs, ys = bench.synthetic_imagenet(1, B, 1000, dev)
    else:
        from lbt_amd.fused import FusedResNet
        from lbt_amd.models import CIFAR10_Resnet20
        B = a.batch or 128
        model = FusedResNet(CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctx))
        xs, ys = bench.synthetic_batches(1, B, seed=1000, device=dev)
    tr = Trainer(model, lr=1e-2, momentum=0.9, batch_size=B, use_graph=False)
    tr.init_model()
    for _ in range(2):
        tr.step(xs[0], ys[0])
    torch.cuda.synchronize()
    ops.PROFILE = {}
    torch.cuda._sleep(300_000_000)
    tr._eager(xs[0], ys[0])
    torch.cuda.synchronize()
    prof, ops.PROFILE = ops.PROFILE, None
    rows = []
    for k, recs in prof.items():
        ts = [e0.elapsed_time(e1) * 1000.0 for e0, e1, _ in recs]
        bs = [b for _, _, b in recs]
        rows.append((sum(ts), k, len(recs), sum(bs) / max(sum(ts), 1e-9) / 1e3))
    rows.sort(reverse=True)
    print("%-40s %7s %10s %8s" % ("kernel", "calls", "us/step", "GB/s"))
    for t, k, n, gbs in rows:
        print("%-40s %7d %10.1f %8.0f" % (k[:40], n, t, gbs))
    for k in a.detail:
        print("\n" + k)
        for e0, e1, b in prof.get(k, []):
            us = e0.elapsed_time(e1) * 1000.0
            print("  %12d B %9.1f us %8.0f GB/s" % (b, us, b / max(us, 1e-9) / 1e3))


if __name__ == "__main__":
    main()
