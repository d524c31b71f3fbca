"""Isolated timings of the batched weight-gradient launch (lbt_conv_wgrad_many_i8) of the ResNet-20
fused plan, per job and for job subsets (kernel studies, GPU):

    python tools/wgrad_probe.py [--batch B] [--reps R]

Each timed launch is captured R times into one HIP graph and replayed between two events on the
launch's stream (tools/launch_bench.py's method); the jobs are the plan's own (lbt_wgrad_job array).
Prints one line per subset: jobs, workgroups, us per launch.
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch

    import bench
    from lbt_amd import _lib
    from lbt_amd._lib import WgradJob
    from lbt_amd.fused import FusedResNet
    from lbt_amd.models import CIFAR10_Resnet20
    from lbt_amd.runtime import DfxpContext
    from lbt_amd.trainer import Trainer
    dev = torch.device("cuda", 0)
    ctx = DfxpContext(device=dev, seed=0)
    model = FusedResNet(CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctx, grad_range=-6))
    xs, ys = bench.synthetic_batches(1, a.batch, seed=1000, device=dev)
    tr = Trainer(model, lr=1e-2, momentum=0.9, batch_size=a.batch, use_graph=False)
    tr.init_model()
    for _ in range(2):
        tr.step(xs[0], ys[0])
    torch.cuda.synchronize()
    arrs = [k for k in model._keep if isinstance(k, ctypes.Array) and k._type_ is WgradJob]
    assert arrs, "no batched weight-gradient job array in the plan"
    jobs = list(arrs[-1])
    lib = _lib.load()
    side = torch.cuda.Stream(device=dev)

    def time_launch(js):
        arr = (WgradJob * len(js))(*js)
        g = torch.cuda.CUDAGraph()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            with torch.cuda.graph(g, stream=side):
                for _ in range(a.reps):
                    rc = lib.lbt_conv_wgrad_many_i8(ctypes.byref(arr), len(js), ctypes.c_void_p(side.cuda_stream))
                    assert rc == 0, rc
        torch.cuda.current_stream().wait_stream(side)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(5):
            e0.record(side)
            with torch.cuda.stream(side):
                g.replay()
            e1.record(side)
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1000.0 / a.reps)
        return best

    def desc(j):
        d = j.d
        return "%dx%d/%d %d->%d %dx%d split %d" % (d.KH, d.KW, d.SH, d.Cin, d.Cout, d.H, d.W, j.nsplit)

    print("batch %d, %d jobs" % (a.batch, len(jobs)))
    print("all jobs: %.2f us" % time_launch(jobs))
    for i, j in enumerate(jobs):
        print("job %2d %-28s %.2f us" % (i, desc(j), time_launch([j])))
    s1 = [j for j in jobs if j.d.Cin == 16 and j.d.Cout == 16]
    if s1:
        print("stage-1 jobs (%d): %.2f us" % (len(s1), time_launch(s1)))
    rest = [j for j in jobs if not (j.d.Cin == 16 and j.d.Cout == 16)]
    if rest:
        print("other jobs (%d): %.2f us" % (len(rest), time_launch(rest)))


if __name__ == "__main__":
    main()
