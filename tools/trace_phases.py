"""Per-workgroup phase timestamps of single launches of the fused ResNet-20 step (kernel studies).

    python tools/trace_phases.py --build              # here: the -DLBT_TRACE build of the library
    python tools/trace_phases.py [--filter K] [--batch B]   # GPU: trace every launch whose kname has K

Kernels mark phases with LBT_TS(i) (dfxp_device.h): thread 0 of each workgroup stores
s_memrealtime (100 MHz) into trace[wg*8 + i], slot 7 = XCC id. For each traced launch this prints
the kernel span, the spread of workgroup start times and the median / p90 duration of every phase.
"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
TRACE_DIR = os.path.join(ROOT, "lbt_amd", "build_trace")
TRACE_LIB = os.path.join(TRACE_DIR, "liblbt_dfxp_trace.so")


def build():
    sys.path.insert(0, ROOT)
    from lbt_amd import _build
    os.makedirs(TRACE_DIR, exist_ok=True)
    objs = []
    import concurrent.futures

    def one(src):
        obj = os.path.join(TRACE_DIR, os.path.basename(src) + ".o")
        subprocess.check_call([_build.HIPCC] + _build.FLAGS + ["-DLBT_TRACE", "-c", src, "-o", obj])
        return obj
    with concurrent.futures.ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(one, _build.sources()))
    subprocess.check_call([_build.HIPCC, "--offload-arch=" + _build.ARCH, "-shared", "-fPIC", "-o", TRACE_LIB] + objs)
    print(TRACE_LIB)


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))] if v else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--filter", default="conv_bwd_kernel")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--max", type=int, default=40)
    ap.add_argument("--lib", default=None, help="another -DLBT_TRACE build (tools/build_variant.py)")
    ap.add_argument("--cold", action="store_true",
                    help="write 512 MB inside the replayed graph before the launch, so its loads miss L2 and the "
                         "256 MB last-level cache as they do in the step (isolated replays re-read warm caches)")
    a = ap.parse_args()
    if a.build:
        return build()
    os.environ["LBT_LIBRARY"] = a.lib or TRACE_LIB
    sys.path.insert(0, ROOT)
    import torch
    import bench
    from lbt_amd import _lib
    from lbt_amd.fused import FusedResNet
    from lbt_amd.models import CIFAR10_Resnet20
    from lbt_amd.runtime import DfxpContext
    from lbt_amd.trainer import Trainer
    dev = torch.device("cuda", 0)
    ctx = DfxpContext(device=dev, seed=0)
    model = FusedResNet(CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctx))
    xs, ys = bench.synthetic_batches(1, a.batch, seed=1000, device=dev)
    tr = Trainer(model, lr=1e-2, momentum=0.9, batch_size=a.batch, use_graph=False)
    tr.init_model()
    for _ in range(3):
        tr.step(xs[0], ys[0])
    torch.cuda.synchronize()
    lib = _lib.load()
    setters = [getattr(lib, "lbt_trace_set_" + t) for t in ("conv", "bn", "head", "stem", "batched") if hasattr(lib, "lbt_trace_set_" + t)]
    for s in setters:
        s.argtypes = [ctypes.c_void_p]
    nwg_max = 1 << 15
    buf = torch.zeros(nwg_max * 8, dtype=torch.int64, device=dev)
    from lbt_amd.roofline import graph_launches
    launches = [f for f in graph_launches(model) if a.filter in getattr(f, "kname", "")]
    side = torch.cuda.Stream(device=dev)
    flush = torch.empty(1 << 27, dtype=torch.float32, device=dev) if a.cold else None
    for idx, f in enumerate(launches[:a.max]):
        # the launch replayed from a graph (as in the timed step), twice: the second one is traced
        g = torch.cuda.CUDAGraph()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            with torch.cuda.graph(g, stream=side):
                if flush is not None:
                    flush.fill_(float(idx))
                f()
        torch.cuda.current_stream().wait_stream(side)
        g.replay()
        buf.zero_()
        torch.cuda.synchronize()
        for s in setters:
            s(ctypes.c_void_p(buf.data_ptr()))
        g.replay()
        torch.cuda.synchronize()
        for s in setters:
            s(None)
        t = buf.view(nwg_max, 8).cpu().numpy()
        live = t[:, 0] != 0
        t = t[live]
        if not len(t):
            print("%2d %s: no trace" % (idx, f.kname))
            continue
        T0 = t[:, 0].min()
        groups = [("all", t)]
        if (t[:, 6] != 0).any():  # slot 6 = job index / role + 1: one line per job, phases 0..3
            for jid in sorted(set(t[:, 6].tolist())):
                tj = t[t[:, 6] == jid].copy()
                tj[:, 6] = 0
                report(idx, "%s:job%d" % (f.kname, jid - 1), tj, T0)
            continue
        has5 = t[:, 5] != 0
        if has5.any() and not has5.all():  # two workgroup roles (e.g. deferred wgrad + dgrad tiles)
            groups = [("A", t[~has5]), ("B", t[has5])]
        for gname, tt in groups:
            report(idx, f.kname + ":" + gname, tt, T0)


def report(idx, name, t, T0):
    if True:
        t0 = T0
        last = t[:, :7].max(axis=1)
        span = (last.max() - t0) * 0.01
        starts = (t[:, 0] - t0) * 0.01
        dur = (last - t[:, 0]) * 0.01
        ph = []
        for k in range(1, 7):
            m = (t[:, k] != 0) & (t[:, k - 1] != 0)
            if m.sum() == 0:
                continue
            d = (t[m, k] - t[m, k - 1]) * 0.01
            ph.append("p%d %.2f/%.2f(%d)" % (k, pct(d, 0.5), pct(d, 0.9), m.sum()))
        print("%2d %-24s wg %5d span %6.2f us  start med %5.2f max %5.2f  wg dur med %5.2f p90 %5.2f | %s" % (
            idx, name[:24], len(t), span, pct(starts, 0.5), starts.max(), pct(dur, 0.5), pct(dur, 0.9), " ".join(ph)))


if __name__ == "__main__":
    main()
