"""Live roofline of the dominant kernel of the training step (used by bench.py).

One eager training step is run with every wrapped launch bracketed by HIP events recorded on
the stream the kernel is launched on (``lbt_amd.dfxp.ops.PROFILE``). The kernel with the largest
total event time is the dominant one; for it

    achieved = (algorithmic bytes per launch, each operand read once and each output written
                once -- see ops._Timed call sites) / (average event-timed launch duration)

is reported against the MI355X HBM3E peak (8 TB/s, MI355X_MICROARCH.md "Chip-level parameters").
Every kernel of this path is an HBM-bound element pass or a low-intensity int8 GEMM
(<= 227 int-op/B vs a ~625 op/B ridge), so the bound is "hbm".
"""
import hashlib
import json
import os
import subprocess
import sys

import torch

from .dfxp import layers, ops

HBM_PEAK_GBS = 8000.0
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# SURVEY 8(d)'s algorithmic model of one ResNet-20 step at B=128 (configs[1]): GEMM bytes 313.3 MB +
# quantiser bytes 777.9 MB (each operand read once, each output written once)
SURVEY_STEP_BYTES_R20 = 313.3e6 + 777.9e6


def csrc_digest():
    """sha256 over the kernel sources (lbt_amd/csrc, include/): the identity of the kernels a PMC
    traffic file was measured on (tools/pmc_summary.py stamps it)."""
    h = hashlib.sha256()
    dirs = [os.path.join(ROOT, "lbt_amd", "csrc"), os.path.join(ROOT, "include")]
    for d in dirs:
        for f in sorted(os.listdir(d)):
            if f.endswith((".hip", ".h")):
                h.update(f.encode())
                h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()[:16]


def git_head():
    try:
        return subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True, text=True,
                              timeout=10).stdout.strip() or None
    except Exception:  # pragma: no cover - no git on the box
        return None


def family(kernel_name):
    """Kernel family of a device symbol / bench label: the unit the roofline and the PMC traffic
    summary (tools/pmc_summary.py) agree on. conv_gemm_kernel<MODE, CS, NT, CF, NB> splits into
    forward, plain dgrad and dgrad fused with a BN pass A (CF != 0); other kernels drop their
    template arguments."""
    n = kernel_name.replace("(anonymous namespace)::", "").replace("void ", "").strip()
    if n.startswith("igemm_kernel<"):
        args = n[len("igemm_kernel<"):].split(">")[0]
        if args in ("fwd", "dgrad", "dgrad+bn_a", "dgrad+bn3_a"):  # already a family label
            return n
        return "igemm_kernel<fwd>" if args.split(",")[0].strip() == "0" else "igemm_kernel<dgrad>"
    # the 256-row / persistent GEMMs under the labels lbt_amd.dfxp.ops times them with:
    # igemm_big_kernel<MODE, A16, ADD, BN, S, BNA, HALO>
    if n.startswith("igemm_big_kernel<"):
        args = [a.strip() for a in n[len("igemm_big_kernel<"):].split(">")[0].split(",")]
        if args[0] == "0":
            return "igemm_kernel<fwd>"
        bna = int(args[5]) if len(args) > 5 and args[5].lstrip("-").isdigit() else 0
        return {1: "igemm_kernel<dgrad+bn_a>", 2: "igemm_kernel<dgrad+bn3_a>",
                3: "igemm_kernel<dgrad+bn3_a>"}.get(bna, "igemm_kernel<dgrad>")
    if n.startswith("igemm_fwdq_kernel"):
        return "igemm_kernel<fwd>"
    if n.startswith("igemm_dgrada_kernel"):
        return "igemm_kernel<dgrad+bn_a>"
    # the storing wide weight gradient (lbt_conv_wgrad_igemm_store) runs one of three bodies
    if n.startswith(("wgrad1_kernel", "wgrad3_kernel", "wgrad_wide_kernel")):
        return "wgrad_wide_kernel"
    # conv1's forward: the row-tile kernel or the gather kernel (lbt_conv_stem_wide_fwd)
    if n.startswith("stem_wide_fwd_tiles_kernel"):
        return "stem_wide_fwd_kernel"
    if n.startswith("conv_gemm_kernel<"):
        args = [a.strip() for a in n[len("conv_gemm_kernel<"):].split(">")[0].split(",")]
        if len(args) < 3:  # already a family label, e.g. "conv_gemm_kernel<1> (dgrad+A)"
            return n
        if args[0] == "0":
            return "conv_gemm_kernel<0> (fwd)"
        cf = int(args[3]) if len(args) >= 4 else 0
        return "conv_gemm_kernel<1> (dgrad+A)" if cf else "conv_gemm_kernel<1> (dgrad)"
    return n.split("(")[0].split("<")[0].strip()


def measure_step_kernels(trainer, x, y, steps=3):
    """{kernel: (launches per step, avg us, avg algorithmic bytes)} over `steps` eager steps.
    Parameters / exponents are restored afterwards so the measurement does not perturb training."""
    flat = trainer.flat
    saved = (flat.w.clone(), flat.a.clone(), trainer.ctx.exps.clone(), trainer.ctx.step.clone())
    ops.PROFILE = {}
    side = layers.SIDE_STREAM
    layers.SIDE_STREAM = False  # one stream: each launch's events bracket it alone
    try:
        for _ in range(steps):
            # hold the stream with a ~150 ms spin so the host enqueues the whole step (event
            # records + launches) before the GPU reaches it: the events then bracket device
            # execution of each kernel, not host submission gaps
            torch.cuda.synchronize()
            torch.cuda._sleep(300_000_000)
            trainer._eager(x, y)
        torch.cuda.synchronize()
        prof = ops.PROFILE
    finally:
        ops.PROFILE = None
        layers.SIDE_STREAM = side
    flat.w.copy_(saved[0])
    flat.a.copy_(saved[1])
    trainer.ctx.exps.copy_(saved[2])
    trainer.ctx.step.copy_(saved[3])
    trainer.ctx.counts.zero_()
    out = {}
    for k, recs in prof.items():
        ms = [e0.elapsed_time(e1) for e0, e1, _ in recs]
        out[k] = (len(recs) / steps, 1000.0 * sum(ms) / len(ms), sum(b for _, _, b in recs) / len(recs),
                  1000.0 * sum(ms) / steps)
    return out


def _snapshot(trainer):
    """Everything a repeated launch may move: parameters, momentum, exponents, noise step,
    overflow counters and BN running statistics."""
    flat, ctx = trainer.flat, trainer.ctx
    t = [flat.w, flat.a, ctx.exps, ctx.step, ctx.counts]
    for bn in trainer._bn_layers():
        t += [bn.X_mean_running, bn.X_var_running]
    return [(x, x.clone()) for x in t]


def _restore(snap):
    for x, v in snap:
        x.copy_(v)


def time_launches(trainer, launches, reps=20, replays=5):
    """Device time (us) of each prebuilt launch of a fused plan, timed in isolation: the launch is
    captured `reps` times into one HIP graph, the graph replayed `replays` times between two events
    on the capturing stream; no host gaps and no per-launch events inside the timed region. State
    the repeats disturb (counters, running statistics, ...) is restored afterwards."""
    snap = _snapshot(trainer)
    s = torch.cuda.Stream(device=trainer.ctx.device)
    s.wait_stream(torch.cuda.current_stream())
    out = []
    try:
        with torch.cuda.stream(s):
            for f in launches:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    for _ in range(reps):
                        f()
                g.replay()  # warm
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(replays):
                    g.replay()
                e1.record(s)
                e1.synchronize()
                out.append(1000.0 * e0.elapsed_time(e1) / (reps * replays))
                del g
    finally:
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        _restore(snap)
        torch.cuda.synchronize()
    return out


def kernel_durations_in_graph(trainer, x, y, replays=30):
    """{kernel family: [durations in us]} of every kernel of `replays` graph-replayed training steps,
    from the device activity records of torch.profiler (the runtime's kernel-dispatch tracer, the
    mechanism rocprofv3 --kernel-trace uses): each kernel timed where it runs -- inside the step's HIP
    graph, after the launch that produced its inputs -- not in isolation. State the steps move is
    restored afterwards."""
    from torch.profiler import ProfilerActivity, profile
    snap = _snapshot(trainer)
    try:
        trainer.step(x, y)  # the graph exists and is warm
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            for _ in range(replays):
                trainer.step(x, y)
            torch.cuda.synchronize()
    finally:
        _restore(snap)
        torch.cuda.synchronize()
    out = {}
    for e in prof.profiler.kineto_results.events():
        if str(e.device_type()).split(".")[-1] not in ("CUDA", "HIP"):
            continue
        out.setdefault(family(e.name()), []).append(e.duration_ns() / 1000.0)
    return out


def graph_launches(m):
    """Every kernel launch of a fused plan's step, in order, each callable on its own (side-stream
    wrappers unwrapped, stream joins dropped)."""
    tail = m.step_tail(True) if hasattr(m, "step_tail") else m._tail_fused
    return [getattr(f, "inner", f) for f in m._fwd + m._hfused + m._bwd + tail if hasattr(f, "nbytes")]


def measure_dominant_graph(trainer, traffic_file=None):
    """Fused plans: every launch of the step timed in isolation by graph replay (time_launches);
    the kernel family with the largest per-step total is the dominant one."""
    m = trainer.model
    # (a launch wrapped onto the side stream is timed as itself: graph_launches unwraps it)
    launches = graph_launches(m)
    us = time_launches(trainer, launches)
    fam = {}
    for f, t in zip(launches, us):
        r = fam.setdefault(f.kname, [0, 0.0, 0])
        r[0] += 1
        r[1] += t
        r[2] += f.nbytes
    stats = {k: (n, t / n, b / n, t) for k, (n, t, b) in fam.items()}
    out = _dominant(stats, traffic_file, "graph replay, each launch captured 20x in isolation")
    out["step_algorithmic_bytes"] = int(sum(f.nbytes for f in launches))
    out["step_launches"] = len(launches)
    out["step_kernel_us_isolated"] = round(sum(us), 1)
    return out


def in_graph(stats_in_graph, dom, replays):
    """The dominant family's in-graph average next to its isolated one; `primary` says which the
    top-level achieved / frac use (the in-graph one when the tracer delivered the records)."""
    name = dom["kernel"]
    d = stats_in_graph.get(family(name), [])
    n = dom["launches_per_step"]
    if len(d) < n * replays:
        return None
    avg = sum(d) / len(d)
    ach = dom["algorithmic_bytes_per_launch"] / (avg * 1e-6) / 1e9
    per_step = {k: round(sum(v) / replays, 1) for k, v in stats_in_graph.items()}
    return {"avg_launch_us": round(avg, 3), "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
            "launches": len(d), "replays": replays,
            "timing": "in the replayed step graph: torch.profiler device activity records (kernel dispatch "
                      "tracer), %d steps" % replays,
            "per_kernel_us_per_step": dict(sorted(per_step.items(), key=lambda kv: -kv[1]))}


def measure_dominant(trainer, x, y, traffic_file=None, replays=30):
    """Fused plans: the dominant family from isolated per-launch graph replays, then its average IN
    the replayed step (kernel_durations_in_graph); the top-level achieved / frac / avg_launch_us are the
    in-graph figures (what rocprofv3's kernel trace of the bench reports), the isolated ones are kept
    under "isolated"."""
    if hasattr(trainer.model, "_tail_fused"):
        out = measure_dominant_graph(trainer, traffic_file)
        try:
            ig = in_graph(kernel_durations_in_graph(trainer, x, y, replays), out, replays)
        except Exception as e:  # pragma: no cover - tracer unavailable: isolated figures only
            print("roofline: in-graph kernel records unavailable (%r)" % (e,), file=sys.stderr)
            ig = None
        iso = {k: out[k] for k in ("avg_launch_us", "achieved", "frac", "timing", "per_kernel_us_per_step")}
        out["isolated"] = iso
        if ig is not None:
            for k in ("avg_launch_us", "achieved", "frac", "timing", "per_kernel_us_per_step"):
                out[k] = ig[k]
            out["in_graph_launches"] = ig["launches"]
        out["primary"] = "in_graph" if ig is not None else "isolated"
        return out
    stats = measure_step_kernels(trainer, x, y)
    return _dominant(stats, traffic_file, "eager step, HIP events around each launch")


def _dominant(stats, traffic_file, timing):
    name = max(stats, key=lambda k: stats[k][3])
    calls, avg_us, avg_bytes, _ = stats[name]
    achieved = avg_bytes / (avg_us * 1e-6) / 1e9
    traffic, prov = None, None
    tf = traffic_file or os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tf):
        t = json.load(open(tf))
        fam = t.get("families", {})
        prov = {"file": os.path.relpath(tf, ROOT), "head": t.get("head"), "csrc": t.get("csrc"),
                "csrc_now": csrc_digest()}
        if prov["csrc"] != prov["csrc_now"]:
            # measured on other kernels: not this build's traffic -- reported as null, loudly
            prov["stale"] = True
            print("roofline: %s was measured on kernel sources %s, this build is %s: traffic = null"
                  % (prov["file"], prov["csrc"], prov["csrc_now"]), file=sys.stderr)
        elif family(name) in fam:
            traffic = fam[family(name)]["hbm_bytes_per_launch"]
    return {"bound": "hbm", "kernel": name, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": prov,
            "avg_launch_us": round(avg_us, 3), "algorithmic_bytes_per_launch": int(avg_bytes),
            "launches_per_step": calls, "timing": timing,
            "per_kernel_us_per_step": {k: round(v[3], 1) for k, v in sorted(stats.items(), key=lambda kv: -kv[1][3])}}
