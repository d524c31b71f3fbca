"""Time single igemm launches on ResNet-50 shapes (diagnostics): python tools/igemm_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from lbt_amd.dfxp import ops  # noqa: E402
from lbt_amd.runtime import DfxpContext  # noqa: E402

dev = "cuda"
ctx = DfxpContext(seed=0)
qx, qw, qg = ctx.quantizer("t/X", 9, 2), ctx.quantizer("t/W", 8, 0), ctx.quantizer("t/g", 16, -3)
# (name, N, H, Cin, Cout, k, s, mode)
B = int(os.environ.get("PROBE_BATCH", "256"))  # ResNet-50 bench batch
shapes = [("l1_c3_fwd", B, 56, 64, 256, 1, 1, "fwd"), ("l1_c1_dgrad16", B, 56, 256, 64, 1, 1, "dgrad"),
          ("l1_c2_fwd", B, 56, 64, 64, 3, 1, "fwd"), ("l1_c2_dgrad16", B, 56, 64, 64, 3, 1, "dgrad"),
          ("l2_c2_fwd", B, 28, 128, 128, 3, 1, "fwd"), ("l2_c2_dgrad16", B, 28, 128, 128, 3, 1, "dgrad"),
          ("l3_c2_fwd", B, 14, 256, 256, 3, 1, "fwd"), ("l3_c2_dgrad16", B, 14, 256, 256, 3, 1, "dgrad"),
          ("l4_c2_fwd", B, 7, 512, 512, 3, 1, "fwd"), ("l4_c2_dgrad16", B, 7, 512, 512, 3, 1, "dgrad"),
          ("l1_c2_fwdq", B, 56, 64, 64, 3, 1, "fwdq"), ("l2_c2_fwdq", B, 28, 128, 128, 3, 1, "fwdq"),
          ("l3_c2_fwdq", B, 14, 256, 256, 3, 1, "fwdq"), ("l1_c3_fwdq", B, 56, 64, 256, 1, 1, "fwdq"),
          ("l3_c3_fwdq", B, 14, 256, 1024, 1, 1, "fwdq"), ("l1_c3_dgrad16", B, 56, 64, 256, 1, 1, "dgrad"),
          ("l2_c3_dgrad16", B, 28, 128, 512, 1, 1, "dgrad")]
# PROBE_QNOISE: inline (Philox in the epilogue), table (a per-step noise table, lbt_dfxp_noise_fill),
# none (round-to-nearest quantiser)
QN = os.environ.get("PROBE_QNOISE", "inline")
qo = ctx.quantizer("t/Y", 8, 2, stochastic=QN != "none")
only = os.environ.get("PROBE_ONLY")
shapes = [sh for sh in shapes if not only or sh[0] in only.split(",")]
for name, N, H, Cin, Cout, k, s, mode in shapes:
    d = ops.conv_desc(N, H, H, Cin, Cout, k, k, s, s, "SAME")
    W = torch.rand((k, k, Cin, Cout), device=dev) * 2 - 1
    ksf, ksd = ops.packed_slices(k, k, Cin), ops.packed_slices(k, k, Cout)
    wf = torch.zeros((Cout, ksf * 16), dtype=torch.int8, device=dev)
    wd = torch.zeros((Cin, ksd * 16), dtype=torch.int8, device=dev)
    ops.quantize_weight(W, qw, w_hwio=torch.empty((k, k, Cin, Cout), dtype=torch.int8, device=dev),
                        wf=wf, ksf=ksf, wd=wd, ksd=ksd)
    if mode == "fwdq":
        x = torch.randint(-128, 128, (N, H, H, Cin), dtype=torch.int8, device=dev)
        yq = torch.empty((N, d.Ho, d.Wo, Cout), dtype=torch.int8, device=dev)
        chs = torch.zeros((64, 2 * Cout), dtype=torch.int64, device=dev)
        if QN == "table":
            from lbt_amd import _lib
            from lbt_amd.fused import _dev_array
            inner = d.Ho * d.Wo * Cout
            tab = torch.zeros((inner + 3) // 4 * 4, dtype=torch.float32, device=dev)
            jobs = _dev_array([_lib.NJob(ctx.step.data_ptr(), ctx.seed, qo.qid, 0, inner, tab.data_ptr())], dev)
            _lib.call("lbt_dfxp_noise_fill", _lib.ptr(jobs), 1, inner, None, 0, _lib.stream())
            qo.desc.noise = tab.data_ptr()
        fn = lambda: ops.conv_fwd_igemm_q(x, 1, wf, ksf, d, qx.desc, qw.desc, yq, qo, chs)  # noqa: E731
        macs = N * d.Ho * d.Wo * Cout * k * k * Cin
    elif mode == "fwd":
        x = torch.randint(-128, 128, (N, H, H, Cin), dtype=torch.int8, device=dev)
        y = torch.empty((N, d.Ho, d.Wo, Cout), device=dev)
        fn = lambda: ops.conv_fwd_igemm(x, 1, wf, ksf, d, qx.desc, qw.desc, y)  # noqa: E731
        macs = N * d.Ho * d.Wo * Cout * k * k * Cin
    else:
        g = torch.randint(-32768, 32768, (N, d.Ho, d.Wo, Cout), dtype=torch.int16, device=dev)
        dx = torch.empty((N, H, H, Cin), device=dev)
        fn = lambda: ops.conv_dgrad_igemm(g, 1, wd, ksd, d, qg.desc, qw.desc, dx)  # noqa: E731
        macs = N * H * H * Cin * k * k * Cout
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1000
    # dgrad16 runs three int8 MFMA passes (hi, lo', all-ones) per useful MAC
    passes = 3 if mode == "dgrad" else 1
    print("%-16s %8.1f us  %7.1f TOPS (algorithmic)  %7.1f TOPS executed  %.3f of the 5 POPS int8 dense peak"
          % (name, us, 2 * macs / us / 1e6, passes * 2 * macs / us / 1e6, passes * 2 * macs / us / 1e6 / 5000),
          flush=True)
