"""Time the BN pass-A dgrad epilogues against the separate launches they replace (diagnostics):
python tools/bna_probe.py. Per ResNet-50 shape at B=256: lbt_conv_dgrad_igemm_bna / _bn3 (fused, the
sample-blocked 256-row kernel) vs lbt_conv_dgrad_igemm_ws + lbt_bn_bwd_a_wide_masked (per BN)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from lbt_amd._lib import NSHARD  # noqa: E402
from lbt_amd.dfxp import ops  # noqa: E402
from lbt_amd.runtime import DfxpContext  # noqa: E402

dev = "cuda"
B = int(os.environ.get("PROBE_BATCH", "256"))
# (name, H, Cin, Cout, k, mode, nbn, gmask): the dgrad's dx is [B, H, H, Cin]
shapes = [("l1_c2_dgrad+bn1", 56, 64, 64, 3, "bna", 1, False), ("l1_c3_dgrad+bn2", 56, 64, 256, 1, "bna", 1, False),
          ("l3_c2_dgrad+bn1", 14, 256, 256, 3, "bna", 1, False),
          ("l1_c1_dgrad+bn3", 56, 256, 64, 1, "bn3", 1, True), ("l1_c1_dgrad+bn3+sc", 56, 256, 64, 1, "bn3", 2, False),
          ("l2_c1_dgrad+bn3", 28, 512, 128, 1, "bn3", 1, True), ("l3_c1_dgrad+bn3", 14, 1024, 256, 1, "bn3", 1, True)]
only = os.environ.get("PROBE_ONLY")
shapes = [sh for sh in shapes if not only or sh[0] in only.split(",")]


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1000


for name, H, Cin, Cout, k, mode, nbn, gm in shapes:
    ctx = DfxpContext(seed=0)
    qw, qg = ctx.quantizer("t/W", 8, 0), ctx.quantizer("t/g", 16, -3)
    d = ops.conv_desc(B, H, H, Cin, Cout, k, k, 1, 1, "SAME")
    W = torch.rand((k, k, Cin, Cout), device=dev) * 2 - 1
    ksf, ksd = ops.packed_slices(k, k, Cin), ops.packed_slices(k, k, Cout)
    wf = torch.zeros((Cout, ksf * 16), dtype=torch.int8, device=dev)
    wd = torch.zeros((Cin, ksd * 16), dtype=torch.int8, device=dev)
    ops.quantize_weight(W, qw, w_hwio=torch.empty((k, k, Cin, Cout), dtype=torch.int8, device=dev),
                        wf=wf, ksf=ksf, wd=wd, ksd=ksd)
    g = torch.randint(-32768, 32768, (B, H, H, Cout), dtype=torch.int16, device=dev)
    shape = (B, H, H, Cin)
    rows, inner = B * H * H, H * H * Cin
    dx = torch.empty(shape, device=dev)
    qr = ctx.quantizer("t/rX", 8, 2)
    bns = []
    for t in range(nbn):
        qrg = ctx.quantizer("t/rg%d" % t, 16, 4)
        qng = ctx.quantizer("t/ng%d" % t, 16, 4)
        R = torch.randint(-128, 128, shape, dtype=torch.int8, device=dev)
        qn = torch.randint(-128, 128, shape, dtype=torch.int8, device=dev)
        gb = torch.rand(2 * Cin, device=dev) * 2 - 1
        G = torch.empty(shape, dtype=torch.int16, device=dev)
        sums = torch.zeros(NSHARD * 4 * Cin, dtype=torch.int64, device=dev)
        bns.append((R, gb, qrg, qng, qn, G, sums))
    g2 = torch.randn(shape, device=dev) if mode == "bn3" else None
    ybits = torch.randint(0, 16, (B * H * H * Cin // 4,), dtype=torch.uint8, device=dev) if mode == "bn3" else None
    gmask = torch.empty(shape, device=dev) if gm else None
    for t in range(nbn):  # the noise tables exist before timing (their fill is the model prologue's)
        for q in bns[t][2:4]:
            ctx.noise_table_desc(q, inner)
    if mode == "bna":
        R, gb, qrg, qng, qn, G, sums = bns[0]
        fused = lambda: ops.conv_dgrad_igemm_bna(g, wd, ksd, d, qg.desc, qw.desc, qr.desc, R, gb, qrg, qng, qn,  # noqa
                                                 G, sums, dx, None)

        def unfused():
            ops.conv_dgrad_igemm_ws(g, 1, wd, ksd, d, qg.desc, qw.desc, dx, None)
            ops.bn_bwd_a_wide_masked(dx, None, True, qr.desc, gb, None, qrg.desc, R, qng.desc, qn, G, sums, rows,
                                     inner, Cin)
    else:
        fused = lambda: ops.conv_dgrad_igemm_bn3(g, wd, ksd, d, qg.desc, qw.desc, g2, ybits, gmask, bns, dx,  # noqa
                                                 None)

        def unfused():
            ops.conv_dgrad_igemm_ws(g, 1, wd, ksd, d, qg.desc, qw.desc, dx, None)
            for t, (R, gb, qrg, qng, qn, G, sums) in enumerate(bns):
                ops.bn_bwd_a_wide_masked(dx, None, False, qr.desc, gb, gmask if t == 0 else None, qrg.desc, R,
                                         qng.desc, qn, G, sums, rows, inner, Cin, g2=g2, y_bits=ybits)
    dg = timed(lambda: ops.conv_dgrad_igemm_ws(g, 1, wd, ksd, d, qg.desc, qw.desc, dx, None))
    uf, fu = timed(unfused), timed(fused)
    # algorithmic bytes of the fused launch: the 16-bit G codes, the weight image, per BN R + qn in and
    # the 16-bit G out, and (bn3) g2 in, y_bits in, the optional gmask out
    nel = rows * Cin
    ab = rows * Cout * 2 + wd.numel() + nbn * nel * 4
    if mode == "bn3":
        ab += nel * 4 + nel // 4 + (nel * 4 if gm else 0)
    print("%-20s dgrad %7.1f us | dgrad + pass A %7.1f us | fused %7.1f us (%.2fx) | %.1f MB, %.2f TB/s" %
          (name, dg, uf, fu, uf / fu, ab / 1e6, ab / fu / 1e6), flush=True)
