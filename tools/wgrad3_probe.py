"""Time the wide 3x3 weight gradient on the ResNet-50 conv2 shapes (diagnostics): python tools/wgrad3_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from lbt_amd.dfxp import ops  # noqa: E402

dev = "cuda"
B = int(os.environ.get("PROBE_BATCH", "256"))
for name, H, C in [("l1_c2", 56, 64), ("l2_c2", 28, 128), ("l3_c2", 14, 256), ("l4_c2", 7, 512)]:
    d = ops.conv_desc(B, H, H, C, C, 3, 3, 1, 1, "SAME")
    ns = ops.wgrad_store_nsplit(d)
    xq = torch.randint(-128, 128, (B, H, H, C), dtype=torch.int8, device=dev)
    gq = torch.randint(-32768, 32768, (B, H, H, C), dtype=torch.int16, device=dev)
    slab = torch.empty((ns, 9 * C, C), dtype=torch.int64, device=dev)
    fn = lambda: ops.conv_wgrad_igemm_store(xq, gq, 1, d, slab, ns)  # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1000
    macs = B * H * H * 9 * C * C
    print("%-8s ns %4d  %8.1f us  %7.1f TOPS (algorithmic, x2 for the hi/lo planes: %.3f of 5 POPS)"
          % (name, ns, us, 2 * macs / us / 1e6, 4 * macs / us / 1e6 / 5000), flush=True)
