"""Time the ResNet-50 conv1 weight gradient (B=256, 224^2, 7x7/2, 3 -> 64, 16-bit G) with the row-chunk
kernel and the gather kernel (diagnostics): python tools/stem_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from lbt_amd.dfxp import ops  # noqa: E402

dev = "cuda"
B = int(os.environ.get("PROBE_BATCH", "256"))
d = ops.conv_desc(B, 224, 224, 3, 64, 7, 7, 2, 2, "SAME")
x = torch.randint(-256, 256, (B, 224, 224, 3), dtype=torch.int16, device=dev)
g = torch.randint(-32768, 32768, (B, d.Ho, d.Wo, 64), dtype=torch.int16, device=dev)
ns = ops.stem_wide_nsplit(d)
slab = torch.empty((ns, 147, 64), dtype=torch.int64, device=dev)
res = {}
for rows, cg in (("1", "32"), ("1", "64"), ("0", "64")):
    os.environ["LBT_STEM_ROWS"], os.environ["LBT_STEM_CG"] = rows, cg
    for _ in range(2):
        ops.conv_stem_wide_wgrad(x, 9, g, d, slab, ns)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        ops.conv_stem_wide_wgrad(x, 9, g, d, slab, ns)
    e1.record()
    torch.cuda.synchronize()
    res[rows + cg] = slab.sum(0).clone()
    print("stem wgrad rows=%s cg=%s: %.1f us" % (rows, cg, e0.elapsed_time(e1) / 10 * 1000), flush=True)
assert torch.equal(res["132"], res["064"]) and torch.equal(res["164"], res["064"])
print("equal")
