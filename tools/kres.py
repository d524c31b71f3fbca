"""Per-kernel register / LDS / occupancy table of one .hip file (hipcc -Rpass-analysis).

    python tools/kres.py lbt_amd/csrc/conv_mfma.hip [name-filter]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lbt_amd import _build  # noqa: E402


def main():
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    cmd = [_build.HIPCC] + _build.FLAGS + ["-c", src, "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark:\s+(.*?):\s+(.*?)\s+\[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                           text=True).stdout.splitlines()
    for r, n in zip(rows, names):
        n = re.sub(r"\(anonymous namespace\)::", "", n)
        n = n.split("(")[0] if "(" in n and filt not in ("", "args") else n
        if filt and filt not in n:
            continue
        print("%-70s vgpr %4s agpr %3s sgpr %3s lds %6s occ %2s spill %s/%s" % (
            n[:70], r.get("VGPRs"), r.get("AGPRs"), r.get("TotalSGPRs"), r.get("LDS Size [bytes/block]"),
            r.get("Occupancy [waves/SIMD]"), r.get("VGPRs Spill"), r.get("ScratchSize [bytes/lane]")))


if __name__ == "__main__":
    main()
