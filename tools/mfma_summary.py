"""MFMA utilisation per kernel family from ONE rocprofv3 --pmc pass of
    SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_INSTS_VALU_MFMA_MOPS_F16
(MI355X_MICROARCH.md "rocprofv3 PMC slots": SQ and GRBM blocks, one pass). Per dispatch:
  elapsed cycles  = GRBM_GUI_ACTIVE / 8          (summed over the 8 XCDs)
  MFMA busy       = SQ_VALU_MFMA_BUSY_CYCLES / (elapsed * 1024 SIMDs)     (rocprof's MfmaUtil)
  executed i8 ops = SQ_INSTS_VALU_MFMA_MOPS_I8 * 512, f16 likewise (rocprof's MfmaFlops scaling)
Kernel times come from the same run's kernel trace (the PMC pass serialises dispatches).

    python tools/mfma_summary.py <pmc_dir> <out.json>
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from lbt_amd.roofline import family  # noqa: E402


def main():
    src, out = sys.argv[1], sys.argv[2]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(dict)
    for f in glob.glob(src + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Kernel_Name"])
            disp[key][r["Counter_Name"]] = disp[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            if "Start_Timestamp" in r and "End_Timestamp" in r:
                disp[key]["_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    for (_, name), c in disp.items():
        fam = family(name)
        p = per[fam]
        p["launches"] += 1
        p["busy"] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        p["cycles"] += c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        p["i8_ops"] += c.get("SQ_INSTS_VALU_MFMA_MOPS_I8", 0.0) * 512
        p["f16_ops"] += c.get("SQ_INSTS_VALU_MFMA_MOPS_F16", 0.0) * 512
        p["ns"] += c.get("_ns", 0.0)
    res = {"note": "MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs); executed ops = "
                   "MOPS * 512; TOPS over the PMC pass's own dispatch times (profiled clocks run lower)",
           "families": {}}
    for fam, p in sorted(per.items(), key=lambda kv: -kv[1]["busy"]):
        if p["i8_ops"] == 0 and p["f16_ops"] == 0:
            continue
        ent = {"launches": int(p["launches"]),
               "mfma_busy_frac": round(p["busy"] / (p["cycles"] * 1024), 4) if p["cycles"] else None,
               "i8_tops_executed": round(p["i8_ops"] / p["ns"] / 1e3, 1) if p["ns"] else None,
               "f16_tflops_executed": round(p["f16_ops"] / p["ns"] / 1e3, 1) if p["ns"] else None}
        res["families"][fam] = ent
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
