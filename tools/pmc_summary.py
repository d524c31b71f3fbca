"""Summarise rocprofv3 --pmc CSVs (one pass per counter, as MI355X_MICROARCH.md prescribes) into
HBM bytes per launch, per kernel family (lbt_amd.roofline.family: the unit bench.py's roofline uses).
gfx950 FETCH_SIZE reports half of a wide coalesced read's bytes: x2 (the guide's correction, which
is calibrated for 16 B/lane loads; this path's 4 B/lane element loads are not calibrated).
Counters are in KB.  usage: pmc_summary.py <fetch_dir> <write_dir> <out.json>"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from lbt_amd.roofline import family  # noqa: E402


def load(path, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(path + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                acc[family(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return acc


fetch = load(sys.argv[1], "FETCH_SIZE")
write = load(sys.argv[2], "WRITE_SIZE")
from lbt_amd.roofline import csrc_digest  # noqa: E402

out = {"head": os.environ.get("LBT_HEAD") or None, "csrc": csrc_digest(),
       "note": "per-launch HBM traffic = (2*FETCH_SIZE + WRITE_SIZE) * 1024 B, averaged over the family's "
               "launches (eager bench step); FETCH_SIZE x2 per MI355X_MICROARCH.md 'HBM'", "families": {}}
for k in sorted(set(fetch) | set(write)):
    f = sum(fetch.get(k, [0])) / max(1, len(fetch.get(k, [])))
    w = sum(write.get(k, [0])) / max(1, len(write.get(k, [])))
    out["families"][k] = {"fetch_kb": round(f, 1), "write_kb": round(w, 1), "launches": len(fetch.get(k, [])),
                          "hbm_bytes_per_launch": int((2 * f + w) * 1024)}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1)[:3000])
