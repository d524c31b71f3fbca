"""Per-kernel-variant SQ wave-state summary from one rocprofv3 --pmc pass (diagnostics):
    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
        SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d <dir> -- python bench.py ... --eager
    python tools/sq_summary.py <dir>
Fractions of wave cycles parked in s_waitcnt / barriers (WAIT_ANY), stalled on issue (WAIT_INST_ANY)
and issuing (ACTIVE_INST_ANY, of which VALU), and instructions per wave-cycle, per kernel variant."""
import collections
import csv
import glob
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")[:60]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
rows = sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))
print("%-60s %6s %6s %6s %6s %8s %8s %8s" % ("kernel", "wait", "winst", "active", "valu", "valu/wc", "salu/wc",
                                             "lds/wc"))
for k, c in rows[:25]:
    wc = max(c.get("SQ_WAVE_CYCLES", 0), 1.0)
    print("%-60s %6.2f %6.2f %6.2f %6.2f %8.3f %8.3f %8.3f" % (
        k, c.get("SQ_WAIT_ANY", 0) / wc, c.get("SQ_WAIT_INST_ANY", 0) / wc, c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
        c.get("SQ_ACTIVE_INST_VALU", 0) / wc, c.get("SQ_INSTS_VALU", 0) / wc, c.get("SQ_INSTS_SALU", 0) / wc,
        c.get("SQ_INSTS_LDS", 0) / wc))
