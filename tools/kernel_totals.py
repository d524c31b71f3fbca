"""Total device time per kernel (summed over a rocprofv3 --kernel-trace CSV), top N.

    python tools/kernel_totals.py <run_kernel_trace.csv> [steps] [N]
"""
import collections
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
tot = collections.Counter()
cnt = collections.Counter()
for r in csv.DictReader(open(path)):
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    n = n.split("(")[0][:80]
    tot[n] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    cnt[n] += 1
all_us = sum(tot.values()) / 1e3 / steps
print("total kernel time per step: %.1f us" % all_us)
for n, t in tot.most_common(top):
    print("%9.1f us/step %6.1f%%  %5d calls  %s" % (t / 1e3 / steps, 100 * t / 1e3 / steps / all_us, cnt[n], n))
