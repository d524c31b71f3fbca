"""Per-kernel, per-grid-shape average durations of a rocprofv3 kernel trace (tools/r50_trace.sh):
   python tools/r50_shapes.py run_kernel_trace.csv [steps]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    n = n.split("(")[0] if not n.startswith("void ") else n[5:].split("(")[0]
    d[(n[:48], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = collections.Counter()
for (n, *_), v in d.items():
    tot[n] += sum(v) / steps
print("# per step (us), %d steps assumed" % steps)
for n, t in tot.most_common(25):
    print("%9.1f  %s" % (t, n))
print("# per shape: kernel grid calls avg_us")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:60]:
    print("%-48s %8s %5s %4s %5d %8.1f" % (k[0], k[1], k[2], k[3], len(v), sum(v) / len(v)))
