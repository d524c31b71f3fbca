"""Median duration of each launch position of the replayed training step, from a rocprofv3
--kernel-trace CSV (steps delimited by step_prologue_kernel).

    python tools/step_positions.py <run_kernel_trace.csv> [skip_steps]
"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 10
pro = [i for i, r in enumerate(rows) if "step_prologue" in r["Kernel_Name"]]
steps = [rows[pro[i]:pro[i + 1]] for i in range(skip, len(pro) - 1)]
n = min(len(s) for s in steps)
tot = 0.0
for j in range(n):
    d = sorted(int(s[j]["End_Timestamp"]) - int(s[j]["Start_Timestamp"]) for s in steps)
    r = steps[0][j]
    nm = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:46]
    med = d[len(d) // 2] / 1e3
    tot += med
    print("%3d %-46s grid %7s lds %6s  %6.1f us" % (j, nm, r["Grid_Size_X"], r["LDS_Block_Size"], med))
wall = [(int(steps[i + 1][0]["Start_Timestamp"]) - int(steps[i][0]["Start_Timestamp"])) / 1e3 for i in range(len(steps) - 1)]
print("launches/step %d, sum of medians %.1f us, median step wall %.1f us" % (n, tot, sorted(wall)[len(wall) // 2]))
