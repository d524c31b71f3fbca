"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV (one step = the launches between
two consecutive occurrences of the step's first kernel).

    python tools/step_timeline.py <run_kernel_trace.csv> [first_kernel_substring] [--full]
"""
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "noise_fill"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    idx = [i for i, n in enumerate(names) if first in n]
    spans, gaps, busy = [], [], []
    for a, b in zip(idx[-30:-1], idx[-29:]):
        s, e = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
        k = sum(int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"]) for i in range(a, b))
        spans.append((e - s) / 1e3)
        busy.append(k / 1e3)
        gaps.append((e - s - k) / 1e3)
    print("steps %d  median step %.1f us  kernel-busy %.1f us  gaps %.1f us  launches/step %d" % (
        len(spans), statistics.median(spans), statistics.median(busy), statistics.median(gaps), idx[-2] - idx[-3]))
    if "--full" in sys.argv:
        a, b = idx[-3], idx[-2]
        for i in range(a, b):
            r = rows[i]
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            g = (int(rows[i + 1]["Start_Timestamp"]) - int(r["End_Timestamp"])) / 1e3
            print("%3d %6.1f %5.1f  %s" % (i - a, d, g, r["Kernel_Name"][:90].replace("(anonymous namespace)::", "")))


if __name__ == "__main__":
    main()
