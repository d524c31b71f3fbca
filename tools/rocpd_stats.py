"""Summarise a rocprofv3 rocpd database: per-kernel stats over the last K steps of a bench run,
and per-step busy time vs wall time. usage: rocpd_stats.py db [steps]"""
import sqlite3, sys, collections, re
db = sys.argv[1]
con = sqlite3.connect(db)
cur = con.cursor()
cols = [r[1] for r in cur.execute("pragma table_info(kernels)")]
rows = cur.execute("select * from kernels").fetchall()
ci = {c: i for i, c in enumerate(cols)}
name_col = 'kernel_name' if 'kernel_name' in ci else 'name'
k = [(r[ci['start']], r[ci['end']], r[ci[name_col]]) for r in rows]
k.sort()
def short(n):
    n = n.replace('(anonymous namespace)::', '')
    n = re.sub(r'\(.*', '', n)
    return n[:60]
# find the step boundary: the noise fill kernel starts each step
starts = [i for i, x in enumerate(k) if 'noise_fill' in x[2]]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
sel = starts[-steps - 1:]
agg = collections.defaultdict(lambda: [0, 0.0])
busy = []
walls = []
for a, b in zip(sel[:-1], sel[1:]):
    seg = k[a:b]
    busy.append(sum(e - s for s, e, _ in seg))
    walls.append(k[b][0] - k[a][0])
    for s, e, n in seg:
        g = agg[short(n)]
        g[0] += 1
        g[1] += e - s
ns = len(busy)
print("steps %d  wall/step %.1f us  kernel-busy/step %.1f us  launches/step %.1f" % (ns, sum(walls) / ns / 1e3, sum(busy) / ns / 1e3, sum(v[0] for v in agg.values()) / ns))
tot = sum(v[1] for v in agg.values())
print("%-62s %6s %9s %9s %6s" % ("kernel", "n/step", "avg us", "us/step", "%"))
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print("%-62s %6.1f %9.2f %9.1f %6.1f" % (n, c / ns, t / c / 1e3, t / ns / 1e3, 100 * t / tot))
