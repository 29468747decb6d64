"""Summarise a rocprofv3 kernel trace: busy fraction (union of kernel intervals) and per-kernel concurrency
over the timed region (the last polish window).  Usage: python tools/trace_timeline.py prof_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict


def short(n):
    for k in ("k_fill_coop<64>", "k_fill_coop<16>", "k_score_edge", "k_score", "k_suffix", "k_reduce", "k_enumerate",
              "k_qv", "k_fill", "k_compact", "copyBuffer", "fillBuffer"):
        if k in n:
            return k
    return "rocprim" if "rocprim" in n else n[:30]


rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), int(r["Grid_Size_X"])))
rows.sort()
# the timed region: from the first k_enumerate of the last group of batches to the end (approx: last 5 k_qv)
t0 = rows[0][0]
t1 = max(r[1] for r in rows)
if len(sys.argv) > 2:
    t0 = t1 - int(float(sys.argv[2]) * 1e9)
sel = [r for r in rows if r[1] > t0]
ev = []
for s, e, n, g in sel:
    ev.append((max(s, t0), 1, n))
    ev.append((e, -1, n))
ev.sort()
busy = 0
active = defaultdict(int)
tot = 0
last = t0
conc = defaultdict(float)
only = defaultdict(float)
for t, d, n in ev:
    dt = t - last
    k = sum(active.values())
    if k > 0:
        busy += dt
    conc[k] += dt
    if k > 0:
        names = tuple(sorted(x for x, c in active.items() if c > 0))
        if len(names) == 1:
            only[names[0]] += dt
    active[n] += d
    last = t
span = t1 - t0
print(f"span {span/1e6:.1f} ms, busy {busy/1e6:.1f} ms ({busy/span:.2%})")
print("concurrency histogram (ms):", {k: round(v / 1e6, 1) for k, v in sorted(conc.items())})
print("time with only one kernel type running (ms):", {k: round(v / 1e6, 1) for k, v in sorted(only.items(), key=lambda kv: -kv[1])})
