#!/usr/bin/env python3
"""Device-idle gaps and runtime copies of a rocprofv3 --kernel-trace --memory-copy-trace run (the ccs
convoy).  Usage: copy_trace.py <rocprofv3 output dir>"""
import csv, glob, sys
d = sys.argv[1]
kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
mt = glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True)
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in csv.DictReader(open(kt)))
T0 = ks[0][0]
print("kernels", len(ks), "span s", (max(k[1] for k in ks) - T0) / 1e9)
ev = sorted((k[0], k[1]) for k in ks); cur = ev[0][1]; gaps = []
for s, e in ev[1:]:
    if s > cur: gaps.append((s - cur, (cur - T0) / 1e9))
    cur = max(cur, e)
big = sorted([g for g in gaps if g[0] > 20e6], key=lambda g: g[1])
print("device-idle gaps > 20 ms (len ms @ s):", [(round(g / 1e6, 1), round(t, 2)) for g, t in big])
if mt:
    rows = list(csv.DictReader(open(mt[0])))
    print("copy columns", list(rows[0].keys())[:12])
    by = {}
    for r in rows:
        k = r.get("Direction", "?")
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        b = by.setdefault(k, [0, 0, 0]); b[0] += 1; b[1] += dur; b[2] += int(r.get("Size", 0) or 0)
    for k, (n, dur, sz) in by.items(): print(k, n, "copies", round(dur / 1e6, 1), "ms", round(sz / 1e6, 1), "MB")
    longest = sorted(rows, key=lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), reverse=True)[:8]
    for r in longest:
        print("long copy", r.get("Direction"), r.get("Size"), round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, 2), "ms @", round((int(r["Start_Timestamp"]) - T0) / 1e9, 2))
