"""GPU busy profile from a rocprofv3 kernel trace: the union of kernel intervals (the fraction of wall time
some kernel runs), the mean number of kernels in flight, and the same per kernel family, over the longest
dense window of dispatches (the timed region).  Usage: python3 tools/trace_busy.py prof_kernel_trace.csv"""
import csv
import sys


def main(path, gap_ms=500.0):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # split into windows at idle gaps longer than gap_ms; report the longest window (the timed polish)
    wins, cur, end = [], [], 0
    for s, e, n in rows:
        if cur and s - end > gap_ms * 1e6:
            wins.append(cur)
            cur = []
        cur.append((s, e, n))
        end = max(end, e)
    if cur:
        wins.append(cur)
    w = max(wins, key=lambda x: max(e for _, e, _ in x) - x[0][0])
    t0, t1 = w[0][0], max(e for _, e, _ in w)
    wall = t1 - t0
    ev = sorted([(s, 1) for s, _, _ in w] + [(e, -1) for _, e, _ in w])
    busy, depth, last, area = 0, 0, t0, 0
    for t, d in ev:
        if depth > 0:
            busy += t - last
        area += depth * (t - last)
        depth += d
        last = t
    fam = {}
    for s, e, n in w:
        k = n.split("(")[0].replace("void ", "")[:40]
        fam[k] = fam.get(k, 0) + (e - s)
    print(f"window {wall / 1e9:.2f} s, {len(w)} dispatches; busy (some kernel running) {busy / wall:.3f}; "
          f"mean kernels in flight {area / wall:.2f}")
    for k, v in sorted(fam.items(), key=lambda x: -x[1])[:8]:
        print(f"  {k:42s} {v / 1e9:8.2f} s kernel time  ({v / wall:.2f} in flight on average)")


if __name__ == "__main__":
    main(sys.argv[1])
