#!/usr/bin/env python3
"""What the device and the slots do over a bench run, from a rocprofv3 --kernel-trace CSV.

Prints one JSON object:
  classes      seconds (and fraction of the traced span) in which some 16-lane fill runs / only scoring runs / only
               64-lane (tall) fills run -- with or without scoring beside them -- / only copies / nothing;
  tall_waves   the mean number of tall-fill grid waves in flight (an upper bound on resident tall waves: a launch's
               waves end at different times);
  slot_gaps    per host thread (one per workspace slot): seconds with none of its kernels on the device for more than
               `gap_s` at a time -- host work or a host call blocked behind other slots' work;
  queues       hardware queues that carried streams of two different host threads at overlapping times (a stream's
               kernels then wait behind another slot's in-order work).
Usage: slot_gaps.py <kernel_trace.csv> [gap_s=1.0]
"""
import collections
import csv
import json
import sys


def kind(name):
    if "k_fill_coop<16" in name:
        return "fill16"
    if "k_fill_coop<64" in name:
        return "tall"
    if name.startswith("__amd_rocclr"):
        return "copy"
    return "score"


def main():
    path = sys.argv[1]
    gap_s = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind(r["Kernel_Name"]),
                 int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), r["Thread_Id"], r["Queue_Id"],
                 r["Stream_Id"]) for r in rows)
    t0, t1 = ks[0][0], max(k[1] for k in ks)
    span = t1 - t0
    ev = []
    for s, e, kd, g, *_ in ks:
        ev.append((s, 1, kd, g))
        ev.append((e, -1, kd, g))
    ev.sort(key=lambda x: (x[0], x[1]))
    act = collections.Counter()
    acc = collections.Counter()
    tw, twsum, last = 0, 0.0, t0
    for t, d, kd, g in ev:
        dt = t - last
        if dt > 0:
            if act["fill16"]:
                c = "fill16"
            elif act["score"]:
                c = "score+tall" if act["tall"] else "score"
            elif act["tall"]:
                c = "tall_only"
            elif act["copy"]:
                c = "copy"
            else:
                c = "idle"
            acc[c] += dt
            twsum += tw * dt
        act[kd] += d
        if kd == "tall":
            tw += d * g
        last = t
    # per host thread: gaps with none of its kernels running
    th = collections.defaultdict(list)
    for s, e, kd, g, tid, q, st in ks:
        th[tid].append((s, e))
    gaps = {}
    for tid, v in th.items():
        v.sort()
        end, tot, n = v[0][1], 0, 0
        for s, e in v[1:]:
            if s - end > gap_s * 1e9:
                tot += s - end
                n += 1
            end = max(end, e)
        gaps[tid] = {"gaps": n, "gap_s": round(tot / 1e9, 2), "active_s": round((end - v[0][0]) / 1e9, 2)}
    # hardware queues shared by two host threads' streams at overlapping times
    use = collections.defaultdict(lambda: [None, 0])
    for s, e, kd, g, tid, q, st in ks:
        u = use[(q, st, tid)]
        u[0] = s if u[0] is None else min(u[0], s)
        u[1] = max(u[1], e)
    byq = collections.defaultdict(list)
    for (q, st, tid), (a, b) in use.items():
        byq[q].append((a, b, st, tid))
    shared = {}
    for q, v in byq.items():
        olap = 0
        for i in range(len(v)):
            for j in range(i + 1, len(v)):
                if v[i][3] != v[j][3]:
                    olap += max(0, min(v[i][1], v[j][1]) - max(v[i][0], v[j][0]))
        if olap > 0:
            shared[q] = {"streams": sorted({x[2] for x in v}), "threads": sorted({x[3] for x in v}),
                         "overlap_s": round(olap / 1e9, 2)}
    out = {"span_s": round(span / 1e9, 2), "kernels": len(ks),
           "classes": {c: {"s": round(v / 1e9, 2), "frac": round(v / span, 4)} for c, v in acc.most_common()},
           "tall_waves": round(twsum / span, 1),
           "slot_gaps": gaps, "slot_gap_total_s": round(sum(g["gap_s"] for g in gaps.values()), 2),
           "queues_shared_across_threads": shared}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
