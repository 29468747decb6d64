#!/usr/bin/env python3
"""Per host thread (one per workspace slot) of a rocprofv3 kernel trace: first and last kernel, kernels, busy
seconds -- how long the slots' tails are (the work queue's balance).  Usage: slot_ends.py <kernel_trace.csv>"""
import collections
import csv
import json
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    t0 = min(int(r["Start_Timestamp"]) for r in rows)
    th = collections.defaultdict(list)
    for r in rows:
        th[r["Thread_Id"]].append((int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0))
    out = {}
    for t, v in th.items():
        v.sort()
        out[t] = {"first_s": round(v[0][0] / 1e9, 2), "last_s": round(max(e for _, e in v) / 1e9, 2), "kernels": len(v)}
    ends = sorted(x["last_s"] for x in out.values())
    print(json.dumps({"threads": out, "ends_s": ends, "span_s": ends[-1]}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
