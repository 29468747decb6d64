#!/usr/bin/env python3
"""Where a slot thread's wall time goes outside its kernels (attribute the configs[3] timed region).

Input: the rocprofv3 --hip-trace CSV of a bench run (run_hip_api_trace.csv).  Prints, per HIP API function, the calls,
total and maximum duration, and the calls longer than a threshold with their thread and start time, so a blocking
call (a device-wide synchronisation behind other slots' multi-second tall fills) shows up by name.
Usage: api_gaps.py <hip_api_trace.csv> [min_ms=200]
"""
import collections
import csv
import json
import sys


def main():
    path = sys.argv[1]
    min_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 200.0
    per = collections.defaultdict(lambda: [0, 0.0, 0.0])
    long_calls = []
    t0 = None
    with open(path) as f:
        for r in csv.DictReader(f):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            t0 = s if t0 is None else min(t0, s)
            ms = (e - s) / 1e6
            name = r.get("Function") or r.get("Operation") or r.get("Kind")
            p = per[name]
            p[0] += 1
            p[1] += ms
            p[2] = max(p[2], ms)
            if ms >= min_ms:
                long_calls.append((s, r.get("Thread_Id"), name, ms))
    long_calls.sort()
    top = sorted(per.items(), key=lambda x: -x[1][1])[:25]
    out = {
        "by_function": {k: {"calls": v[0], "total_s": round(v[1] / 1e3, 3), "max_ms": round(v[2], 1)} for k, v in top},
        "long_calls": [{"t_s": round((s - t0) / 1e9, 2), "thread": th, "fn": n, "ms": round(ms, 1)}
                       for s, th, n, ms in long_calls[:400]],
        "long_calls_total_s": round(sum(c[3] for c in long_calls) / 1e3, 2),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
