#!/usr/bin/env python3
"""Split a bench run's timed region by what the device is doing.

Input: a rocprofv3 --kernel-trace CSV of `bench.py` (any --streams).  The timed region is taken from the start of
the first AddRead fill after the warmup (the 16-lane fill launch over every read of a batch, the largest 16-lane
grid) to the last kernel end.  Every instant of it is assigned to exactly one class, in this priority:

  fill16      some 16-lane fill (k_fill_coop<16, ...>) runs (tall fills may run beside it)
  score       no fill; some scoring kernel runs (k_score, k_score_edge, k_score_ckpt, k_reduce, k_alive, k_qv,
              k_best_subset, hipCUB selects, k_suffix, k_enumerate)
  tall_only   only 64-lane fills run (k_fill_coop<64, ...>): the tall tail, a few tall waves on an otherwise idle GPU
  copy        only runtime copies / fills run
  idle        no kernel at all: host work between launches (selection, ApplyMutations, launch latency)

Prints one JSON object: seconds per class over the timed region and per timed step, plus the tall fills' wave
counts (grid blocks) by launch.
Usage: critical_path.py <kernel_trace.csv> <steps> [warmup] [batches_per_step]
"""
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
    path, steps = sys.argv[1], int(sys.argv[2])
    warmup = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    split = int(sys.argv[4]) if len(sys.argv) > 4 else 1   # device batches per step (bench.py --batch-split)
    rows = list(csv.DictReader(open(path)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind(r["Kernel_Name"]), r["Kernel_Name"],
           int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))) for r in rows]
    ks.sort()
    # AddRead fills: the 16-lane launches with the largest grid (every read of a batch)
    g16 = [k for k in ks if k[2] == "fill16"]
    big = max(k[4] for k in g16)
    starts = [k[0] for k in g16 if k[4] == big]
    skip = warmup * split
    t0 = starts[skip] if len(starts) > skip else starts[0]
    t1 = max(k[1] for k in ks)
    events = []
    for s, e, kd, _, _ in ks:
        s, e = max(s, t0), min(e, t1)
        if e > s:
            events.append((s, 1, kd))
            events.append((e, -1, kd))
    events.sort()
    active = {"fill16": 0, "score": 0, "tall": 0, "copy": 0}
    acc = {"fill16": 0, "score": 0, "tall_only": 0, "copy": 0, "idle": 0}
    last = t0
    for t, d, kd in events:
        if t > last:
            if active["fill16"]:
                c = "fill16"
            elif active["score"]:
                c = "score"
            elif active["tall"]:
                c = "tall_only"
            elif active["copy"]:
                c = "copy"
            else:
                c = "idle"
            acc[c] += t - last
            last = t
        active[kd] += d
    total = t1 - t0
    tall = [k for k in ks if k[2] == "tall" and k[0] >= t0]
    out = {"timed_s": round(total / 1e9, 4), "steps": steps,
           "seconds": {c: round(v / 1e9, 4) for c, v in acc.items()},
           "ms_per_step": {c: round(v / 1e6 / steps, 1) for c, v in acc.items()},
           "fraction": {c: round(v / total, 4) for c, v in acc.items()},
           "tall_launches": len(tall),
           "tall_waves_per_launch": {"mean": round(sum(k[4] for k in tall) / max(1, len(tall)), 1),
                                     "max": max((k[4] for k in tall), default=0),
                                     "under_200": sum(1 for k in tall if k[4] < 200)},
           "tall_device_ms_per_step": round(sum(k[1] - k[0] for k in tall) / 1e6 / steps, 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
