#!/usr/bin/env python3
"""Per-slot critical path of a multi-slot bench run.

Input: a rocprofv3 --kernel-trace CSV of `bench.py` with several workspace slots.  Each slot polishes its batches on
its own host thread (pbccs_batch_polish_many), so the trace's Thread_Id attributes every dispatch to a slot.  For
each slot, every instant between its first and last dispatch of the timed region is put in one class, in this
priority (the same classes as critical_path.py, per slot):

  fill16      one of the slot's 16-lane fills runs (its tall fills may run beside it)
  score       no fill of the slot; one of its scoring kernels runs
  tall_only   only the slot's 64-lane fills run: the slot waits on its tall reads
  copy        only the slot's runtime copies / fills run
  host        nothing of the slot runs: its host thread is between launches (selection, ApplyMutations, uploads,
              launch latency) or its kernels wait in a queue

Prints one JSON object: per class the mean over slots of the fraction of the slot's span, and per slot the spans.
Usage: slot_path.py <kernel_trace.csv> [skip_first_seconds]
"""
import csv
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from critical_path import kind  # noqa: E402

ORDER = ["fill16", "score", "tall", "copy"]


def classify(intervals, lo, hi):
    """Seconds per class over [lo, hi) for one slot's (start, end, kind) intervals."""
    ev = []
    for s, e, k in intervals:
        s, e = max(s, lo), min(e, hi)
        if e > s:
            ev.append((s, 1, k))
            ev.append((e, -1, k))
    ev.sort()
    active = {k: 0 for k in ORDER}
    out = {"fill16": 0.0, "score": 0.0, "tall_only": 0.0, "copy": 0.0, "host": 0.0}
    t = lo
    for ts, d, k in ev + [(hi, 0, None)]:
        if ts > t:
            dt = ts - t
            if active["fill16"]:
                out["fill16"] += dt
            elif active["score"]:
                out["score"] += dt
            elif active["tall"]:
                out["tall_only"] += dt
            elif active["copy"]:
                out["copy"] += dt
            else:
                out["host"] += dt
            t = ts
        if k is not None:
            active[k] += d
    return out


def main():
    path = sys.argv[1]
    skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    rows = list(csv.DictReader(open(path)))
    by_thread = {}
    for r in rows:
        k = kind(r["Kernel_Name"])
        by_thread.setdefault(r["Thread_Id"], []).append(
            (int(r["Start_Timestamp"]) * 1e-9, int(r["End_Timestamp"]) * 1e-9, k))
    t0 = min(s for v in by_thread.values() for s, _, _ in v) + skip
    slots = {}
    for tid, iv in by_thread.items():
        iv = [x for x in iv if x[0] >= t0]
        if len(iv) < 50 or not any(k == "fill16" for _, _, k in iv):
            continue   # not a polishing slot (setup / warmup threads)
        lo, hi = min(s for s, _, _ in iv), max(e for _, e, _ in iv)
        c = classify(iv, lo, hi)
        slots[tid] = {"span_s": round(hi - lo, 3), **{k: round(v, 3) for k, v in c.items()}}
    frac = {}
    for k in ("fill16", "score", "tall_only", "copy", "host"):
        vals = [s[k] / s["span_s"] for s in slots.values() if s["span_s"] > 0]
        frac[k] = round(sum(vals) / max(1, len(vals)), 4)
    print(json.dumps({"slots": len(slots), "mean_fraction": frac, "per_slot": slots}, indent=1))


if __name__ == "__main__":
    main()
