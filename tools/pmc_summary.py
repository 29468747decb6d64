#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel (sum over dispatches)."""
import collections
import csv
import sys


def short(n):
    n = n.replace("void ", "").replace("pbccs::", "")
    return n.split("(")[0][:40]


def load(paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    dur = collections.defaultdict(dict)
    for p in paths:
        for row in csv.DictReader(open(p)):
            k = short(row["Kernel_Name"])
            agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[k].add((p, row["Dispatch_Id"]))
            dur[k][(p, row["Dispatch_Id"])] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    return agg, disp, dur


if __name__ == "__main__":
    agg, disp, dur = load(sys.argv[1:])
    for k in sorted(agg, key=lambda k: -agg[k].get("SQ_WAVE_CYCLES", 0)):
        c = agg[k]
        if "k_" not in k:
            continue
        print(f"== {k}  dispatches={len(disp[k])}")
        for n in sorted(c):
            print(f"   {n:24s} {c[n]:.4g}")
        wc = c.get("SQ_WAVE_CYCLES", 0)
        if wc:
            print("   frac: wait_any %.2f wait_inst %.2f active %.2f valu_active %.2f lds_wait %.2f" % (
                c.get("SQ_WAIT_ANY", 0) / wc, c.get("SQ_WAIT_INST_ANY", 0) / wc, c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                c.get("SQ_ACTIVE_INST_VALU", 0) / wc, c.get("SQ_WAIT_INST_LDS", 0) / wc))
