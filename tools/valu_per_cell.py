#!/usr/bin/env python3
"""VALU instructions per counted DP cell, per fill / score kernel: rocprofv3 --pmc SQ_INSTS_VALU (wave64 VALU
instructions summed over the kernel's dispatches) over the same bench run's in-kernel cell counts (its JSON line's
`kernels`).  The run must have profiling on (the default), so the cells are counted.  Also LDS bank conflicts per
LDS-active cycle when the pass collected SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.
Usage: valu_per_cell.py COUNTER_CSV BENCH_JSON OUT_JSON [SOURCE_DIGEST]"""
import csv
import json
import sys


def kind(name):
    n = name.replace("void ", "").replace("pbccs::", "")
    if n.startswith("(anonymous namespace)::"):
        n = n[len("(anonymous namespace)::"):]
    if n.startswith("k_fill_coop<16"):
        return "k_fill"
    if n.startswith("k_fill_coop<64"):
        return "k_fill_tall"
    for k in ("k_score_ckpt", "k_score_edge", "k_score", "k_suffix", "k_reduce", "k_qfill_grp", "k_qfill_coop", "k_qscore_mid"):
        if n.startswith(k + "(") or n.startswith(k + "<") or n == k:
            return k
    return None


def main(csv_path, bench_path, out_path, digest=None):
    agg, disp = {}, {}
    for row in csv.DictReader(open(csv_path)):
        k = kind(row["Kernel_Name"])
        if not k:
            continue
        c = agg.setdefault(k, {})
        c[row["Counter_Name"]] = c.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
        disp.setdefault(k, set()).add(row["Dispatch_Id"])
    bench = json.loads(open(bench_path).read().strip().splitlines()[-1])
    out = {"source_digest": digest, "bench_value": bench.get("value"), "workload": bench.get("config", {}).get("workload"),
           "note": "SQ_INSTS_VALU (wave64 VALU instructions) per DP cell the kernel counted in-kernel, same run",
           "kernels": {}}
    for k, c in sorted(agg.items()):
        cells = bench.get("kernels", {}).get(k, {}).get("gcells", 0.0) * 1e9
        d = {"dispatches": len(disp[k]), "valu_insts": c.get("SQ_INSTS_VALU"), "cells": cells}
        if c.get("SQ_INSTS_VALU") is not None and cells:
            d["valu_per_cell"] = round(c["SQ_INSTS_VALU"] / cells, 3)
        if c.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_bank_conflict_frac"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"], 4)
        for n in ("SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_WAVES", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"):
            if n in c:
                d[n] = c[n]
        out["kernels"][k] = d
    json.dump(out, open(out_path, "w"), indent=1)
    print(json.dumps({k: v.get("valu_per_cell") for k, v in out["kernels"].items()}))


if __name__ == "__main__":
    main(*sys.argv[1:])
