#!/usr/bin/env python3
"""HBM traffic per launch of one kernel family from two rocprofv3 --pmc passes.

Usage: pmc_traffic.py FETCH_CSV WRITE_CSV BENCH_JSON OUT_JSON BENCH_KERNEL

FETCH_CSV / WRITE_CSV are the counter_collection.csv files of two separate passes of the same bench
command (`--pmc FETCH_SIZE`, `--pmc WRITE_SIZE`: the two do not fit one pass, MI355X_MICROARCH.md
"Counter slots").  Correction per MI355X_MICROARCH.md §HBM: both counters are in KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced read, so
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
The result is averaged over every dispatch of the device kernels behind BENCH_KERNEL, the name bench.py's
kernel table uses (KERNELS below: k_fill = the 16-lane fill, k_fill_tall = the 64-lane and lane-serial fills
of tall bands, k_score).  BENCH_JSON is the bench line of the FETCH pass (same command); its kernel table
gives the algorithmic bytes per launch for the ratio.  The output records the digest of the kernel sources
(bench.kernel_source_digest), so that bench.py only reports the traffic while the build is the same.
"""
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

KERNELS = {"k_fill": r"k_fill_coop<16", "k_fill_tall": r"k_fill_coop<64|k_fill$",
           "k_score": r"k_score"}   # k_score + k_score_edge (one Timed launch in the engine)


def short(n):
    return n.replace("void ", "").replace("pbccs::", "").split("(")[0]


def per_dispatch(path, counter, pattern):
    vals = {}
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        k = short(row["Kernel_Name"])
        if not re.match(pattern, k):
            continue
        key = (row["Dispatch_Id"], k)
        vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return vals


def main():
    fetch_csv, write_csv, bench_json, out_json, prefix = sys.argv[1:6]
    pattern = KERNELS[prefix]
    f = per_dispatch(fetch_csv, "FETCH_SIZE", pattern)
    w = per_dispatch(write_csv, "WRITE_SIZE", pattern)
    nf, nw = len(f), len(w)
    if nf == 0 or nw == 0:
        sys.exit(f"no {prefix}* dispatches with FETCH_SIZE ({nf}) / WRITE_SIZE ({nw})")
    fetch_b = 2.0 * sum(f.values()) * 1024 / nf
    write_b = sum(w.values()) * 1024 / nw
    bench = {}
    for line in open(bench_json):
        line = line.strip()
        if line.startswith("{"):
            bench = json.loads(line)
    roof = bench.get("roofline", {})
    alg = None
    if roof.get("kernel") == prefix:
        alg = roof.get("bytes_per_launch")
    else:
        k = bench.get("kernels", {}).get(prefix)
        if k and k.get("launches"):
            alg = k["gbytes"] * 1e9 / k["launches"]
    by_kernel = {}
    for (_, k), v in f.items():
        by_kernel.setdefault(k, [0, 0.0])
        by_kernel[k][0] += 1
        by_kernel[k][1] += 2.0 * v * 1024
    from bench import kernel_source_digest
    out = {
        "bench_kernel": prefix,
        "device_kernels": pattern,
        "source_digest": kernel_source_digest(),
        "dispatches_fetch_pass": nf,
        "dispatches_write_pass": nw,
        "fetch_bytes_per_launch": fetch_b,
        "write_bytes_per_launch": write_b,
        "traffic_bytes_per_launch": fetch_b + write_b,
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": (fetch_b + write_b) / alg if alg else None,
        "fetch_bytes_per_launch_by_kernel": {k: v[1] / v[0] for k, v in sorted(by_kernel.items())},
        "dispatches_by_kernel": {k: v[0] for k, v in sorted(by_kernel.items())},
        "correction": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md §HBM, gfx950)",
        "workload": bench.get("config", {}).get("workload"),
    }
    json.dump(out, open(out_json, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
