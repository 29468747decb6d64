#!/usr/bin/env python3
"""Where each kernel family's wave time goes, from one rocprofv3 --pmc pass of the bench:
SQ_WAVE_CYCLES = SQ_ACTIVE_INST_ANY (issuing) + SQ_WAIT_INST_ANY (ready to issue but stalled: a dependency or a busy
pipe) + SQ_WAIT_ANY (parked on s_waitcnt / barrier: memory or LDS latency) (MI355X_MICROARCH.md, rocprofv3 PMC slots);
SQ_ACTIVE_INST_VALU the cycles issuing VALU.  Per dispatch the kernel runs alone (a --pmc run serialises dispatches),
so SQ_WAVE_CYCLES x 4 / (dispatch cycles) is the family's mean resident waves when it has the device to itself, and
SQ_BUSY_CU_CYCLES / GRBM_GUI_ACTIVE how many CUs it keeps busy.  TCC hit rate over the family's L2 requests.
Usage: binding.py COUNTER_CSV OUT_JSON [SOURCE_DIGEST]"""
import csv
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from valu_per_cell import kind  # noqa: E402

ENGINE_HZ = 2.4e9


def main(csv_path, out_path, digest=None):
    agg, disp, span = {}, {}, {}
    for row in csv.DictReader(open(csv_path)):
        k = kind(row["Kernel_Name"])
        if not k:
            continue
        c = agg.setdefault(k, {})
        c[row["Counter_Name"]] = c.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
        d = row["Dispatch_Id"]
        if d not in disp.setdefault(k, set()):
            disp[k].add(d)
            if row.get("Start_Timestamp") and row.get("End_Timestamp"):
                span[k] = span.get(k, 0) + int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    out = {"source_digest": digest, "counters_csv": csv_path.split("gpurun_out/")[-1], "kernels": {},
           "note": "one --pmc pass: dispatches serialised, so each family's figures are for it running alone; "
                   "SQ_* wave counters in quad-cycles (x4 = cycles)"}
    for k, c in sorted(agg.items()):
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        d = {"dispatches": len(disp[k])}
        if wc:
            for n, lab in (("SQ_ACTIVE_INST_ANY", "issuing"), ("SQ_WAIT_INST_ANY", "issue_stalled"),
                           ("SQ_WAIT_ANY", "waitcnt_parked"), ("SQ_ACTIVE_INST_VALU", "valu_issuing")):
                if n in c:
                    d[lab + "_frac"] = round(c[n] / wc, 4)
        if k in span and span[k] > 0 and wc:
            cyc = span[k] * 1e-9 * ENGINE_HZ
            d["resident_waves_alone"] = round(4.0 * wc / cyc, 1)
            if "SQ_INSTS_VALU" in c:   # VALU issue over the device's SIMD cycles while the family runs alone
                d["valu_issue_frac_alone"] = round(4.0 * c["SQ_INSTS_VALU"] / (cyc * 1024), 4)
            d["device_ms"] = round(span[k] / 1e6, 1)
        if c.get("GRBM_GUI_ACTIVE") and "SQ_BUSY_CU_CYCLES" in c:
            d["busy_cu_per_gui_cycle"] = round(c["SQ_BUSY_CU_CYCLES"] / c["GRBM_GUI_ACTIVE"], 3)
        h, m = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
        if h is not None and m is not None and h + m > 0:
            d["l2_hit_frac"] = round(h / (h + m), 4)
        d["raw"] = {n: v for n, v in c.items()}
        out["kernels"][k] = d
    json.dump(out, open(out_path, "w"), indent=1)
    print(json.dumps({k: {x: y for x, y in v.items() if x != "raw"} for k, v in out["kernels"].items()}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
