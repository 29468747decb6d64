#!/usr/bin/env python3
"""Build check: no kernel of the library may need a private (scratch) segment or spill VGPRs.

A dispatch that needs scratch must get it from the runtime at launch, and under a full HBM that allocation
fails (HSA_STATUS_ERROR_OUT_OF_RESOURCES aborted a 12-slot run in round 1, profiles/r1i_mixed240_s12_abort.err.txt).
Reads the `-Rpass-analysis=kernel-resource-usage` remarks hipcc wrote for each object (*.res) and exits 1
naming every offending kernel.
Usage: check_resources.py [--json OUT.json] FILE.res...
--json writes every kernel's registers, LDS and compiler occupancy (bench.py's occupancy block reads it).
A/B builds only (tools/build_ab.sh): PBCCS_ALLOW_SCRATCH=<substring> exempts the kernels whose mangled name
contains it (reported, not failed), so a spilling variant can be measured before the rule is revisited.
"""
import json
import os
import re
import sys


def main(paths):
    out_json = None
    if paths and paths[0] == "--json":
        out_json, paths = paths[1], paths[2:]
    table = {}
    bad = []
    kernels = 0
    allow = os.environ.get("PBCCS_ALLOW_SCRATCH", "")
    for p in paths:
        name = None
        for line in open(p, errors="replace"):
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                name = m.group(1)
                kernels += 1
                table[name] = {}
                continue
            for key, pat in (("vgprs", r"remark:\s+VGPRs: (\d+)"), ("agprs", r"AGPRs: (\d+)"),
                             ("sgprs", r"TotalSGPRs: (\d+)"), ("waves_per_simd", r"Occupancy \[waves/SIMD\]: (\d+)"),
                             ("lds_bytes", r"LDS Size \[bytes/block\]: (\d+)"),
                             ("scratch_bytes", r"ScratchSize \[bytes/lane\]: (\d+)")):
                m = re.search(pat, line)
                if m and name:
                    table[name][key] = int(m.group(1))
            m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
            if m and int(m.group(1)) > 0:
                bad.append(f"{p}: {name}: private segment {m.group(1)} bytes/lane")
            m = re.search(r"VGPRs Spill: (\d+)", line)
            if m and int(m.group(1)) > 0:
                bad.append(f"{p}: {name}: {m.group(1)} VGPRs spilled")
    if allow:
        exempt = [b for b in bad if allow in b]
        for b in exempt:
            print(f"kernel resource check: exempted (PBCCS_ALLOW_SCRATCH) {b}")
        bad = [b for b in bad if allow not in b]
    if out_json:
        with open(out_json, "w") as f:
            json.dump(table, f, indent=0, sort_keys=True)
    if bad:
        print("kernel resource check failed:\n  " + "\n  ".join(bad), file=sys.stderr)
        return 1
    print(f"kernel resource check: {kernels} kernels, no scratch, no VGPR spills")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
