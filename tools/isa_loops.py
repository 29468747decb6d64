#!/usr/bin/env python3
"""Static instruction mix of a kernel's loops from its gfx950 assembly (where a fill's VALU
instructions per cell go).  Generate the assembly with the Makefile's flags plus `--cuda-device-only -S`, e.g.
  hipcc -std=c++17 -O3 -ffp-contract=off -fno-fast-math -fno-gpu-flush-denormals-to-zero --offload-arch=gfx950 \\
        --cuda-device-only -S pbccs_amd/csrc/fill_coop.hip -o /tmp/fill_coop.s
then: isa_loops.py /tmp/fill_coop.s <kernel-name substring> [max loops]
Each natural loop (a backward branch to an earlier block) is listed innermost first with its blocks' instruction
classes: VALU (FP64 arithmetic, DPP moves, other), SALU, LDS, global/flat memory, waits, branches.  A loop body's
VALU count over the band rows one iteration advances is the static VALU per cell of that loop's path."""
import collections
import re
import sys


def classify(op):
    if op.startswith("v_"):
        if "_dpp" in op or op.startswith("v_mov_b32_dpp") or op.startswith("v_mov_b64_dpp"):
            return "valu_dpp"
        if op.startswith(("v_fma_f64", "v_mul_f64", "v_add_f64", "v_max_f64", "v_min_f64", "v_div", "v_rcp_f64",
                          "v_ldexp_f64", "v_cmp_", "v_cndmask")):
            if op.startswith("v_cmp_") or op.startswith("v_cndmask"):
                return "valu_cmp_sel"
            return "valu_f64"
        return "valu_other"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "flat_", "buffer_", "scratch_")):
        return "vmem"
    return "other"


def main(path, name, max_loops=12):
    lines = open(path).read().splitlines()
    start = None
    for i, ln in enumerate(lines):
        if re.match(r"^_Z\S*:", ln) and name in ln.split(":")[0]:
            start = i
            break
    if start is None:
        sys.exit(f"no kernel matching {name}")
    blocks, order, cur = {}, [], "entry"
    blocks[cur] = []
    order.append(cur)
    for ln in lines[start + 1:]:
        if ln.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\d+_\d+):", ln)
        if m:
            cur = m.group(1)
            blocks[cur] = []
            order.append(cur)
            continue
        t = ln.strip()
        if not t or t.startswith((";", ".", "//")):
            continue
        blocks[cur].append(t.split()[0])
    pos = {b: k for k, b in enumerate(order)}
    loops = []
    # re-scan with operands for branch targets
    cur, k = "entry", 0
    targets = collections.defaultdict(list)
    for ln in lines[start + 1:]:
        if ln.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\d+_\d+):", ln)
        if m:
            cur = m.group(1)
            continue
        t = ln.strip()
        if t.startswith(("s_cbranch", "s_branch")):
            mt = re.search(r"(\.LBB\d+_\d+)", t)
            if mt:
                targets[cur].append(mt.group(1))
    for b, tl in targets.items():
        for t in tl:
            if t in pos and pos[t] <= pos[b]:
                loops.append((pos[t], pos[b]))
    loops = sorted(set(loops), key=lambda x: x[1] - x[0])
    total = collections.Counter()
    for b in order:
        for op in blocks[b]:
            total[classify(op)] += 1
    print(f"kernel {lines[start].split(':')[0][:90]}: {sum(total.values())} instructions, {len(order)} blocks, "
          f"{len(loops)} loops")
    print(" whole kernel:", dict(total))
    for h, e in loops[:max_loops]:
        c = collections.Counter()
        for b in order[h:e + 1]:
            for op in blocks[b]:
                c[classify(op)] += 1
        valu = c["valu_f64"] + c["valu_dpp"] + c["valu_cmp_sel"] + c["valu_other"]
        print(f" loop {order[h]}..{order[e]} ({e - h + 1} blocks): VALU {valu} "
              f"(f64 {c['valu_f64']}, dpp {c['valu_dpp']}, cmp/sel {c['valu_cmp_sel']}, other {c['valu_other']}), "
              f"SALU {c['salu']}, LDS {c['lds']}, vmem {c['vmem']}, waits {c['wait']}, branches {c['branch']}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 12)
