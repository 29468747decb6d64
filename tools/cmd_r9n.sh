# hybrid scan vs exact: per-launch cycles per cell of the tall paths (PBCCS_FILL_PATHS=2), configs[3] at 300 ZMWs
TAG=r9n MIXN=300 MIXARGS="--cpu-sample 0" VARIANTS="PBCCS_SCAN_PATHS=3 PBCCS_FILL_PATHS=2;PBCCS_SCAN_PATHS=1 PBCCS_FILL_PATHS=2;PBCCS_SCAN_PATHS=3 PBCCS_FILL_PATHS=2 PBCCS_SCAN_DEV_SCALE=1;PBCCS_SCAN_PATHS=1 PBCCS_FILL_PATHS=2" bash tools/gpu_steps.sh abmixed
for k in 1 2 3 4; do python3 - gpurun_out/r9n/abmixed_$k.err gpurun_out/r9n/abmixed_$k.json <<'PY'
import json, re, sys
d = json.load(open(sys.argv[2]))
agg = {}
for ln in open(sys.argv[1]):
    m = re.search(r"\[fillread\] path=(\d) n=(\d+) span=([\d.]+)ms .* all: ([\d.]+) cyc/cell", ln)
    if m:
        a = agg.setdefault(m.group(1), [0, 0, 0.0, 0.0])
        a[0] += 1; a[1] += int(m.group(2)); a[2] += float(m.group(3)); a[3] += float(m.group(4)) * int(m.group(2))
print(d["value"], d["certified_scan"]["exact_rounds"], {p: {"launches": a[0], "reads": a[1], "span_s": round(a[2] / 1e3, 1), "cyc_per_cell": round(a[3] / max(1, a[1]), 1)} for p, a in sorted(agg.items())})
PY
done
