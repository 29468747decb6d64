"""Debug: MatrixTester KATs through the scorer API, printing every value (GPU)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import pbccs_amd as P
k = json.load(open("tests/golden/arrow_kats.json"))
print("HWQ", os.environ.get("GPU_MAX_HW_QUEUES"), os.environ.get("AMD_SERIALIZE_KERNEL"), os.environ.get("AMD_SERIALIZE_COPY"))
bad = 0
for b in k["baseline"]:
    g = P.ArrowMultiReadMutationScorer(P.ArrowConfig(k["snr"]), b["tpl"])
    for r in b["reads"]:
        g.AddRead(r)
    v = g.BaselineScore()
    ok = abs(1 - v / b["expected"]) < k["tolerance_rel"]
    bad += not ok
    print("baseline", v, b["expected"], ok, g.BaselineScores(), g.NumFlipFlops())
for m in k["mutations"]:
    g = P.ArrowMultiReadMutationScorer(P.ArrowConfig(k["snr"]), m["tpl"])
    for r in m["reads"] * m.get("copies", 1):
        g.AddRead(r)
    mu = P.Mutation(m["type"], m["start"], m["base"])
    v = g.Score(mu) / m.get("divide_by", 1)
    ok = abs(1 - v / m["expected"]) < k["tolerance_rel"]
    bad += not ok
    print("mut", m["line"], v, m["expected"], ok, g.Scores(mu, -1e300), g.BaselineScores())
print("BAD", bad)
