"""Debug: 10 kb fine-grained AddRead one read at a time with timing (GPU box)."""
import sys, time
sys.path.insert(0, ".")
import pbccs_amd as P
from pbccs_amd import synth
zs = synth.make_zmws(2, 10000, 8, seed=81)
for zi, z in enumerate(zs):
    g = P.ArrowMultiReadMutationScorer(P.ArrowConfig([10.0, 7.0, 5.0, 11.0]), z["draft"])
    for k, r in enumerate(z["reads"]):
        t = time.time()
        res = g.AddRead(r["seq"], r.get("strand", 0), r.get("ts", 0), r.get("te", len(z["draft"])), float("nan"))
        print(zi, k, len(r["seq"]), res, "%.3fs" % (time.time() - t), flush=True)
    print(g.NumFlipFlops(), flush=True)
