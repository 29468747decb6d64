#!/usr/bin/env python3
"""How the restatement's polish time grows with bench.py's cost model (template length x read bases), measured on
controlled ZMWs (all full passes, fixed SNR, so no gate cuts a ZMW short): the exponent alpha of t = a cost^alpha
that bench.py's CPU leg uses when its capped sample cannot determine the slope (test infrastructure: it runs the
oracle, like the CPU leg).  Usage: python tests/calibrate_cpu_alpha.py [out.json]"""
import json
import math
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import oracle as O  # noqa: E402
from pbccs_amd import shard, synth  # noqa: E402

SHAPES = [(1000, 10), (2000, 10), (4000, 10), (8000, 10), (2000, 5), (2000, 20), (4000, 20)]


def main(out=None):
    zs = []
    for k, (L, P) in enumerate(SHAPES):
        zs += [(L, P, z) for z in synth.make_zmws(2, L, P, seed=900 + k)]

    def one(item):
        L, P, z = item
        t = time.perf_counter()
        O.polish_zmw(z["draft"], z["reads"], z["snr"])
        return L, P, shard.zmw_cost(z), time.perf_counter() - t

    O.lib()
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        rows = list(ex.map(one, zs))
    pts = [(math.log(c), math.log(t)) for _, _, c, t in rows]
    mx = sum(x for x, _ in pts) / len(pts)
    my = sum(y for _, y in pts) / len(pts)
    alpha = sum((x - mx) * (y - my) for x, y in pts) / sum((x - mx) ** 2 for x, _ in pts)
    res = {"alpha": round(alpha, 3), "shapes": [{"length": L, "passes": P, "cost": c, "s": round(t, 3)}
                                                for L, P, c, t in rows],
           "note": "oracle/arrow_oracle.cpp polish of synthetic full-pass ZMWs, one per thread (8 threads in "
                   "parallel), least squares of log t on log cost"}
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
