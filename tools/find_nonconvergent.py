#!/usr/bin/env python3
"""Find synthetic ZMWs that the oracle polishes to NonConvergent (test-case discovery; CPU only)."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from pbccs_amd import synth  # noqa: E402

n, length, passes, seed = (int(x) for x in sys.argv[1:5])
zs = synth.make_zmws(n, length, passes, seed=seed)
O.lib()
with ThreadPoolExecutor(max_workers=int(os.environ.get("THREADS", "8"))) as ex:
    res = list(ex.map(lambda z: O.polish_zmw(z["draft"], z["reads"], z["snr"]), zs))
for i, r in enumerate(res):
    if not r["converged"]:
        print(f"seed={seed} n={n} index={i} n_tested={r['n_tested']} n_applied={r['n_applied']}", flush=True)
