"""Diagnostics: polish a small synthetic batch with fill tracing and print per-kernel stats."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import argparse
ap = argparse.ArgumentParser()
ap.add_argument("--zmws", type=int, default=256)
ap.add_argument("--length", type=int, default=2000)
ap.add_argument("--passes", type=int, default=10)
ap.add_argument("--iters", type=int, default=3)
a = ap.parse_args()
import torch  # noqa: F401  (same HIP runtime as the engine)
import pbccs_amd
from pbccs_amd import synth
zs = synth.make_zmws(a.zmws, a.length, a.passes, seed=5)
eng = pbccs_amd.Engine(0)
eng.set_profiling(True)
b = pbccs_amd.PreparedBatch(zs, pbccs_amd.ConsensusSettings(max_iterations=a.iters), eng)
t = time.time(); b.polish(); print("polish", time.time() - t, flush=True)
print({k: (v['launches'], round(v['device_ms'], 2), v['cells']) for k, v in eng.kernel_stats().items()})
