import sys, time
sys.path.insert(0, '.')
import pbccs_amd
from pbccs_amd import synth
zs = synth.make_zmws(64, 2000, 10, seed=5)
eng = pbccs_amd.Engine(0)
eng.set_profiling(True)
b = pbccs_amd.PreparedBatch(zs, pbccs_amd.ConsensusSettings(max_iterations=1), eng)
t = time.time(); b.polish(); print("polish", time.time() - t)
print({k: (v['launches'], round(v['device_ms'], 2), v['cells']) for k, v in eng.kernel_stats().items()})
