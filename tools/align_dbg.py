import ctypes, json, subprocess, sys
sys.path.insert(0, '.')
import pbccs_amd as P
from pbccs_amd import lib as L
d = json.load(open('tests/golden/quiver_kats.json'))
k = d['kats'][0]
qp = P.QvModelParams(**d['params'])
cfg = P.QuiverConfig(qp, moves=k['moves'], score_diff=k['score_diff'], fast_score_threshold=k['fast_threshold'])
s = P.QuiverMultiReadMutationScorer(cfg, k['tpl'])
s.AddRead(k['reads'][0]['seq'], 0, 0, len(k['tpl']))
print('py first', s.Alignment(0))
print('py second', s.Alignment(0))
n = ctypes.c_int()
rc = L.load().pbccs_quiver_scorer_alignment(s._h, 0, None, None, 0, ctypes.byref(n))
print('probe rc', rc, n.value)
print('py after probe', s.Alignment(0))
