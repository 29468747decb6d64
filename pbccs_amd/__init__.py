"""pbccs_amd -- MI355X-native consensus polishing (the pbccs / ConsensusCore Arrow hot path).

Python mirror of the reference's polishing API, calling the HIP engine through the C ABI in
include/pbccs_amd.h (libpbccs_amd.so, built in-tree by __graft_entry__.build()).  Names follow
ConsensusCore: ArrowConfig, ArrowMultiReadMutationScorer, Mutation, RefineConsensus, ConsensusQVs.
There is no CPU fallback: if the library is missing or no GPU is present, calls raise.
"""
import ctypes
import math
import os

# Batches in flight each polish on their own HIP streams; HIP's default of 4 hardware queues makes the
# streams of different batches share queues (a long fill of one batch then blocks the others).  Takes
# effect only if the HIP runtime has not been initialised yet in this process.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:   # the boxes export HIP's default (4)
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

from . import lib as _lib_mod
from .lib import PbccsError, load

INSERTION, DELETION, SUBSTITUTION = 0, 1, 2
FORWARD_STRAND, REVERSE_STRAND = 0, 1
SUCCESS, ALPHABETAMISMATCH, MEM_FAIL, POOR_ZSCORE, OTHER = 0, 1, 2, 3, 4
AddReadResultNames = ["SUCCESS", "ALPHA/BETA MISMATCH", "EXCESSIVE MEMORY USAGE", "POOR Z-SCORE", "OTHER"]
ZMW_STATUS = ["Success", "NoSubreads", "TooShort", "TooManyUnusable", "TooFewPasses", "NonConvergent",
              "PoorQuality", "Other"]
DBL_MAX = 1.7976931348623157e308


class Mutation:
    """ConsensusCore::Mutation for single-base edits (Mutation.hpp:56-129)."""

    __slots__ = ("type", "start", "end", "new_base")

    def __init__(self, mtype, position, base="-"):
        self.type = mtype
        self.start = position
        self.end = position if mtype == INSERTION else position + 1
        self.new_base = "-" if mtype == DELETION else base

    def _c(self):
        return _lib_mod.CMutation(self.type, self.start, self.end, self.new_base.encode()[:1] or b"-")

    def __repr__(self):
        name = ["Insertion", "Deletion", "Substitution"][self.type]
        return f"{name}({self.new_base})@{self.start}"

    def __eq__(self, o):
        return (self.type, self.start, self.end, self.new_base) == (o.type, o.start, o.end, o.new_base)

    def __hash__(self):
        return hash((self.type, self.start, self.end, self.new_base))


class ArrowConfig:
    """ArrowConfig(ContextParameters(SNR), BandingOptions(scoreDiff), fastScoreThreshold, addThreshold)."""

    def __init__(self, snr, score_diff=12.5, fast_score_threshold=-12.5, add_threshold=float("nan")):
        self.snr = tuple(float(x) for x in snr)
        self.score_diff = float(score_diff)
        self.fast_score_threshold = float(fast_score_threshold)
        self.add_threshold = float(add_threshold)

    def _c(self):
        c = _lib_mod.CArrowConfig()
        for i in range(4):
            c.snr[i] = self.snr[i]
        c.score_diff = self.score_diff
        c.fast_score_threshold = self.fast_score_threshold
        c.add_threshold = self.add_threshold
        return c


class Engine:
    """One engine per GPU (device ordinal)."""

    def __init__(self, device=0):
        L = load()
        h = ctypes.c_void_p()
        _lib_mod.check(L.pbccs_engine_create(device, ctypes.byref(h)))
        self._h = h
        self._lib = L   # kept for interpreter shutdown, when module globals are already cleared
        self.device = device

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.pbccs_engine_destroy(self._h)
            self._h = None

    def set_concurrency(self, batches_in_flight):
        """Workspace slots = batches polished at the same time by polish_many (set before creating batches)."""
        _lib_mod.check(load().pbccs_engine_set_concurrency(self._h, int(batches_in_flight)))

    def reserve_pool(self, bytes_per_slot):
        """Map each workspace slot's band pool now (a one-time cost a long run pays once)."""
        _lib_mod.check(load().pbccs_engine_reserve_pool(self._h, int(bytes_per_slot)))

    def set_profiling(self, on=True):
        _lib_mod.check(load().pbccs_engine_set_profiling(self._h, 1 if on else 0))

    def kernel_stats(self, reset=False):
        arr = (_lib_mod.CKernelStat * 16)()
        n = ctypes.c_int()
        _lib_mod.check(load().pbccs_engine_kernel_stats(self._h, arr, 16, ctypes.byref(n), 1 if reset else 0))
        return {arr[i].name.decode(): {"launches": arr[i].launches, "device_ms": arr[i].device_ms,
                                       "cells": arr[i].cells, "bytes": arr[i].bytes, "wave_s": arr[i].wave_s}
                for i in range(n.value)}

    def counters(self, reset=False):
        c = _lib_mod.CCounters()
        _lib_mod.check(load().pbccs_engine_counters(self._h, ctypes.byref(c), 1 if reset else 0))
        return {k: (list(getattr(c, k)) if k in ("fill_work", "uncertain_why") else getattr(c, k))
                for k, _ in _lib_mod.CCounters._fields_}


_default_engine = None


def default_engine():
    global _default_engine
    if _default_engine is None:
        _default_engine = Engine(int(os.environ.get("PBCCS_DEVICE", os.environ.get("LOCAL_RANK", "0"))))
    return _default_engine


class ArrowMultiReadMutationScorer:
    """ConsensusCore::Arrow::ArrowMultiReadMutationScorer on the GPU (MultiReadMutationScorer.hpp:82-284)."""

    def __init__(self, config, tpl, engine=None):
        self.engine = engine or default_engine()
        self.config = config
        h = ctypes.c_void_p()
        b = tpl.encode()
        _lib_mod.check(load().pbccs_scorer_create(self.engine._h, ctypes.byref(config._c()), b, len(b), ctypes.byref(h)))
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            load().pbccs_scorer_destroy(self._h)
            self._h = None

    def AddRead(self, seq, strand=FORWARD_STRAND, template_start=0, template_end=None, threshold=None):
        if template_end is None:
            template_end = self.TemplateLength()
        if threshold is None:
            threshold = self.config.add_threshold
        res = ctypes.c_int()
        b = seq.encode()
        _lib_mod.check(load().pbccs_scorer_add_read(self._h, b, len(b), strand, template_start, template_end,
                                                    float(threshold), ctypes.byref(res)))
        return res.value

    def Score(self, m, fast_score_threshold=-DBL_MAX):
        v = ctypes.c_double()
        _lib_mod.check(load().pbccs_scorer_score(self._h, ctypes.byref(m._c()), fast_score_threshold, ctypes.byref(v)))
        return v.value

    def FastScore(self, m):
        return self.Score(m, self.config.fast_score_threshold)

    def ScoreMany(self, muts, fast_score_threshold=-DBL_MAX):
        arr = (_lib_mod.CMutation * max(1, len(muts)))(*[m._c() for m in muts])
        out = (ctypes.c_double * max(1, len(muts)))()
        _lib_mod.check(load().pbccs_scorer_score_many(self._h, arr, len(muts), fast_score_threshold, out))
        return list(out[: len(muts)])

    def Scores(self, m, unscored_value=0.0):
        out = (ctypes.c_double * max(1, self.NumReads()))()
        _lib_mod.check(load().pbccs_scorer_scores(self._h, ctypes.byref(m._c()), unscored_value, out))
        return list(out[: self.NumReads()])

    def IsFavorable(self, m):
        f = ctypes.c_int()
        _lib_mod.check(load().pbccs_scorer_is_favorable(self._h, ctypes.byref(m._c()), 0, ctypes.byref(f)))
        return bool(f.value)

    def FastIsFavorable(self, m):
        f = ctypes.c_int()
        _lib_mod.check(load().pbccs_scorer_is_favorable(self._h, ctypes.byref(m._c()), 1, ctypes.byref(f)))
        return bool(f.value)

    def ApplyMutations(self, muts):
        arr = (_lib_mod.CMutation * max(1, len(muts)))(*[m._c() for m in muts])
        _lib_mod.check(load().pbccs_scorer_apply_mutations(self._h, arr, len(muts)))

    def Template(self, strand=FORWARD_STRAND):
        n = ctypes.c_int()
        cap = self.TemplateLength() + 1
        buf = ctypes.create_string_buffer(cap)
        _lib_mod.check(load().pbccs_scorer_template(self._h, strand, buf, cap, ctypes.byref(n)))
        return buf.value.decode()

    def TemplateLength(self):
        return load().pbccs_scorer_template_length(self._h)

    def NumReads(self):
        return load().pbccs_scorer_num_reads(self._h)

    def ReadInfo(self, i):
        a, s, ts, te = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib_mod.check(load().pbccs_scorer_read_info(self._h, i, ctypes.byref(a), ctypes.byref(s), ctypes.byref(ts),
                                                     ctypes.byref(te)))
        return {"active": bool(a.value), "strand": s.value, "template_start": ts.value, "template_end": te.value}

    def BaselineScore(self):
        v = ctypes.c_double()
        _lib_mod.check(load().pbccs_scorer_baseline_score(self._h, ctypes.byref(v)))
        return v.value

    def BaselineScores(self):
        out = (ctypes.c_double * max(1, self.NumReads()))()
        n = ctypes.c_int()
        _lib_mod.check(load().pbccs_scorer_baseline_scores(self._h, out, self.NumReads(), ctypes.byref(n)))
        return list(out[: n.value])

    def ZScores(self):
        zg, za = ctypes.c_double(), ctypes.c_double()
        out = (ctypes.c_double * max(1, self.NumReads()))()
        _lib_mod.check(load().pbccs_scorer_zscores(self._h, ctypes.byref(zg), ctypes.byref(za), out))
        return (zg.value, za.value), list(out[: self.NumReads()])

    def NumFlipFlops(self):
        out = (ctypes.c_int * max(1, self.NumReads()))()
        _lib_mod.check(load().pbccs_scorer_num_flipflops(self._h, out))
        return list(out[: self.NumReads()])


def RefineConsensus(mms, max_iterations=40, mutation_separation=10, mutation_neighborhood=20):
    """bool RefineConsensus(MRMS&, size_t* nTested, size_t* nApplied, const RefineOptions&) -> (converged, nT, nA).
    Templated on the scorer in the reference (Consensus.hpp:63-67): Arrow or Quiver scorers."""
    if isinstance(mms, _quiver.QuiverMultiReadMutationScorer):
        return _quiver.RefineConsensus(mms, max_iterations, mutation_separation, mutation_neighborhood)
    o = _lib_mod.CRefineOptions(max_iterations, mutation_separation, mutation_neighborhood)
    nt, na, conv = ctypes.c_longlong(0), ctypes.c_longlong(0), ctypes.c_int()
    _lib_mod.check(load().pbccs_refine_consensus(mms._h, ctypes.byref(o), ctypes.byref(nt), ctypes.byref(na),
                                                 ctypes.byref(conv)))
    return bool(conv.value), nt.value, na.value


def ConsensusQVs(mms):
    if isinstance(mms, _quiver.QuiverMultiReadMutationScorer):
        return _quiver.ConsensusQVs(mms)
    cap = mms.TemplateLength()
    out = (ctypes.c_int * max(1, cap))()
    n = ctypes.c_int()
    _lib_mod.check(load().pbccs_consensus_qvs(mms._h, out, cap, ctypes.byref(n)))
    return list(out[: n.value])


def QVsToASCII(qvs):
    """include/pacbio/ccs/Consensus.h:327-338"""
    return "".join(chr(min(max(0, q), 93) + 33) for q in qvs)


from .polish import (ConsensusSettings, PreparedBatch, plan_batches, polish_many, polish_stream,  # noqa: E402
                     polish_zmws)  # batched ccs driver
from . import quiver as _quiver  # noqa: E402
from .quiver import (QvModelParams, QuiverConfig, QuiverConfigTable,  # noqa: E402,F401
                     QuiverMultiReadMutationScorer, QvEvaluator, QvSequenceFeatures, ALL_MOVES, BASIC_MOVES)

__all__ = [
    "ArrowConfig", "ArrowMultiReadMutationScorer", "ConsensusQVs", "ConsensusSettings", "Engine", "Mutation",
    "PbccsError", "QVsToASCII", "RefineConsensus", "polish_many", "polish_zmws", "polish_stream", "plan_batches", "INSERTION", "DELETION", "SUBSTITUTION",
    "FORWARD_STRAND", "REVERSE_STRAND",
]
