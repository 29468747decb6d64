"""ctypes declarations of include/pbccs_amd.h and the loader of the in-tree libpbccs_amd.so."""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# PBCCS_LIB: load another in-tree build of the same library (A/B experiments: tools/build_ab.sh, then the ab_lib
# step of tools/gpu_steps.sh)
LIB_PATH = os.environ.get("PBCCS_LIB") or os.path.join(HERE, "_lib", "libpbccs_amd.so")

PBCCS_OK = 0
ERRORS = {-1: "EINVAL", -2: "EOOM", -3: "EDEVICE", -4: "ESTATE", -5: "ERANGE"}

_lib = None


class PbccsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"pbccs {ERRORS.get(code, code)}: {msg}")
        self.code = code


class CMutation(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("start", ctypes.c_int), ("end", ctypes.c_int), ("new_base", ctypes.c_char)]


class CArrowConfig(ctypes.Structure):
    _fields_ = [("snr", ctypes.c_double * 4), ("score_diff", ctypes.c_double),
                ("fast_score_threshold", ctypes.c_double), ("add_threshold", ctypes.c_double)]


class CRefineOptions(ctypes.Structure):
    _fields_ = [("max_iterations", ctypes.c_int), ("mutation_separation", ctypes.c_int),
                ("mutation_neighborhood", ctypes.c_int)]


class CZmwInput(ctypes.Structure):
    _fields_ = [("draft", ctypes.c_char_p), ("draft_len", ctypes.c_int), ("snr", ctypes.c_double * 4),
                ("n_reads", ctypes.c_int), ("seqs", ctypes.POINTER(ctypes.c_char_p)),
                ("lens", ctypes.POINTER(ctypes.c_int)), ("strands", ctypes.POINTER(ctypes.c_int)),
                ("tstarts", ctypes.POINTER(ctypes.c_int)), ("tends", ctypes.POINTER(ctypes.c_int)),
                ("full_pass", ctypes.POINTER(ctypes.c_ubyte))]


class CPolishOptions(ctypes.Structure):
    _fields_ = [("min_passes", ctypes.c_int), ("min_length", ctypes.c_int), ("min_zscore", ctypes.c_double),
                ("max_drop_fraction", ctypes.c_double), ("min_predicted_accuracy", ctypes.c_double),
                ("score_diff", ctypes.c_double), ("refine", CRefineOptions), ("zmws_per_batch", ctypes.c_int)]


class CZmwOutput(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int), ("consensus", ctypes.c_char_p), ("consensus_cap", ctypes.c_int),
                ("consensus_len", ctypes.c_int), ("qvs", ctypes.POINTER(ctypes.c_int)),
                ("add_read_results", ctypes.POINTER(ctypes.c_int)), ("zscores", ctypes.POINTER(ctypes.c_double)),
                ("zg", ctypes.c_double), ("za", ctypes.c_double), ("predicted_accuracy", ctypes.c_double),
                ("n_tested", ctypes.c_longlong), ("n_applied", ctypes.c_longlong), ("n_passes", ctypes.c_int),
                ("status_counts", ctypes.c_int * 5)]


class CKernelStat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 32), ("launches", ctypes.c_longlong), ("device_ms", ctypes.c_double),
                ("cells", ctypes.c_double), ("bytes", ctypes.c_double), ("wave_s", ctypes.c_double)]


class CCounters(ctypes.Structure):
    _fields_ = [("fill_launches", ctypes.c_longlong), ("score_launches", ctypes.c_longlong),
                ("score_tasks", ctypes.c_longlong), ("mutations", ctypes.c_longlong),
                ("band_top_bytes", ctypes.c_longlong), ("band_region_bytes", ctypes.c_longlong),
                ("band_used_bytes", ctypes.c_longlong), ("pool_mapped_bytes", ctypes.c_longlong),
                ("oom_retries", ctypes.c_longlong), ("create_host_ns", ctypes.c_longlong),
                ("create_upload_ns", ctypes.c_longlong), ("derive_ns", ctypes.c_longlong),
                ("fill_work", ctypes.c_longlong * 16), ("scan_reads", ctypes.c_longlong),
                ("uncertain_reads", ctypes.c_longlong), ("exact_rounds", ctypes.c_longlong),
                ("uncertain_why", ctypes.c_longlong * 4)]


class CQvModelParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in ("match", "mismatch", "mismatch_s", "branch", "branch_s", "deletion_n",
                                              "deletion_with_tag", "deletion_with_tag_s", "nce", "nce_s")] + \
               [("merge", ctypes.c_float * 4), ("merge_s", ctypes.c_float * 4)]


class CQuiverConfig(ctypes.Structure):
    _fields_ = [("params", CQvModelParams), ("moves_available", ctypes.c_int), ("score_diff", ctypes.c_float),
                ("fast_score_threshold", ctypes.c_float), ("add_threshold", ctypes.c_float),
                ("sum_product", ctypes.c_int), ("recursor", ctypes.c_int)]


class CQuiverRead(ctypes.Structure):
    _fields_ = [("seq", ctypes.c_char_p), ("len", ctypes.c_int), ("ins_qv", ctypes.POINTER(ctypes.c_float)),
                ("subs_qv", ctypes.POINTER(ctypes.c_float)), ("del_qv", ctypes.POINTER(ctypes.c_float)),
                ("del_tag", ctypes.POINTER(ctypes.c_float)), ("merge_qv", ctypes.POINTER(ctypes.c_float)),
                ("chemistry", ctypes.c_char_p), ("strand", ctypes.c_int), ("tstart", ctypes.c_int),
                ("tend", ctypes.c_int), ("threshold", ctypes.c_float)]


class CQvFeatures(ctypes.Structure):
    _fields_ = [("seq", ctypes.c_char_p), ("len", ctypes.c_int), ("ins_qv", ctypes.POINTER(ctypes.c_float)),
                ("subs_qv", ctypes.POINTER(ctypes.c_float)), ("del_qv", ctypes.POINTER(ctypes.c_float)),
                ("del_tag", ctypes.POINTER(ctypes.c_float)), ("merge_qv", ctypes.POINTER(ctypes.c_float))]


class CQuiverZmw(ctypes.Structure):
    _fields_ = [("tpl", ctypes.c_char_p), ("tpl_len", ctypes.c_int), ("reads", ctypes.POINTER(CQuiverRead)),
                ("n_reads", ctypes.c_int)]


class CQuiverResult(ctypes.Structure):
    _fields_ = [("consensus", ctypes.c_char_p), ("consensus_cap", ctypes.c_int), ("consensus_len", ctypes.c_int),
                ("qvs", ctypes.POINTER(ctypes.c_int)), ("n_tested", ctypes.c_longlong),
                ("n_applied", ctypes.c_longlong), ("converged", ctypes.c_int), ("ok", ctypes.c_int),
                ("n_active", ctypes.c_int)]


class CPoaInput(ctypes.Structure):
    _fields_ = [("seqs", ctypes.POINTER(ctypes.c_char_p)), ("lens", ctypes.POINTER(ctypes.c_int)),
                ("n_reads", ctypes.c_int)]


class CPoaOutput(ctypes.Structure):
    _fields_ = [("consensus", ctypes.c_char_p), ("cap", ctypes.c_int), ("len", ctypes.c_int),
                ("keys", ctypes.POINTER(ctypes.c_int)), ("rc", ctypes.POINTER(ctypes.c_int)),
                ("extents", ctypes.POINTER(ctypes.c_int)), ("n_keys", ctypes.c_int)]


class CCcsInput(ctypes.Structure):
    _fields_ = [("snr", ctypes.c_double * 4), ("n_subreads", ctypes.c_int), ("seqs", ctypes.POINTER(ctypes.c_char_p)),
                ("lens", ctypes.POINTER(ctypes.c_int)), ("flags", ctypes.POINTER(ctypes.c_ubyte))]


class CCcsOutput(ctypes.Structure):
    _fields_ = [("polish", CZmwOutput), ("draft", ctypes.c_char_p), ("draft_cap", ctypes.c_int),
                ("draft_len", ctypes.c_int), ("add_order", ctypes.POINTER(ctypes.c_int))]


class CPoaStats(ctypes.Structure):
    _fields_ = [("alignments", ctypes.c_longlong), ("cells", ctypes.c_longlong), ("launches", ctypes.c_longlong),
                ("trace_steps", ctypes.c_longlong), ("fill_ms", ctypes.c_double), ("trace_ms", ctypes.c_double),
                ("bytes", ctypes.c_double), ("prog_ms", ctypes.c_double), ("device_ms", ctypes.c_double),
                ("thread_ms", ctypes.c_double), ("consensus_ms", ctypes.c_double), ("total_ms", ctypes.c_double)]


# exported symbol -> (restype, argtypes); tests check that every symbol of include/pbccs_amd.h is exported
P = ctypes.c_void_p
I = ctypes.c_int
D = ctypes.c_double
PI = ctypes.POINTER(ctypes.c_int)
PD = ctypes.POINTER(ctypes.c_double)
PLL = ctypes.POINTER(ctypes.c_longlong)
PM = ctypes.POINTER(CMutation)
PF = ctypes.POINTER(ctypes.c_float)
SIGNATURES = {
    "pbccs_engine_create": (I, [I, ctypes.POINTER(P)]),
    "pbccs_engine_destroy": (None, [P]),
    "pbccs_last_error": (ctypes.c_char_p, []),
    "pbccs_device_count": (I, []),
    "pbccs_engine_counters": (I, [P, ctypes.POINTER(CCounters), I]),
    "pbccs_scorer_create": (I, [P, ctypes.POINTER(CArrowConfig), ctypes.c_char_p, I, ctypes.POINTER(P)]),
    "pbccs_scorer_destroy": (None, [P]),
    "pbccs_scorer_add_read": (I, [P, ctypes.c_char_p, I, I, I, I, D, PI]),
    "pbccs_scorer_score": (I, [P, PM, D, PD]),
    "pbccs_scorer_score_many": (I, [P, PM, I, D, PD]),
    "pbccs_scorer_scores": (I, [P, PM, D, PD]),
    "pbccs_scorer_is_favorable": (I, [P, PM, I, PI]),
    "pbccs_scorer_apply_mutations": (I, [P, PM, I]),
    "pbccs_scorer_template": (I, [P, I, ctypes.c_char_p, I, PI]),
    "pbccs_scorer_template_length": (I, [P]),
    "pbccs_scorer_num_reads": (I, [P]),
    "pbccs_scorer_read_info": (I, [P, I, PI, PI, PI, PI]),
    "pbccs_scorer_baseline_score": (I, [P, PD]),
    "pbccs_scorer_baseline_scores": (I, [P, PD, I, PI]),
    "pbccs_scorer_zscores": (I, [P, PD, PD, PD]),
    "pbccs_scorer_num_flipflops": (I, [P, PI]),
    "pbccs_refine_consensus": (I, [P, ctypes.POINTER(CRefineOptions), PLL, PLL, PI]),
    "pbccs_consensus_qvs": (I, [P, PI, I, PI]),
    "pbccs_polish_options_default": (None, [ctypes.POINTER(CPolishOptions)]),
    "pbccs_polish_batch": (I, [P, ctypes.POINTER(CZmwInput), I, ctypes.POINTER(CPolishOptions),
                               ctypes.POINTER(CZmwOutput)]),
    "pbccs_plan_batches": (I, [ctypes.POINTER(CZmwInput), I, D, I, D, PI, PI, PD, PI]),
    "pbccs_batch_create": (I, [P, ctypes.POINTER(CZmwInput), I, ctypes.POINTER(CPolishOptions), ctypes.POINTER(P)]),
    "pbccs_batch_polish": (I, [P, ctypes.POINTER(CZmwOutput)]),
    "pbccs_batch_destroy": (None, [P]),
    "pbccs_batch_polish_many": (I, [ctypes.POINTER(P), I, ctypes.POINTER(ctypes.POINTER(CZmwOutput))]),
    "pbccs_engine_set_concurrency": (I, [P, I]),
    "pbccs_engine_reserve_pool": (I, [P, ctypes.c_size_t]),
    "pbccs_engine_set_profiling": (I, [P, I]),
    "pbccs_engine_kernel_stats": (I, [P, ctypes.POINTER(CKernelStat), I, PI, I]),
    # Quiver family
    "pbccs_quiver_scorer_create": (I, [P, ctypes.POINTER(CQuiverConfig), ctypes.POINTER(ctypes.c_char_p), I,
                                       ctypes.c_char_p, I, ctypes.POINTER(P)]),
    "pbccs_quiver_scorer_destroy": (None, [P]),
    "pbccs_quiver_scorer_add_read": (I, [P, ctypes.c_char_p, I, PF, PF, PF, PF, PF, ctypes.c_char_p, I, I, I,
                                         ctypes.c_float, PI]),
    "pbccs_quiver_scorer_score_many": (I, [P, PM, I, I, PF]),
    "pbccs_quiver_scorer_scores": (I, [P, PM, ctypes.c_float, PF]),
    "pbccs_quiver_scorer_read_score_mutation": (I, [P, I, PM, PF]),
    "pbccs_quiver_scorer_is_favorable": (I, [P, PM, I, PI]),
    "pbccs_quiver_scorer_apply_mutations": (I, [P, PM, I]),
    "pbccs_quiver_scorer_template": (I, [P, I, ctypes.c_char_p, I, PI]),
    "pbccs_quiver_scorer_num_reads": (I, [P]),
    "pbccs_quiver_scorer_read_info": (I, [P, I, PI, PI, PI, PI]),
    "pbccs_quiver_scorer_baseline_score": (I, [P, PF]),
    "pbccs_quiver_scorer_baseline_scores": (I, [P, PF, I, PI]),
    "pbccs_quiver_scorer_num_flipflops": (I, [P, PI]),
    "pbccs_quiver_scorer_allocated_entries": (I, [P, I, PLL, PLL]),
    "pbccs_quiver_scorer_alignment": (I, [P, I, ctypes.c_char_p, ctypes.c_char_p, I, PI]),
    "pbccs_quiver_refine_consensus": (I, [P, ctypes.POINTER(CRefineOptions), PLL, PLL, PI]),
    "pbccs_quiver_consensus_qvs": (I, [P, PI, I, PI]),
    "pbccs_qv_evaluator_moves": (I, [P, ctypes.POINTER(CQvFeatures), ctypes.c_char_p, I, ctypes.POINTER(CQvModelParams),
                                     I, I, PI, PI, I, PF, PF, PF, PF]),
    "pbccs_quiver_polish_batch": (I, [P, ctypes.POINTER(CQuiverConfig), ctypes.POINTER(ctypes.c_char_p), I,
                                      ctypes.POINTER(CQuiverZmw), I, ctypes.POINTER(CRefineOptions),
                                      ctypes.POINTER(CQuiverResult)]),
    # POA draft
    "pbccs_poa_batch": (I, [P, ctypes.POINTER(CPoaInput), I, ctypes.c_longlong, I, ctypes.POINTER(CPoaOutput)]),
    "pbccs_sparse_poa_create": (I, [P, ctypes.POINTER(P)]),
    "pbccs_sparse_poa_destroy": (None, [P]),
    "pbccs_sparse_poa_orient_and_add_read": (I, [P, ctypes.c_char_p, I, ctypes.c_float, PI]),
    "pbccs_sparse_poa_find_consensus": (I, [P, I, ctypes.c_char_p, I, PI, PI, PI, PI]),
    "pbccs_sparse_poa_graphviz": (I, [P, I, I, ctypes.c_char_p, I, PI]),
    "pbccs_poa_consensus": (I, [P, ctypes.POINTER(ctypes.c_char_p), PI, I, I, I, ctypes.c_char_p, I, PI, I,
                                ctypes.c_char_p, I, PI]),
    "pbccs_poa_stats_get": (I, [P, ctypes.POINTER(CPoaStats), I]),
    "pbccs_ccs_batch": (I, [P, ctypes.POINTER(CCcsInput), I, ctypes.c_longlong, ctypes.POINTER(CPolishOptions),
                            ctypes.POINTER(CCcsOutput)]),
}


def load():
    """Load the HIP engine.  Raises (never falls back) when the library has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PbccsError(-3, f"{LIB_PATH} is missing: run __graft_entry__.build() (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc != PBCCS_OK:
        msg = load().pbccs_last_error()
        raise PbccsError(rc, msg.decode() if msg else "")
    return rc
