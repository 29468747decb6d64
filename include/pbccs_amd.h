/*
 * pbccs_amd.h -- C ABI of the MI355X consensus-polishing engine (drop-in for pbccs' polish path).
 *
 * The reference's hot path is a C++ template API, not an FFI: pbccs' per-ZMW driver
 * (include/pacbio/ccs/Consensus.h:436-512) drives ConsensusCore's
 *   Arrow::MultiReadMutationScorer  (ConsensusCore/include/ConsensusCore/Arrow/MultiReadMutationScorer.hpp:82-284)
 *   RefineConsensus / ConsensusQVs  (ConsensusCore/include/ConsensusCore/Consensus.hpp:63-79, Consensus-inl.hpp:159-295)
 * Every entry point below replaces one of those calls (cited per function); include/pbccs_amd/ConsensusCore.hpp
 * wraps them back into the reference's C++ class names so a Consensus.h-equivalent compiles unchanged
 * (INTEGRATION.md).  Plain pointers and sizes only; nothing throws across this boundary.
 */
#ifndef PBCCS_AMD_H
#define PBCCS_AMD_H

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes -------------------------------------------------------------------------- */
#define PBCCS_OK 0
#define PBCCS_EINVAL (-1)   /* bad argument (InvalidInputError, std::out_of_range in the reference) */
#define PBCCS_EOOM (-2)     /* device allocation failed */
#define PBCCS_EDEVICE (-3)  /* HIP runtime / kernel failure */
#define PBCCS_ESTATE (-4)   /* call out of order (e.g. BadExecutionOrderException) */
#define PBCCS_ERANGE (-5)   /* caller buffer too small; the required size is returned through *len */

/* Mutation types (ConsensusCore/include/ConsensusCore/Mutation.hpp:50-53) */
#define PBCCS_INSERTION 0
#define PBCCS_DELETION 1
#define PBCCS_SUBSTITUTION 2
/* Strands (ConsensusCore/include/ConsensusCore/Read.hpp:66-70) */
#define PBCCS_FORWARD_STRAND 0
#define PBCCS_REVERSE_STRAND 1
/* AddReadResult (ConsensusCore/include/ConsensusCore/Arrow/MultiReadMutationScorer.hpp:60) */
#define PBCCS_ADD_SUCCESS 0
#define PBCCS_ADD_ALPHABETAMISMATCH 1
#define PBCCS_ADD_MEM_FAIL 2
#define PBCCS_ADD_POOR_ZSCORE 3
#define PBCCS_ADD_OTHER 4
/* Per-ZMW outcome (pbccs ResultType counters, include/pacbio/ccs/Consensus.h:150-210) */
#define PBCCS_ZMW_SUCCESS 0
#define PBCCS_ZMW_NO_SUBREADS 1
#define PBCCS_ZMW_TOO_SHORT 2
#define PBCCS_ZMW_TOO_MANY_UNUSABLE 3
#define PBCCS_ZMW_TOO_FEW_PASSES 4
#define PBCCS_ZMW_NON_CONVERGENT 5
#define PBCCS_ZMW_POOR_QUALITY 6
#define PBCCS_ZMW_OTHER 7

typedef struct pbccs_engine pbccs_engine; /* one per GPU; externally synchronised */
typedef struct pbccs_scorer pbccs_scorer; /* one ArrowMultiReadMutationScorer */

/* A single-base mutation: start/end as in ConsensusCore::Mutation (insertion: end == start). */
typedef struct {
    int type;
    int start;
    int end;
    char new_base; /* 'A','C','G','T'; ignored for deletions */
} pbccs_mutation;

/* ArrowConfig + BandingOptions (ConsensusCore/include/ConsensusCore/Arrow/ArrowConfig.hpp:104-128) */
typedef struct {
    double snr[4];               /* SNR(A, C, G, T) -> ContextParameters */
    double score_diff;           /* BandingOptions::ScoreDiff (ccs: 12.5) */
    double fast_score_threshold; /* ArrowConfig::FastScoreThreshold (default -12.5) */
    double add_threshold;        /* ArrowConfig::AddThreshold (default NaN = no z-score gate) */
} pbccs_arrow_config;

/* RefineOptions (ConsensusCore/include/ConsensusCore/Consensus.hpp:48-60), defaults 40/10/20 */
typedef struct {
    int max_iterations;
    int mutation_separation;
    int mutation_neighborhood;
} pbccs_refine_options;

/* ---- engine --------------------------------------------------------------------------------- */
int pbccs_engine_create(int device, pbccs_engine** out);
void pbccs_engine_destroy(pbccs_engine* eng);
const char* pbccs_last_error(void); /* thread-local message of the last failed call */
int pbccs_device_count(void);

/* ---- ArrowMultiReadMutationScorer (Arrow/MultiReadMutationScorer.cpp) ---------------------- */
/* MultiReadMutationScorer(const ArrowConfig&, std::string tpl)                       (.cpp:143-154) */
int pbccs_scorer_create(pbccs_engine* eng, const pbccs_arrow_config* cfg, const char* tpl, int tpl_len,
                        pbccs_scorer** out);
void pbccs_scorer_destroy(pbccs_scorer* s);
/* AddReadResult AddRead(const MappedArrowRead&, double threshold)                    (.cpp:275-325)
 * threshold NaN = no z-score gate; pass cfg->add_threshold for the one-argument overload (.cpp:334). */
int pbccs_scorer_add_read(pbccs_scorer* s, const char* seq, int len, int strand, int tstart, int tend,
                          double threshold, int* result);
/* double Score(const Mutation&, double fastScoreThreshold = -DBL_MAX)                (.cpp:338-368)
 * FastScore(m) == Score(m, cfg->fast_score_threshold)                                (.cpp:380-383) */
int pbccs_scorer_score(pbccs_scorer* s, const pbccs_mutation* m, double fast_threshold, double* score);
/* Batched Score over n mutations (same semantics per element). */
int pbccs_scorer_score_many(pbccs_scorer* s, const pbccs_mutation* m, int n, double fast_threshold, double* scores);
/* std::vector<double> Scores(const Mutation&, double unscoredValue)                  (.cpp:384-417)
 * per_read must hold NumReads() entries. */
int pbccs_scorer_scores(pbccs_scorer* s, const pbccs_mutation* m, double unscored, double* per_read);
/* IsFavorable / FastIsFavorable (score > 0.04)                                       (.cpp:428-440) */
int pbccs_scorer_is_favorable(pbccs_scorer* s, const pbccs_mutation* m, int fast, int* favorable);
/* void ApplyMutations(const std::vector<Mutation>&)                                  (.cpp:235-267) */
int pbccs_scorer_apply_mutations(pbccs_scorer* s, const pbccs_mutation* m, int n);
/* std::string Template(StrandEnum)                                                   (.cpp:183-188)
 * writes at most cap bytes (NUL-terminated); *len = template length. */
int pbccs_scorer_template(pbccs_scorer* s, int strand, char* out, int cap, int* len);
int pbccs_scorer_template_length(pbccs_scorer* s);                                 /* (.cpp:169-173) */
int pbccs_scorer_num_reads(pbccs_scorer* s);                                       /* (.cpp:176-180) */
/* Read(i): active flag and current mapping (MappedArrowRead*, NULL when inactive)    (.cpp:192-196) */
int pbccs_scorer_read_info(pbccs_scorer* s, int i, int* active, int* strand, int* tstart, int* tend);
/* double BaselineScore() / std::vector<double> BaselineScores()                      (.cpp:495-520) */
int pbccs_scorer_baseline_score(pbccs_scorer* s, double* score);
int pbccs_scorer_baseline_scores(pbccs_scorer* s, double* out, int cap, int* n);
/* ZScores(): ((zg, za), per-read z)  per_read must hold NumReads() entries      (.hpp:208-263) */
int pbccs_scorer_zscores(pbccs_scorer* s, double* zg, double* za, double* per_read);
/* NumFlipFlops() per read                                                            (.cpp:480-488) */
int pbccs_scorer_num_flipflops(pbccs_scorer* s, int* out);

/* bool RefineConsensus(MRMS&, size_t* nTested, size_t* nApplied, const RefineOptions&)
 *                                                       (Consensus.hpp:63-67, Consensus-inl.hpp:159-262) */
int pbccs_refine_consensus(pbccs_scorer* s, const pbccs_refine_options* opts, long long* n_tested,
                           long long* n_applied, int* converged);
/* std::vector<int> ConsensusQVs(MRMS&)                  (Consensus.hpp:77-78, Consensus-inl.hpp:274-295) */
int pbccs_consensus_qvs(pbccs_scorer* s, int* qvs, int cap, int* n);

/* ---- batched ccs polish: Consensus<>() after the POA, for many ZMWs per call ------------------
 * Mirrors include/pacbio/ccs/Consensus.h:436-552 from `ArrowConfig config(...)` on: AddRead(mr,
 * MinZScore) per read with status counts, the MinPasses / MaxDropFraction gates, ZScores(),
 * RefineConsensus(), ConsensusQVs(), predicted accuracy and the MinPredictedAccuracy gate.
 * Results are written in input order (WorkQueue.h:128-167 ordering). */
typedef struct {
    const char* draft;         /* POA consensus (ACGT) */
    int draft_len;
    double snr[4];
    int n_reads;
    const char* const* seqs;   /* read bases as passed to MappedArrowRead (already extent-clipped); NULL: a
                                * read the driver did not add (POA key -1 or ExtractMappedRead none,
                                * Consensus.h:448-451) -- counted in the drop fraction's denominator only */
    const int* lens;
    const int* strands;
    const int* tstarts;        /* mapped window on the draft [tstart, tend) */
    const int* tends;
    const unsigned char* full_pass; /* ADAPTER_BEFORE && ADAPTER_AFTER per read (NULL: all full passes) */
} pbccs_zmw_input;

typedef struct {
    int min_passes;               /* ConsensusSettings::MinPasses (3) */
    int min_length;               /* ConsensusSettings::MinLength (10): draft shorter -> TOO_SHORT */
    double min_zscore;            /* ConsensusSettings::MinZScore (-5; NaN disables) */
    double max_drop_fraction;     /* ConsensusSettings::MaxDropFraction (0.34) */
    double min_predicted_accuracy;/* ConsensusSettings::MinPredictedAccuracy (0.90) */
    double score_diff;            /* BandingOptions(12.5) */
    pbccs_refine_options refine;  /* {40, 10, 20} */
    int zmws_per_batch;           /* device batch size (0 = auto from the memory budget) */
} pbccs_polish_options;

typedef struct {
    int status;          /* PBCCS_ZMW_* */
    char* consensus;     /* caller buffer, consensus_cap bytes; NUL-terminated */
    int consensus_cap;
    int consensus_len;   /* -required length when the buffer was too small */
    int* qvs;            /* caller buffer, consensus_cap entries (raw, unclipped QVs) */
    int* add_read_results; /* caller buffer, n_reads entries (-1: read not added) */
    double* zscores;     /* caller buffer, n_reads entries */
    double zg, za;
    double predicted_accuracy;
    long long n_tested, n_applied;
    int n_passes;
    int status_counts[5]; /* AddReadResult histogram */
} pbccs_zmw_output;

void pbccs_polish_options_default(pbccs_polish_options* o);
/* One call: upload, polish and download n ZMWs -- the ZMW work queue of ccs (src/main/ccs.cpp:222-262,
 * WorkQueue.h:64-167) for a stream of heterogeneous ZMWs.  With opts->zmws_per_batch == 0 the ZMWs are
 * bucketed by template length and pass count into device batches sized to the free device memory
 * (pbccs_plan_batches), and the engine's workspace slots pull batches largest-first from a shared queue;
 * otherwise consecutive chunks of zmws_per_batch.  Outputs land in input order either way.  A batch that
 * runs the device out of memory (PBCCS_EOOM) while the other slots hold theirs is rerun alone after the
 * slots' band pools are unmapped, halved while it still does not fit. */
int pbccs_polish_batch(pbccs_engine* eng, const pbccs_zmw_input* in, int n, const pbccs_polish_options* opts,
                       pbccs_zmw_output* out);

/* Host-only batch plan behind pbccs_polish_batch (no device needed).  ZMWs are ordered by (draft length,
 * read count); a batch closes when it holds max_per_batch ZMWs, when its estimated FP64 band footprint
 * would pass budget_bytes, or when a draft is more than max_len_ratio times the batch's first draft
 * (length buckets limit divergence inside a launch).  A ZMW whose own estimate exceeds the budget gets a
 * batch of its own.  order[n] receives the ZMW permutation, batch_start[n + 1] the batch offsets into it
 * (batch b is order[batch_start[b] .. batch_start[b + 1])), est_bytes[n] (may be NULL) each ZMW's
 * estimate; *n_batches the batch count.  Batches are listed largest estimate first. */
int pbccs_plan_batches(const pbccs_zmw_input* in, int n, double budget_bytes, int max_per_batch,
                       double max_len_ratio, int* order, int* batch_start, double* est_bytes, int* n_batches);

/* The same in two phases, so that inputs can be made resident in HBM ahead of time:
 * pbccs_batch_create copies the ZMWs to the device; pbccs_batch_polish runs the hot path (AddRead fills,
 * gates, ZScores, RefineConsensus, ConsensusQVs) and writes the outputs.  A batch polishes once. */
typedef struct pbccs_batch pbccs_batch;
int pbccs_batch_create(pbccs_engine* eng, const pbccs_zmw_input* in, int n, const pbccs_polish_options* opts,
                       pbccs_batch** out);
int pbccs_batch_polish(pbccs_batch* b, pbccs_zmw_output* out);
void pbccs_batch_destroy(pbccs_batch* b);

/* Polish several batches of one engine concurrently: one host thread and one HIP stream per workspace
 * slot, so that one batch's convergence tail (the last refine rounds of a few ZMWs) overlaps the other
 * batches' work.  The analogue of ccs's ZMW thread pool (src/main/ccs.cpp:222-230, WorkQueue.h).
 * outs[i] receives batch i's outputs.  A batch that runs the device out of memory (PBCCS_EOOM) while the
 * others hold their band pools is rebuilt from its inputs (the batch keeps a host copy) and rerun alone once
 * every slot's pool is unmapped, halved while it still does not fit; pbccs_batch_polish does the same for
 * a single batch.  Returns the first failure. */
int pbccs_batch_polish_many(pbccs_batch* const* batches, int n, pbccs_zmw_output* const* outs);

/* Number of workspace slots = batches that may polish at the same time (default 4).  Set it before
 * creating batches; each slot holds its own resident band pools. */
int pbccs_engine_set_concurrency(pbccs_engine* eng, int batches_in_flight);

/* Map `bytes_per_slot` of band-value pool for every workspace slot now, instead of on first use.  Pool
 * memory stays mapped for the engine's lifetime and is reused by every batch the slot polishes, so a
 * long run pays the mapping once; this moves that one-time cost out of a timed region.  The mapped
 * memory is also written once (zeroed), so call it while no batch is polishing.  Optional. */
int pbccs_engine_reserve_pool(pbccs_engine* eng, size_t bytes_per_slot);

/* Work counters of the engine since the last reset (for roofline accounting). */
typedef struct {
    long long fill_launches, score_launches, score_tasks, mutations;
    long long band_top_bytes;    /* max over batches: band value pool handed out (the bump top) */
    long long band_region_bytes; /* max over batches: the reads' current band regions (2 x capacity each) */
    long long band_used_bytes;   /* max over batches: band cells the reads' last fills stored */
    long long pool_mapped_bytes; /* device memory the workspace slots' band pools hold mapped now */
    long long oom_retries;       /* device batches rerun after running the device out of memory */
    long long create_host_ns;    /* pbccs_batch_create: the batch's own copy of its inputs and the read pool */
    long long create_upload_ns;  /* pbccs_batch_create: device reservations + the read upload */
    long long derive_ns;         /* the per-ZMW setup of Consensus.h:437-453 (transition tables, expectations,
                                    reverse-complement template), run by the polish at its first device step */
    long long fill_work[16];     /* PBCCS_FILL_WORK=1 diagnostics, per fill kind k (0: 16-lane, 1: 64-lane) at
                                    [8 k + ...]: counted cells, cells thrown away by a tall abort, count-only
                                    regrow cells, count-only overflow cells, group chunk steps, wave chunk issues,
                                    reads, counted passes */
    long long scan_reads;        /* certified fast path: reads its tall fills took */
    long long uncertain_reads;   /* ... reads re-run exactly (a fill decision or the AddRead gate within the bound) */
    long long exact_rounds;      /* ... ZMW rounds re-scored on exact bands (a score decision within the bound) */
    long long uncertain_why[4];  /* ... uncertain fills by decision: band end, begin hint, loop entry, final mismatch */
} pbccs_counters;
int pbccs_engine_counters(pbccs_engine* eng, pbccs_counters* out, int reset);

/* Per-kernel profile (enabled by pbccs_engine_set_profiling): launches, summed device time from HIP
 * events on the engine's stream, and algorithmic work counted in-kernel: `cells` DP cell-updates,
 * `bytes` algorithmic band bytes (8 B per stored/read band cell + 16 B per column),
 * `wave_s` wavefront-seconds resident on the device (each wavefront's start-to-end time, summed; over a
 * timed region it gives the family's average resident waves; the fills, k_score family, k_suffix, k_reduce). */
typedef struct {
    char name[32];
    long long launches;
    double device_ms;
    double cells;
    double bytes;
    double wave_s;
} pbccs_kernel_stat;
int pbccs_engine_set_profiling(pbccs_engine* eng, int on);
int pbccs_engine_kernel_stats(pbccs_engine* eng, pbccs_kernel_stat* out, int cap, int* n, int reset);


/* ---- Quiver family (ConsensusCore/include/ConsensusCore/Quiver/) ---------------------------------
 * ccs does not call it; the north_star names it (QuiverConfig, QvEvaluator, SseRecursor).  One scorer =
 * MultiReadMutationScorer<SparseSseQvRecursor> (Viterbi) or <SparseSseQvSumProductRecursor>
 * (Quiver/MultiReadMutationScorer.hpp:242-245).  Scores are FP32 log-likelihoods. */
typedef struct pbccs_quiver_scorer pbccs_quiver_scorer;

/* QvModelParams (Quiver/QuiverConfig.hpp:79-176); merge / merge_s per template base A, C, G, T */
typedef struct {
    float match, mismatch, mismatch_s, branch, branch_s, deletion_n, deletion_with_tag, deletion_with_tag_s, nce,
        nce_s;
    float merge[4], merge_s[4];
} pbccs_qv_model_params;

/* Recursor types of ConsensusCore's Quiver MutationScorer typedefs (Quiver/MutationScorer.hpp:93-99):
 * SseRecursor or SimpleRecursor (Quiver/SimpleRecursor.cpp: row-by-row fills, moves combined Inc, Extra,
 * Del, Merge) over SparseMatrixF or DenseMatrixF storage (AllocatedEntries = Rows * Columns). */
#define PBCCS_QV_RECURSOR_SPARSE_SSE 0
#define PBCCS_QV_RECURSOR_SPARSE_SIMPLE 1
#define PBCCS_QV_RECURSOR_DENSE_SSE 2
#define PBCCS_QV_RECURSOR_DENSE_SIMPLE 3

/* QuiverConfig (QuiverConfig.hpp:181-199) + the recursor's combiner */
typedef struct {
    pbccs_qv_model_params params;
    int moves_available;         /* Move bits: INCORPORATE 1, EXTRA 2, DELETE 4, MERGE 8 (ALL_MOVES 15) */
    float score_diff;            /* BandingOptions::ScoreDiff (the diagonal-cross argument is ignored) */
    float fast_score_threshold;  /* QuiverConfig::FastScoreThreshold */
    float add_threshold;         /* QuiverConfig::AddThreshold (1.0 = no memory gate) */
    int sum_product;             /* 0: Viterbi (SparseSseQvRecursor), 1: sum-product (logAdd) */
    int recursor;                /* PBCCS_QV_RECURSOR_*: the recursor family and matrix storage */
} pbccs_quiver_config;

/* MultiReadMutationScorer(const QuiverConfigTable&, std::string tpl)  (Quiver/MultiReadMutationScorer.cpp:123-136)
 * The table: n configs with their chemistry names ("*" = the InsertDefault fallback, QuiverConfig.cpp:67-138). */
int pbccs_quiver_scorer_create(pbccs_engine* eng, const pbccs_quiver_config* configs, const char* const* chemistries,
                               int n_configs, const char* tpl, int tpl_len, pbccs_quiver_scorer** out);
void pbccs_quiver_scorer_destroy(pbccs_quiver_scorer* s);
/* bool AddRead(const MappedQvRead&, float threshold)                                    (.cpp:246-290)
 * QvSequenceFeatures tracks of len floats each (NULL = zeros); del_tag holds the tag bases as float(char).
 * threshold NaN = the read's config AddThreshold (the one-argument overload). *active = the return value. */
int pbccs_quiver_scorer_add_read(pbccs_quiver_scorer* s, const char* seq, int len, const float* ins_qv,
                                 const float* subs_qv, const float* del_qv, const float* del_tag,
                                 const float* merge_qv, const char* chemistry, int strand, int tstart, int tend,
                                 float threshold, int* active);
/* float Score(m) / FastScore(m) (.cpp:312-353); many at once */
int pbccs_quiver_scorer_score_many(pbccs_quiver_scorer* s, const pbccs_mutation* m, int n, int fast, float* scores);
/* MutationScorer<R>::ScoreMutation (Quiver/MutationScorer.cpp:113-226) on read i's own scorer: the mutation is
 * in the read's window coordinates and the absolute score of the mutated window is returned */
int pbccs_quiver_scorer_read_score_mutation(pbccs_quiver_scorer* s, int i, const pbccs_mutation* m, float* score);
/* std::vector<float> Scores(m, unscoredValue) (.cpp:355-371); per_read holds NumReads() entries */
int pbccs_quiver_scorer_scores(pbccs_quiver_scorer* s, const pbccs_mutation* m, float unscored, float* per_read);
/* IsFavorable / FastIsFavorable (.cpp:382-409) */
int pbccs_quiver_scorer_is_favorable(pbccs_quiver_scorer* s, const pbccs_mutation* m, int fast, int* favorable);
int pbccs_quiver_scorer_apply_mutations(pbccs_quiver_scorer* s, const pbccs_mutation* m, int n);   /* (.cpp:205-239) */
int pbccs_quiver_scorer_template(pbccs_quiver_scorer* s, int strand, char* out, int cap, int* len);
int pbccs_quiver_scorer_num_reads(pbccs_quiver_scorer* s);
int pbccs_quiver_scorer_read_info(pbccs_quiver_scorer* s, int i, int* active, int* strand, int* tstart, int* tend);
int pbccs_quiver_scorer_baseline_score(pbccs_quiver_scorer* s, float* score);          /* (.cpp:467-476) */
int pbccs_quiver_scorer_baseline_scores(pbccs_quiver_scorer* s, float* out, int cap, int* n);
int pbccs_quiver_scorer_num_flipflops(pbccs_quiver_scorer* s, int* out);
/* AllocatedEntries of read i's alpha / beta (SparseMatrix-inl.hpp:275-284) */
int pbccs_quiver_scorer_allocated_entries(pbccs_quiver_scorer* s, int i, long long* alpha, long long* beta);
/* RecursorBase::Alignment(e, alpha) (Quiver/detail/RecursorBase.cpp:124-264) of read i on its template window:
 * the Viterbi traceback through the read's alpha band, as PairwiseAlignment Target() / Query() (gapped,
 * len characters each).  PBCCS_ESTATE for a sum-product scorer (the reference's ShouldNotReachHere) or a
 * read without a scorer; PBCCS_ERANGE when cap < len. */
int pbccs_quiver_scorer_alignment(pbccs_quiver_scorer* s, int i, char* target, char* query, int cap, int* len);
int pbccs_quiver_refine_consensus(pbccs_quiver_scorer* s, const pbccs_refine_options* opts, long long* n_tested,
                                  long long* n_applied, int* converged);
int pbccs_quiver_consensus_qvs(pbccs_quiver_scorer* s, int* qvs, int cap, int* n);

/* QvEvaluator (Quiver/QvEvaluator.hpp:90-317): the four move scores of one read (QvSequenceFeatures,
 * Features.hpp:69-100) against a template under QvModelParams, at n cells (i[k], j[k]), evaluated on the device
 * with the recursions' own evaluator.  Inc(i, j) (:160-167), Del(i, j) with the pinStart / pinEnd rule (:169-184),
 * Extra(i, j) (:186-193), Merge(i, j) (:195-207).  A cell outside a move's domain -- the reference's asserts:
 * Inc 0 <= i < I, 0 <= j < J; Del 0 <= i <= I, 0 <= j < J; Extra 0 <= i < I, 0 <= j <= J; Merge 0 <= i < I,
 * 0 <= j < J - 1 -- gives NaN.  Feature tracks of len floats (NULL = zeros; del_tag as float(char)); any output
 * array may be NULL. */
typedef struct {
    const char* seq;
    int len;
    const float* ins_qv;
    const float* subs_qv;
    const float* del_qv;
    const float* del_tag;
    const float* merge_qv;
} pbccs_qv_features;
int pbccs_qv_evaluator_moves(pbccs_engine* eng, const pbccs_qv_features* read, const char* tpl, int tpl_len,
                             const pbccs_qv_model_params* params, int pin_start, int pin_end, const int* i,
                             const int* j, int n, float* inc, float* del, float* extra, float* merge);

/* Batched Quiver polish: for every ZMW, what a caller of the scorer API above does with one scorer --
 * create over (configs, chemistries), AddRead each read (threshold NaN = its config's add_threshold),
 * RefineConsensus(opts), ConsensusQVs -- with every scorer's fills, mutation scores, Score /
 * FastIsFavorable reduction and BestSubset on the device in lock-step rounds (one refill launch per
 * round).  Results equal the per-scorer calls'.  consensus / qvs: caller buffers of consensus_cap; qvs
 * NULL skips ConsensusQVs.  ok = 0: RefineConsensus refused an edit (the scorer call's PBCCS_EINVAL). */
typedef struct {
    const char* seq;
    int len;
    const float* ins_qv;
    const float* subs_qv;
    const float* del_qv;
    const float* del_tag;   /* float(char) per base, as pbccs_quiver_scorer_add_read */
    const float* merge_qv;
    const char* chemistry;  /* NULL = "*" */
    int strand, tstart, tend;
    float threshold;
} pbccs_quiver_read;

typedef struct {
    const char* tpl;
    int tpl_len;
    const pbccs_quiver_read* reads;
    int n_reads;
} pbccs_quiver_zmw;

typedef struct {
    char* consensus;
    int consensus_cap;
    int consensus_len;
    int* qvs;
    long long n_tested, n_applied;
    int converged;
    int ok;
    int n_active;           /* reads AddRead kept */
} pbccs_quiver_result;

int pbccs_quiver_polish_batch(pbccs_engine* eng, const pbccs_quiver_config* configs, const char* const* chemistries,
                              int n_configs, const pbccs_quiver_zmw* zmws, int n, const pbccs_refine_options* opts,
                              pbccs_quiver_result* out);

/* ---- POA draft (pbccs src/SparsePoa.cpp, ConsensusCore/src/C++/Poa) ---------------------------------
 * The read-vs-graph DP and its traceback run on the device (k_poa_fill / k_poa_trace); the graph lives on
 * the host.  Scores use DefaultPoaConfig (match 3, mismatch -5, insert -4, delete -4). */
#define PBCCS_POA_GLOBAL 0
#define PBCCS_POA_SEMIGLOBAL 1
#define PBCCS_POA_LOCAL 2

/* One ZMW's subreads in FilterReads order (include/pacbio/ccs/Consensus.h:223-292); a NULL sequence is a
 * read FilterReads dropped (key -1, as Consensus.h:378 passes nullptr reads). */
typedef struct {
    const char* const* seqs;
    const int* lens;
    int n_reads;
} pbccs_poa_input;

typedef struct {
    char* consensus;   /* caller buffer of cap bytes (not NUL-terminated); len = consensus length */
    int cap;
    int len;
    int* keys;         /* n_reads: SparsePoa::ReadKey per read; -1 not added; -2 not reached (maxPoaCov) */
    int* rc;           /* n_reads, by key: PoaAlignmentSummary::ReverseComplementedRead */
    int* extents;      /* 4 * n_reads, by key: ExtentOnRead begin/end, ExtentOnConsensus begin/end */
    int n_keys;
} pbccs_poa_output;

/* Consensus.h's PoaConsensus (:352-390) for n ZMWs at once: SparsePoa::OrientAndAddRead per read until
 * max_coverage reads were added, then FindConsensus(min_coverage) with the per-read summaries.
 * min_coverage < 0 uses Consensus.h's rule ((cov < 5) ? 1 : (cov + 1) / 2 - 1).  A consensus longer
 * than its buffer sets that output's len and makes the call return PBCCS_ERANGE after all outputs are
 * written.  A NULL sequence is a dropped read; an empty one is never added either (key -1). */
int pbccs_poa_batch(pbccs_engine* eng, const pbccs_poa_input* in, int n, long long max_coverage, int min_coverage,
                    pbccs_poa_output* out);

/* SparsePoa (include/pacbio/ccs/SparsePoa.h:94-131), one graph per handle */
typedef struct pbccs_sparse_poa pbccs_sparse_poa;
int pbccs_sparse_poa_create(pbccs_engine* eng, pbccs_sparse_poa** out);
void pbccs_sparse_poa_destroy(pbccs_sparse_poa* p);
/* ReadKey OrientAndAddRead(seq, alnOptions, minScoreToAdd)                       (src/SparsePoa.cpp:95-138) */
int pbccs_sparse_poa_orient_and_add_read(pbccs_sparse_poa* p, const char* seq, int len, float min_score_to_add,
                                         int* key);
/* FindConsensus(minCoverage, &summaries)                                          (src/SparsePoa.cpp:140-201)
 * rc / extents as in pbccs_poa_output, one entry per key. */
int pbccs_sparse_poa_find_consensus(pbccs_sparse_poa* p, int min_coverage, char* out, int cap, int* len, int* rc,
                                    int* extents, int* n_keys);
/* ToGraphViz(flags, pc) with pc = FindConsensus(min_coverage)'s consensus; flags: COLOR_NODES 1, VERBOSE_NODES 2 */
int pbccs_sparse_poa_graphviz(pbccs_sparse_poa* p, int flags, int min_coverage, char* out, int cap, int* len);

/* PoaConsensus::FindConsensus(reads, mode, minCoverage) (ConsensusCore PoaConsensus.cpp:86-115): every read
 * added with AddRead in the given mode (no orientation choice).  dot (optional) receives
 * pc->Graph.ToGraphViz(flags, pc).  PBCCS_EINVAL for an empty read (InvalidInputError). */
int pbccs_poa_consensus(pbccs_engine* eng, const char* const* reads, const int* lens, int n, int mode,
                        int min_coverage, char* out, int cap, int* len, int flags, char* dot, int dot_cap,
                        int* dot_len);
/* ---- ccs end to end: Consensus.h's per-ZMW driver for many ZMWs -------------------------------------
 * Each chunk is one ZMW after ccs.cpp's grouping gates (src/main/ccs.cpp:402-475: PoorSNR, read score,
 * TooFewPasses).  pbccs_ccs_batch runs include/pacbio/ccs/Consensus.h:395-552 for all of them:
 * FilterReads (NO_SUBREADS when nothing is left), the POA draft on the GPU (pbccs_poa_batch, with
 * max_poa_coverage), TOO_SHORT for a draft below opts->min_length, ExtractMappedRead per POA key, and the
 * polish (pbccs_polish_batch: AddRead gates, RefineConsensus, ConsensusQVs, the accuracy gate).
 * out[z].polish.add_read_results / zscores are indexed like in[z].seqs, the caller's subread order (size
 * them by n_subreads): a read FilterReads dropped, the POA did not add, ExtractMappedRead rejected or the
 * maxPoaCov stop never reached reads -1 / NaN, as does every read of a ZMW that ended before the polish.
 * A zero-length subread takes part in FilterReads but is never added to the POA (key -1); the same rule
 * holds in pbccs_poa_batch and pbccs_sparse_poa_orient_and_add_read.  A NULL sequence with a positive
 * length or a negative length is PBCCS_EINVAL.  out[z].draft (optional, draft_cap bytes) receives the POA
 * consensus; a draft longer than its buffer sets draft_len and makes the call return PBCCS_ERANGE after
 * all outputs are written.  out[z].add_order (optional, n_subreads ints) receives the caller subread index of
 * each AddRead call in the scorer's order -- FilterReads' stable order (Consensus.h:281, 451-453), which
 * ZScores() and the ccs.bam zs tag follow -- padded with -1. */
typedef struct {
    double snr[4];
    int n_subreads;
    const char* const* seqs;
    const int* lens;
    const unsigned char* flags;   /* LocalContextFlags per subread (ADAPTER_BEFORE 1, ADAPTER_AFTER 2); NULL: full passes */
} pbccs_ccs_input;

typedef struct {
    pbccs_zmw_output polish;
    char* draft;
    int draft_cap;
    int draft_len;
    int* add_order;   /* optional: AddRead order as caller subread indices, -1 padded (n_subreads ints) */
} pbccs_ccs_output;

int pbccs_ccs_batch(pbccs_engine* eng, const pbccs_ccs_input* in, int n, long long max_poa_coverage,
                    const pbccs_polish_options* opts, pbccs_ccs_output* out);

/* POA work counters since the last reset: alignments, DP cells, fill/trace device ms (profiling on) */
typedef struct {
    long long alignments, cells, launches, trace_steps;
    double fill_ms, trace_ms, bytes;
    double prog_ms, device_ms, thread_ms, consensus_ms, total_ms;   /* host wall time of each phase */
} pbccs_poa_stats;
int pbccs_poa_stats_get(pbccs_engine* eng, pbccs_poa_stats* out, int reset);

#ifdef __cplusplus
}
#endif

#endif /* PBCCS_AMD_H */
