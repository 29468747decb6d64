// pbccs_amd/csrc/arrow_kernels.hpp -- host-visible launch interface of arrow_kernels.hip.
#pragma once

#include <hip/hip_runtime.h>

#include "arrow_device.hpp"

namespace pbccs {

// A scoring round: a list of work items, each = one ZMW with a contiguous list of mutation codes.
struct ScoreWork {
    int nWork = 0;
    const int* zmw = nullptr;              // [nWork]
    const int* nMut = nullptr;             // [nWork]
    const long long* mutBase = nullptr;    // [nWork] offset of the item's codes / scores
    const long long* deltaBase = nullptr;  // [nWork] offset of the item's (read x mutation) deltas
    const long long* waveStart = nullptr;  // [nWork + 1] cumulative waves (reads x ceil(M / 64))
    const long long* mutStart = nullptr;   // [nWork + 1] cumulative mutations
    const long long* posStart = nullptr;   // [nWork + 1] cumulative template positions (QV rounds)
    const int* codes = nullptr;
    double* delta = nullptr;
    // tasks near a read's window ends, appended by k_score for k_score_edge
    int* edgeList = nullptr;   // [edgeCap][3] = (work item, read, mutation)
    int* edgeCount = nullptr;
    int edgeCap = 0;
    // Phased scoring (ArrowBatch::RunRound): a phase scores reads [readLo, readHi) of every item, and after
    // the first phase only the mutations whose ordered fast-score prefix has not broken yet (sel: their
    // global indices, ascending; item k owns sel[selBase[k] .. selBase[k] + nSel[k])).  waveStart then
    // counts (reads in the phase) x ceil(nSel / 64) waves per item.
    int readLo = 0;
    int readHi = 1 << 30;
    const long long* sel = nullptr;
    const long long* selBase = nullptr;
    const int* nSel = nullptr;
    // Certified fast path: per item a bound on how far any of its summed mutation scores may lie from
    // the reference's (3x the reads' LL bounds: the mutated read, its baseline and the bands' prefix / suffix sums);
    // k_reduce sets amb[k] when the fast-score break or the favourable test of a mutation lies within it.
    // nullptr: every read of the round was filled exactly.
    const double* dev = nullptr;
    int* amb = nullptr;
};

// Scoring of reads with checkpointed bands (k_score_ckpt): a persistent grid of nSlots waves, each with a
// slot of slotCap doubles for the columns it replays, pulls the round's tasks -- the 64-mutation chunks of
// the (work item, read) pairs whose read is checkpointed -- from `counter`.  `need` receives the largest
// slot a skipped block needed (0 when every block fit); the host then grows the slots and reruns.
constexpr int kCkptMaxK = 32;                             // largest checkpoint interval the replay supports
constexpr unsigned long long kCkptBadGeometry = 1ull << 62;   // CkptWork::need: a block outgrew the replay tables
struct CkptWork {
    const int2* pairs = nullptr;           // [nPairs] (work item, read index within the ZMW)
    const long long* taskStart = nullptr;  // [nPairs + 1] cumulative chunks
    int nPairs = 0;
    long long nTasks = 0;
    unsigned long long* counter = nullptr;
    double* slots = nullptr;
    long long slotCap = 0;
    int nSlots = 0;
    unsigned long long* need = nullptr;
};

// Bump-allocated scratch for the rare whole-window refill case (tiny windows).
struct ScoreScratch {
    double* pool = nullptr;
    unsigned long long* top = nullptr;
    unsigned long long cap = 0;
    int* overflow = nullptr;
};

// Lane-interleaved fill scratch: group g (64 reads) x matrix (alpha, beta) x slot/column x lane.
struct FillScratch {
    double* val = nullptr;    // [2G][capSlots][64]
    int2* range = nullptr;    // [2G][capCols][64]
    int* off = nullptr;
    double* ls = nullptr;
    double* pre = nullptr;    // [G][capCols + 1][64] alpha log-scale prefix
    int* usedA = nullptr;     // per read: values used by the final alpha / beta
    int* usedB = nullptr;
    long long capSlots = 0;
    int capCols = 0;
    long long* trace = nullptr;   // optional [n][8] per-lane timing (PBCCS_FILL_TRACE diagnostics)
};

// Cooperative fill (fill_coop.hip): bands written straight into each read's compact region.
struct CoopFill {
    int* usedA = nullptr;    // per read: values used by the final alpha / beta (or needed, on overflow)
    int* usedB = nullptr;
    int* maxH = nullptr;     // per read: the tallest column of the fill's passes (routing of its next refill)
    int hcap = 0;            // LDS rows per column buffer
    int readWords = 0;       // nibble-packed read words per group (>= ceil(I / 8) of every read)
    int tplWords = 0;        // nibble-packed template words per group (>= ceil((J + 1) / 8))
    size_t groupBytes = 0;   // coop_group_bytes(hcap, readWords, tplWords)
    bool prio = false;       // waves at raised issue priority (the tall paths: each round's critical path)
    bool chainExit = true;   // G = 64 serial chain leaves a chunk early once its stop row is final
    bool scan = false;       // G = 64: the reassociated (scan) chain, certified against a bound
    double devScale = 1.0;   // test hook (PBCCS_SCAN_DEV_SCALE): the certified path's bounds inflated, so its exact
                             // re-runs and re-scored rounds are exercised
    int rows = 1;            // band rows per lane (a chunk is G x rows rows)
    // relative width of the band around the row threshold pm / sdn in which the fill divides (thr_ge, 2^-50 x 3
    // roundings); tests widen it (PBCCS_FILL_THR_MARGIN) so that the division path runs on most rows
    double thrMargin = 0x1p-50;
    int regrowSlackDiv = 16;   // regrow_bands: a re-homed region holds need + need / regrowSlackDiv + 64
    // In-kernel band growth: a read whose alpha/beta region overflows takes a larger region pair from
    // the pool's free top (valBump, in values; mapped up to valLimit), copies what it must keep, and
    // carries on -- no count-only pass and no relaunch.  The new region is written back to the
    // descriptor arrays (aliases of DevBatch::rValA/rValB/rValCap).  Only when the mapped headroom runs
    // out does the read fall back to count-only mode (kFillOverflow).
    unsigned long long* valBump = nullptr;
    long long valLimit = 0;
    long long* rValA = nullptr;
    long long* rValB = nullptr;
    long long* rValCap = nullptr;
    // Hybrid 64-lane path: column rows past the hcap LDS rows live in 2 * gRows doubles per launch slot of
    // colScratch, so no column is ever too tall.  nullptr: the column buffers are LDS only.
    double* colScratch = nullptr;
    int gRows = 0;
    // diagnostics (PBCCS_FILL_PATHS=2): per listed read [6]: wall-clock start / end (100 MHz), shader cycles,
    // cells, passes, columns
    long long* trace = nullptr;
    // diagnostics (PBCCS_FILL_WORK=1): where the fill's computed cells go, per kind (k = 0: the 16-lane fill,
    // 1: the 64-lane fills) at work[kFillWorkSlots * k + ...] (kFillWork*)
    unsigned long long* work = nullptr;
};
// work[] slots per fill kind: cells of the passes that count (the bench's GCUPS); cells computed and thrown away
// because the read aborted as too tall (its passes restart on the 64-lane path); cells of count-only passes that
// re-run after a regrow; cells of fills that ended in count-only overflow (re-run by the host); the groups' chunk
// steps (a G x R-row chunk of a column's chain); the wavefront's chunk issues (the chunk body executed for some
// subset of the wave's groups: 4 x issues - steps are group-steps spent idle or serialised in lock-step); reads;
// counted passes
enum FillWork : int {
    kFillWorkCells = 0, kFillWorkTallAbort, kFillWorkRegrow, kFillWorkOverflow, kFillWorkSteps, kFillWorkIssues,
    kFillWorkReads, kFillWorkPasses, kFillWorkSlots
};
size_t coop_group_bytes(int hcap, int readWords, int tplWords);
constexpr int kNarrowGroupLanes = 16;   // typical bands: lanes per read (four reads per wavefront)
constexpr int kTallRowsPerLane = 2;   // tall fills: band rows per lane (a 128-row chunk)
void launch_fill_coop(int G, const DevBatch& B, const CoopFill& F, const int* reads, int n, hipStream_t s);

void launch_fill(const DevBatch& B, const FillScratch& F, const int* reads, int n, hipStream_t s);
void launch_compact(const DevBatch& B, const FillScratch& F, const int* reads, int n, hipStream_t s);
void launch_suffix(const DevBatch& B, const int* reads, int n, hipStream_t s, bool withPrefix = false);
void launch_enumerate(const DevBatch& B, const int* zmws, int n, const long long* mutBase, const long long* posBase,
                      int* codes, int* posOff, hipStream_t s);
void launch_score(const DevBatch& B, const ScoreWork& W, long long nWaves, const ScoreScratch& scratch, hipStream_t s,
                  const CkptWork* ck = nullptr);
// Phased scoring helpers: alive[g] = the ordered fast-score sum of mutation g over reads [0, readHi) never
// fell below fastThr (k_reduce's break has not happened yet); per-item ranges of the selected list.
void launch_alive(const DevBatch& B, const ScoreWork& W, long long nMut, double fastThr, int readHi,
                  unsigned char* alive, hipStream_t s);
void launch_sel_ranges(const ScoreWork& W, const long long* sel, const long long* count, long long* selBase,
                       int* nSel, hipStream_t s);
void launch_reduce(const DevBatch& B, const ScoreWork& W, long long nMut, double fastThr, double* score,
                   unsigned char* fav, hipStream_t s);
// BestSubset (Consensus-inl.hpp:98-118) on the compacted favourable list: one wavefront per work item over
// [selBase[k], selBase[k] + nSel[k]); rank = pick order (1-based) or 0.  The first ldsCap entries
// (-1 = the kernel's maximum) of a list are staged in LDS, the rest read from HBM.
void launch_best_subset(int nWork, const long long* selBase, const int* nSel, const int* code, const double* score,
                        int sep, int ldsCap, int* rank, hipStream_t s);
void launch_qv(const DevBatch& B, const ScoreWork& W, long long nPos, const long long* posBase, const int* posOff,
               const double* score, const long long* qvBase, int* qv, hipStream_t s);

}  // namespace pbccs
