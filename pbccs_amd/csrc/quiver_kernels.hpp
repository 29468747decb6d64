// pbccs_amd/csrc/quiver_kernels.hpp -- launch interface of the Quiver kernels (quiver_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "quiver_device.hpp"

namespace pbccs {
namespace quiver {

// Batch of Quiver scorers resident in HBM (struct of arrays; see quiver_engine.hpp for the host side).
struct QBatch {
    // per scorer (a ZMW's template + config)
    const long long* zFwd;     // forward template offset in tplPool
    const long long* zRev;     // reverse-complement template offset
    const int* zLen;
    const char* tplPool;
    const QParams* params;     // per read config (QuiverConfigTable lookup done on the host)
    // per read
    const int* rZmw;
    const int* rParam;
    const int* rStrand;
    const int* rTs;
    const int* rTe;
    const int* rLen;
    const long long* rSeq;     // offset of the bases in seqPool and of the 5 feature tracks in featPool
    const char* seqPool;
    const float* featPool;     // 5 consecutive tracks per read: ins, subs, del, tag, merge (each rLen floats)
    const long long* rColBase; // column slots: 4 arenas (alpha 0/1, beta 0/1) x colCap + alloc slots
    const int* rColCap;
    const long long* rValBase; // 4 value arenas of rValCap floats each
    const long long* rValCap;
    const long long* rColBuf;  // beta column buffer (rLen + 1 floats) in valPool
    int2* range;
    int* off;
    QAlloc* alloc;             // 2 x colCap per read (alpha, beta): AllocatedEntries bookkeeping
    int4* hint;                // colCap per read: k_qfill_coop's per-column RangeGuide rows / band record
    float* valPool;
    // fill results
    int* rCurA;                // arena (0/1) holding the final alpha / beta
    int* rCurB;
    float* rScore;             // MutationScorer::Score() = beta(0, 0)
    int* rFlips;
    int* rStatus;
    long long* rUsed;          // [2 r] alpha / [2 r + 1] beta values needed (overflow sizing)
    long long* rAlloc;         // [2 r] alpha / [2 r + 1] beta AllocatedEntries
    // profiling (nullable): per fill kind (kQStatGrp / kQStatCoop / kQStatLane) the band cells the completed fills
    // stored over all their passes, and their algorithmic bytes (4 B per cell + 12 B per column per pass: range
    // int2 + offset)
    unsigned long long* stats;
};
enum QStatKind : int { kQStatGrp = 0, kQStatCoop = 1, kQStatLane = 2 };   // stats[2 k] cells, stats[2 k + 1] bytes

__host__ __device__ inline int qcols(int J) { return J + 1; }

// Scoring work: per (mutation, read) task of one scorer.
struct QScoreWork {
    const int* taskRead;       // read index
    const int* taskMut;        // index into codes
    const int* codes;          // pos << 4 | type << 2 | base (single-base mutations)
    float* delta;              // ScoreMutation(oriented) - Score(), or NaN when the read does not score it
    float* scratch;            // extend buffers, bump-allocated
    unsigned long long* scratchTop;
    unsigned long long scratchCap;
    int* overflow;
    long long nTasks;
    int raw;                   // 1: codes are already in the read's own coordinates (MutationScorer API):
                               //    no ReadScoresMutation / orientation, delta = the absolute score
    // Batched form (nWork > 0): tasks [taskBase, taskBase + nTasks) of work items laid out as
    // [item][mutation][read]; item w owns tasks [wTaskStart[w], wTaskStart[w + 1]), its mutations are
    // codes[wMutBase[w] ...] and its reads readList[wReadBase[w] ...] (wNReads of them).  taskRead /
    // taskMut are unused; delta is indexed by the global task number; inactive reads give NaN.
    int nWork = 0;
    long long taskBase = 0;
    const long long* wTaskStart = nullptr;
    const long long* wMutBase = nullptr;
    const int* wReadBase = nullptr;
    const int* wNReads = nullptr;
    const int* readList = nullptr;
    const int* rActive = nullptr;
    // listed form (taskList != nullptr): the kernel's tasks are taskList[0 .. nTasks), global task numbers of
    // the batched layout above (the edge-case tasks k_qscore_mid handed back)
    const long long* taskList = nullptr;
};

// Batched middle-case scoring (k_qscore_mid): one wavefront per (item, read, 64-mutation chunk), the lanes
// on consecutive mutations of the item's list -- adjacent template positions of one read, so the wave walks
// a handful of neighbouring band columns and the same QV-feature rows, staged in LDS.  Item w owns waves
// [waveStart[w], waveStart[w + 1]): read-major, wNReads[w] x ceil(M / 64).  Mutations within 3 columns of a
// read's window ends (ScoreMutation's edge cases) are appended to edgeList as global task numbers for
// k_qscore's listed form; the rest write delta[wTaskStart[w] + m * nReads + read] directly.
constexpr int kQMidWaves = 4;        // waves per workgroup
constexpr int kQMidStageRows = 320;  // staged QV-feature rows per wave (a wider span reads HBM directly)
struct QMidWork {
    int nWork;
    const long long* waveStart;
    const long long* wTaskStart;
    const long long* wMutBase;
    const long long* wMutCount;   // mutations of item w
    const int* wReadBase;
    const int* wNReads;
    const int* readList;
    const int* rActive;
    const int* codes;
    float* delta;
    long long* edgeList;
    unsigned long long* edgeCount;
    long long edgeCap;
};

// MultiReadMutationScorer::Score / FastIsFavorable per mutation of a batched round (Quiver/
// MultiReadMutationScorer.cpp:312-353, 392-409): the float sum over the item's reads in read order (NaN
// deltas skipped); fav = the fast sum never fell below the item's fast threshold and ends > 0.04.
struct QReduceWork {
    int nWork;
    const long long* wMutStart;   // item w's mutations [wMutStart[w], wMutStart[w + 1])
    const long long* wTaskStart;
    const int* wNReads;
    const float* wFastThreshold;
    const float* delta;
    double* score;                // the full float sum, widened (k_best_subset casts back to float)
    unsigned char* fav;
    long long nMut;
};

// ConsensusQVs (Consensus-inl.hpp:274-295) of a batched QV round, one lane per template position: the sum of
// exp(score) over the position's mutations with a negative (float) score, then -10 log10(1 - 1 / (1 + sum)).
struct QQvWork {
    int nWork;
    const long long* posStart;     // item w's positions [posStart[w], posStart[w + 1]) (global position index)
    const long long* wMutStart;    // item w's mutations start in score[]
    const long long* posOffBase;   // item w's position offsets at posOff + posOffBase[w] (L + 1 of them)
    const int* posOff;             // mutation offset of each position within its item
    const double* score;           // k_qreduce's per-mutation sums
    int* qv;                       // per global position (-1: left to the host, see k_qqv)
    int hostAll = 0;               // test hook (PBCCS_QQV_HOST=1): every position left to the host
};
void launch_qqv(const QQvWork& W, long long nPos, hipStream_t s);
// QVsMany's host path: out[dst[a] .. dst[a + 1]) = score[src[a] ..], one thread per position a (n positions)
void launch_qgather(const double* score, const long long* src, const long long* dst, int n, double* out, hipStream_t s);

void launch_qfill(const QBatch& B, const int* reads, int n, hipStream_t s);
// FillAlphaBeta with one wavefront per read (SparseSse recursors; reads of I + 1 <= kQCoopRows rows and windows
// of J + 1 <= kQCoopCols columns); maxRows / maxCols = the largest I + 1 / J + 1 of the listed reads
constexpr int kQCoopRows = 4096;
constexpr int kQRingRows = 128;   // k_qfill_coop band-height ring rows (a power of two; taller columns: kQTall); 128 / 256 / 512 / 1024 measured 1760 / 1583-1626 / 1241 / 1178 ZMWs/s (profiles/r3t_quiver_ab.txt, r3v_quiver_ab.txt)
constexpr int kQCoopCols = 8192;
void launch_qfill_coop(const QBatch& B, const int* reads, int n, int maxRows, int maxCols, hipStream_t s);
// The same with four reads per wavefront (a 16-lane DPP row each, 64-row band ring): the default first try for
// SparseSse reads; a read with a taller column comes back kQTall and is refilled by k_qfill_coop.
void launch_qfill_grp(const QBatch& B, const int* reads, int n, hipStream_t s);
void launch_qscore(const QBatch& B, const QScoreWork& W, hipStream_t s);
void launch_qscore_mid(const QBatch& B, const QMidWork& W, long long nWaves, hipStream_t s);
void launch_qreduce(const QReduceWork& W, hipStream_t s);
// QvEvaluator (Quiver/QvEvaluator.hpp:90-317) on one read's features against `tpl`: Inc, Del, Extra and Merge at the
// n cells (ci[k], cj[k]) into out[0 .. 4n) (move-major; NaN outside a move's domain).  r, p, tpl, ci, cj, out are
// device pointers.
void launch_qv_moves(const QRead& r, const QParams* p, const char* tpl, int tplLen, int pinStart, int pinEnd,
                     const int* ci, const int* cj, int n, float* out, hipStream_t s);
// RecursorBase::Alignment per listed read: moves (from the end) at moveOff[t], nMoves[t] of them
void launch_qalign(const QBatch& B, const int* reads, int n, const long long* moveOff, unsigned char* moves,
                   int* nMoves, hipStream_t s);

}  // namespace quiver
}  // namespace pbccs
