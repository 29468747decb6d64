// pbccs_amd/csrc/quiver_engine.hpp -- host side of the Quiver engine (ConsensusCore Quiver family).
//
// QuiverBatch keeps Quiver scorers (a template + mapped QV-feature reads each) resident in HBM and runs
// the MultiReadMutationScorer surface on them (Quiver/MultiReadMutationScorer.cpp:60-504): AddRead with
// the memory-fraction gate, Score / FastScore / Scores / (Fast)IsFavorable, ApplyMutations + refills,
// BaselineScore(s), and RefineConsensus / ConsensusQVs on top (Consensus-inl.hpp:159-295).  Fills and
// mutation scores run on the GPU (quiver_kernels.hip); the read-ordered float sums run on the host.
#pragma once

#include <hip/hip_runtime.h>

#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "arrow_model.hpp"
#include "engine.hpp"
#include "quiver_kernels.hpp"

namespace pbccs {
namespace quiver {

struct QReadFeatures {
    std::string seq;
    std::vector<float> ins, subs, del, tag, merge;   // tag: DelTag as float(char)
};

// Append-only host buffer that grows without value-initialising (the QV tracks of a 10000-scorer batch are ~4 GB:
// their first touch happens in AddReads' parallel copies, not in a zero fill).  pinned: page-locked memory
// (hipHostMalloc), so the append-only uploads of the pools run at DMA speed; a long-lived batch pins once.
template <class T>
struct HostPool {
    T* p = nullptr;
    size_t n = 0, cap = 0;
    bool pinned = false;
    HostPool() = default;
    HostPool(const HostPool&) = delete;
    HostPool& operator=(const HostPool&) = delete;
    ~HostPool() { release(); }
    size_t size() const { return n; }
    T* data() { return p; }
    const T* data() const { return p; }
    size_t grow(size_t add)   // returns the old size
    {
        const size_t at = n;
        if (n + add > cap) {
            // 25% headroom: a pinned allocation costs ~0.1 s per GB, and the next batch of a long-lived pool is
            // rarely exactly as large as the one that sized it
            const size_t nc = std::max(n + add + (n + add) / 4, cap + cap / 2);
            T* q = nullptr;
            bool qp = false;
            if (pinned && hipHostMalloc((void**)&q, nc * sizeof(T), hipHostMallocDefault) == hipSuccess) qp = true;
            else {
                (void)hipGetLastError();
                q = new T[nc];
            }
            if (n) std::memcpy(q, p, n * sizeof(T));
            release();
            p = q;
            pinnedAlloc_ = qp;
            cap = nc;
        }
        n += add;
        return at;
    }

private:
    bool pinnedAlloc_ = false;
    void release()
    {
        if (p) {
            if (pinnedAlloc_) (void)hipHostFree(p);
            else delete[] p;
        }
        p = nullptr;
        cap = 0;
    }
};

class QuiverBatch {
public:
    explicit QuiverBatch(int device);
    ~QuiverBatch();
    QuiverBatch(const QuiverBatch&) = delete;
    QuiverBatch& operator=(const QuiverBatch&) = delete;

    // Drop every config, scorer and read, keeping the device buffers and host pools at their size: a long-lived
    // batch (the engine's, for pbccs_quiver_polish_batch) reaches its steady-state allocation once.
    void Reset();
    // page-locked host read pools (a long-lived batch: the pinning cost is paid once)
    void PinHostPools() { hSeq_.pinned = hFeat_.pinned = hCodes_.pinned = true; }
    int AddConfig(const QParams& p);
    int AddZmw(const std::string& tpl, float fastScoreThreshold);
    // AddRead (Quiver/MultiReadMutationScorer.cpp:246-283): fills the read; returns whether it is active.
    bool AddRead(int z, const QReadFeatures& f, int strand, int ts, int te, int config, float threshold);

    // per (mutation, read) deltas ScoreMutation(oriented) - Score(), NaN where the read does not score it;
    // out[m * nReads + k]
    void Deltas(int z, const std::vector<int>& codes, std::vector<float>* out);
    // MutationScorer<R>::ScoreMutation on read r's own scorer, mutation in the read's window coordinates
    float ReadScoreMutation(int r, int code);
    float Score(int z, const std::vector<float>& deltas, int m, bool fast) const;   // read-ordered float sum
    bool FastIsFavorable(int z, const std::vector<float>& deltas, int m) const;
    bool ApplyMutations(int z, const std::vector<Mutation>& muts);
    bool Refine(int z, const RefineOptions& ro, long long* nTested, long long* nApplied, bool* converged);
    std::vector<int> QVs(int z);

    // ---- batched forms (pbccs_quiver_polish_batch): many scorers in lock-step rounds ------------------
    // a read of the batch path: the caller's buffers (bases and five tracks of len entries; a null track reads
    // as zeros), copied once into the engine's host pools
    struct ReadSpec {
        int z, strand, ts, te, config;
        float threshold;
        const char* seq;
        int len;
        const float* track[5];   // ins, subs, del, tag (DelTag as float(char)), merge
    };
    // AddRead for every spec, one fill launch for all; returns each read's active flag
    std::vector<char> AddReads(std::vector<ReadSpec>* specs);
    // RefineConsensus on every listed scorer: one scoring launch series, one device reduction / select and
    // one refill per round.  ok[k] = 0 where ApplyMutations refused an edit (the scorer's Refine returns false).
    void RefineMany(const std::vector<int>& zs, const RefineOptions& ro, std::vector<long long>* nTested,
                    std::vector<long long>* nApplied, std::vector<char>* converged, std::vector<char>* ok);
    std::vector<std::vector<int>> QVsMany(const std::vector<int>& zs);
    // RecursorBase::Alignment (detail/RecursorBase.cpp:124-264) of read r against its template window,
    // from the read's alpha band (Viterbi configs only): the gapped target and query strings.
    bool Alignment(int r, std::string* target, std::string* query);

    const std::string& Template(int z) const { return zmws_[z].tpl; }
    int NumReads(int z) const { return (int)zmws_[z].reads.size(); }
    int ReadIndex(int z, int k) const { return zmws_[z].reads[k]; }
    bool Active(int r) const { return reads_[r].active; }
    int Ts(int r) const { return reads_[r].ts; }
    int Te(int r) const { return reads_[r].te; }
    int Strand(int r) const { return reads_[r].strand; }
    int Flips(int r) const { return reads_[r].flips; }
    float ReadScore(int r) const { return reads_[r].score; }
    long long Allocated(int r, int which) const { return reads_[r].alloc[which]; }
    float BaselineScore(int z) const;
    // profiling: HIP events around the fill and middle-case scoring launches on their own streams, plus the fills'
    // in-kernel stored-cell counters (QBatch::stats); CollectProfile adds them to `out` and clears
    void SetProfiling(bool on);
    void CollectProfile(KernelStat out[kKernelKinds]);

private:
    struct HZmw {
        std::string tpl;
        float fastThreshold = 0.0f;
        std::vector<int> reads;
    };
    struct HRead {
        int zmw = 0, config = 0, strand = 0, ts = 0, te = 0, len = 0;
        bool active = false, hasScorer = false;
        long long seqOff = 0;
        long long colBase = 0;
        int colCap = 0;
        long long valBase = 0, valCap = 0, colBuf = 0;
        int curA = 0, curB = 0, flips = 0;
        float score = 0.0f;
        long long alloc[2] = {0, 0};
        bool grpTall = false;    // a column outgrew k_qfill_grp's 64-row ring: fill with k_qfill_coop
        bool tallRing = false;   // a column outgrew the band-height LDS ring: fill with the full-height one
    };
    // a read, unfilled, whose bases and five tracks are at seqOff / 5 * seqOff of the host pools
    int RegisterRaw(int z, long long seqOff, int len, int strand, int ts, int te, int config);
    void Upload();
    void EnsureCapacity(int r);
    QBatch View();
    void Fill(const std::vector<int>& reads);
    void RunScore(const std::vector<int>& taskRead, const std::vector<int>& taskMut, const std::vector<int>& codes,
                  bool raw, std::vector<float>* d);
    // One batched scoring round over scorers zs with their mutation lists: per scorer the favourable
    // mutations (list order, float scores) and, with sep >= 0, BestSubset's picks (pick order) from the
    // device select.
    struct Scored {
        int code;
        float score;
    };
    void ScoreDeltas(const std::vector<int>& zs, const std::vector<std::vector<int>>& codes,
                     std::vector<long long>* taskStart, std::vector<long long>* mutStart);
    void ScoreRound(const std::vector<int>& zs, const std::vector<std::vector<int>>& codes, int sep,
                    std::vector<std::vector<Scored>>* fav, std::vector<std::vector<Scored>>* picked);
    // after a scoring launch whose extension scratch overflowed: grow it to the floats the launch asked for
    // (the kernel's bump counter keeps counting past the cap) plus an eighth, so the rerun fits
    void grow_scratch(unsigned long long requested);

    template <class F>
    void Timed(KernelKind k, F&& launch, hipStream_t st);

    int device_ = 0;
    bool profiling_ = false;
    struct Pending {
        int kind;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending_;
    std::vector<hipEvent_t> eventPool_;
    KernelStat stats_[kKernelKinds];
    DevVec<unsigned long long> dStats_;
    hipStream_t stream_ = nullptr;
    // the fill's tall reads (k_qfill_coop's lists) run on a side stream beside k_qfill_grp: their long serial
    // chains overlap the grouped launch instead of following it
    hipStream_t side_ = nullptr;
    hipEvent_t evFork_ = nullptr, evJoin_ = nullptr;
    std::vector<QParams> configs_;
    std::vector<HZmw> zmws_;
    std::vector<HRead> reads_;
    HostPool<char> hSeq_;
    HostPool<float> hFeat_;
    HostPool<int> hCodes_;   // a scoring round's mutation lists back to back (staging for the upload)
    long long colTop_ = 0, valTop_ = 0;
    size_t seqUp_ = 0, featUp_ = 0;   // host read pools already on the device (append-only)
    bool dirty_ = true;
    // device
    DevVec<long long> dZFwd_, dZRev_, dRSeq_, dRColBase_, dRValBase_, dRValCap_, dRColBuf_, dRUsed_, dRAlloc_;
    DevVec<int> dZLen_, dRZmw_, dRParam_, dRStrand_, dRTs_, dRTe_, dRLen_, dRColCap_, dRCurA_, dRCurB_, dRFlips_,
        dRStatus_, dList_, dTaskRead_, dTaskMut_, dCodes_, dOverflow_, dOff_;
    DevVec<char> dTpl_, dSeq_;
    DevVec<float> dFeat_, dRScore_, dDelta_, dScratch_;
    DevVec<QParams> dParams_;
    DevVec<int2> dRange_;
    DevVec<QAlloc> dAlloc_;
    DevVec<int4> dHint_;
    DevVec<float> dVal_;
    DevVec<unsigned long long> dScratchTop_;
    DevVec<long long> dMoveOff_;
    DevVec<unsigned char> dMoves_;
    DevVec<int> dNMoves_;   // k_qalign's move count per listed read
    // batched rounds
    DevVec<long long> dWTaskStart_, dWMutBase_, dSel_, dSelCount_, dSelBase_;
    DevVec<long long> dWaveStart_, dWMutCount_, dEdge_;   // k_qscore_mid work + its edge-case task list
    DevVec<unsigned long long> dEdgeCount_;
    DevVec<long long> dPosStart_, dPosOffBase_;   // QVsMany: per-position QVs on the device (k_qqv)
    DevVec<long long> dAmbSrc_, dAmbDst_;         // QVsMany: the positions left to the host (k_qgather)
    DevVec<double> dAmbScore_;
    DevVec<int> dPosOff_, dQv_;
    DevVec<int> dWReadBase_, dWNReads_, dReadList_, dRActive_, dSelCode_, dSelRank_, dNSel_;
    DevVec<float> dWFast_;
    DevVec<double> dMScore_, dSelScore_;
    DevVec<unsigned char> dFav_, dSelTmp_;
};

}  // namespace quiver
}  // namespace pbccs
