// pbccs_amd/csrc/arrow_device.hpp
//
// Device-side core of the MI355X Arrow polishing engine: the data layout of a ZMW batch in HBM and
// the per-lane recursions (band fill, extend, link) that the kernels in arrow_kernels.hip run.
//
// Execution model: one lane owns one alignment task -- a (read, template-window)
// fill, or a (mutation, read) score.  Within a task the work is column-serial exactly as in
// ConsensusCore's Arrow::SimpleRecursor, because per-column rescaling makes every cell of column j
// depend on the *scaled* column j-1; parallelism comes from the tens of
// thousands of tasks in a batch.  All arithmetic is IEEE FP64 in the reference's operation order and
// the library is built with -ffp-contract=off, so band shapes and cell values are bit-identical to the
// reference; only libm `log` (device OCML vs glibc) may differ in the last ulp.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pbccs {

// ---------------------------------------------------------------------------------------------
// Constants (reference citations in DESIGN.md and at each use)
// ---------------------------------------------------------------------------------------------
constexpr int kCtxZero = 8;           // index of the all-zero TransitionParameters slot
constexpr int kCtxStride = 5;         // {Match, Stick, Branch, Deletion, Stick/3.0}
constexpr int kNoMutation = -100;     // TemplateParameterPair::NO_MUTATION_SET_FLAG (.hpp:33)
constexpr int kMaxExtCols = 4;        // max extension columns any single-base mutation needs
constexpr int kMaxFlipFlops = 5;      // SimpleRecursor.cpp:52
constexpr double kAlphaBetaTol = 0.001;   // SimpleRecursor.cpp:53
constexpr double kRebandFrac = 0.04;      // SimpleRecursor.cpp:54

enum MutType : int { kIns = 0, kDel = 1, kSub = 2 };   // Mutation.hpp:50-53
enum Strand : int { kFwd = 0, kRev = 1 };

// kFillTall: a column did not fit the cooperative fill's LDS buffer (re-run on a wider path)
// kFillUncertain: the certified fast path (reassociated chain) could not prove one of the fill's
// decisions equal to the reference's (a band end, a begin hint or a flip-flop test within the deviation bound of
// its threshold): the host re-runs the read on the exact path
enum FillStatus : int { kFillOk = 0, kFillMismatch = 1, kFillOverflow = 2, kFillBadInput = 3, kFillTall = 4,
                        kFillUncertain = 5 };
constexpr double kUnitRoundoff = 0x1p-53;   // u: |fl(x) - x| <= u |x| for a normal result

// Mutation code: pos << 4 | type << 2 | base(0..3).  Single-base mutations only (what ccs enumerates).
__host__ __device__ inline int mut_code(int pos, int type, int base) { return (pos << 4) | (type << 2) | base; }
__host__ __device__ inline int mut_pos(int c) { return c >> 4; }
__host__ __device__ inline int mut_type(int c) { return (c >> 2) & 3; }
__host__ __device__ inline int mut_base(int c) { return c & 3; }

__host__ __device__ inline char base_char(int b) { return "ACGT"[b & 3]; }
__host__ __device__ inline int base_index(char b)
{
    return b == 'A' ? 0 : b == 'C' ? 1 : b == 'G' ? 2 : b == 'T' ? 3 : -1;
}
__host__ __device__ inline int complement_index(int b) { return 3 - b; }

// ContextParameters::GetParametersForContext (ContextParameters.cpp:35-47): "XX" for a homopolymer
// pair, "N" + second base otherwise.  Slots 0..3 = AA CC GG TT, 4..7 = NA NC NG NT.
__host__ __device__ inline int context_index(char b1, char b2)
{
    const int i2 = base_index(b2);
    return (b1 == b2) ? i2 : 4 + i2;
}

// ---------------------------------------------------------------------------------------------
// Batch layout in HBM (struct of arrays).  Every array is indexed by zmw id z, read id r, or a
// column slot (read's column base + j).  Band values live in one FP64 pool; each read owns two
// regions (alpha, beta) addressed by offsets, with a capacity that the host grows on overflow.
// ---------------------------------------------------------------------------------------------
struct DevBatch {
    // per ZMW
    const int* zFwdOff;       // offset of the forward template in tplPool
    const int* zRevOff;       // offset of the reverse-complement template in tplPool
    const int* zLen;          // template length L
    const double* zCtx;       // [Z][9][kCtxStride] transition parameters (slot 8 = zeros)
    const int* zReadBegin;    // reads of zmw z are [zReadBegin, zReadBegin + zNReads)
    const int* zNReads;
    const char* tplPool;
    // per read
    const long long* rSeqOff; // read bases in seqPool
    const int* rLen;          // I
    const int* rStrand;
    const int* rTs;           // mapped window [ts, te) in forward coordinates
    const int* rTe;
    const int* rActive;
    const int* rZmw;
    const long long* rColBase;   // column slot base
    const long long* rValA;      // alpha value region offset in valPool
    const long long* rValB;      // beta value region offset in valPool
    const long long* rValCap;    // capacity (values) of each region
    const int* rCkpt;            // checkpoint interval K of the read's bands (0: every column's values stored)
    const char* seqPool;
    // column slots
    int2* aRange;
    int* aOff;
    double* aLs;
    double* aPre;             // exclusive prefix of alpha log-scales (GetLogProdScales(0, k))
    int2* bRange;
    int* bOff;
    double* bLs;
    double* bSuf;             // GetLogProdScales(k, J+1) accumulated left to right (exact order)
    double* valPool;
    // per read results of the last fill
    double* rBaseline;        // MutationScorer::Score() = log(beta(0,0)) + sum(beta log-scales)
    // per read: a bound on |LL - LL_reference| of the last fill's alpha and beta bands (their log-likelihoods and log-
    // scale sums): 0 for the exact paths, > 0 for a read the certified fast path filled
    double* rDev;
    int* rFlips;
    int* rStatus;
    // model constants
    double prNot;             // ModelParams::PrNotMiscall
    double prThird;           // ModelParams::PrThirdOfMiscall
    double sdn;               // exp(BandingOptions::ScoreDiff)
    // optional algorithmic-work counters (profiling): [2k] cells, [2k+1] bytes for kernel kind k
    unsigned long long* stats;
};

enum StatKind : int { kStatFill = 0, kStatSuffix = 1, kStatScore = 2, kStatFillTall = 3 };   // stats[] has 16 slots
// stats[10..14]: resident wave time per kernel family, in s_memrealtime ticks (100 MHz): each wavefront adds the
// ticks from its first instruction to its end (wave_t0 / wave_ticks).  Over the timed region it gives the waves of
// each family resident on the device on average -- what the concurrent batches hold of its wave slots and VGPR file.
enum WaveSlot : int { kWaveFill = 10, kWaveFillTall = 11, kWaveScore = 12, kWaveSuffix = 13, kWaveReduce = 14 };
#ifndef PBCCS_WAVE_STAMPS   // 1: the occupancy build (tools/gpu_steps.sh occ); off by default: the stamps cost 5% (A/B)
#define PBCCS_WAVE_STAMPS 0
#endif
__device__ __forceinline__ long long wave_t0(const unsigned long long* stats)
{
    if (!PBCCS_WAVE_STAMPS) return 0;
    return stats ? (long long)__builtin_amdgcn_s_memrealtime() : 0;
}
// at a point every lane of the wavefront that is still running reaches once (the end of the kernel)
__device__ __forceinline__ void wave_ticks(unsigned long long* stats, int slot, long long t0)
{
    if (!PBCCS_WAVE_STAMPS || !stats) return;
    const long long t1 = (long long)__builtin_amdgcn_s_memrealtime();
    const unsigned long long act = __ballot(1);
    if ((int)(threadIdx.x & 63) == __ffsll((long long)act) - 1) atomicAdd(&stats[slot], (unsigned long long)(t1 - t0));
}

struct TaskStat {
    unsigned long long cells = 0;
    unsigned long long bytes = 0;
};

// ---------------------------------------------------------------------------------------------
// Checkpointed bands.  A read with checkpoint interval K > 0 keeps every column's range,
// offset and log-scale, but the values of only these columns; the scorer replays the others from the
// nearest kept column (a column depends only on the scaled column before it and on its own range, so the
// replay is bit-identical).  Alpha keeps j % K == 0 and the last kCkptTail + 1 columns (ExtendAlpha to
// the end reads them), beta j % K == 0, the first kCkptTail + 1 columns (ExtendBeta) and column J.
// ---------------------------------------------------------------------------------------------
constexpr int kCkptTail = 6;
__host__ __device__ inline bool ckpt_col_a(int j, int J, int K) { return j % K == 0 || j >= J - kCkptTail; }
__host__ __device__ inline bool ckpt_col_b(int j, int J, int K) { return j % K == 0 || j <= kCkptTail || j == J; }

// ---------------------------------------------------------------------------------------------
// Template views: WrappedTemplateParameterPair over a TemplateParameterPair with an optional
// virtual mutation (TemplateParameterPair.hpp:88-147, TemplateParameterPair.cpp:61-140).
// Transition parameters are never stored per position: ctx(T[g], T[g+1]) is recomputed from the
// bases, which is exactly what the reference keeps in trans_probs after any sequence of real edits.
// ---------------------------------------------------------------------------------------------
struct VirtualMut {
    int mpos = kNoMutation;
    int moff = 0;
    int mb0 = '0', mb1 = '0';   // base chars (int: byte-sized members of a by-value struct were kept in scratch)
    int mc0 = kCtxZero, mc1 = kCtxZero;
};

struct TplView {
    const char* T;   // strand template bases
    int L;           // strand template length
    int start;       // window start on this strand
    int len;         // window length (unmutated)
    VirtualMut vm;

    __device__ __forceinline__ int Length() const
    {
        return (vm.mpos >= start && vm.mpos < start + len) ? len - vm.moff : len;
    }
    __device__ __forceinline__ void Plain(int g, char& b, int& c) const
    {
        b = T[g];
        c = (g + 1 < L) ? context_index(T[g], T[g + 1]) : kCtxZero;
    }
    __device__ __forceinline__ void At(int idx, char& b, int& c) const
    {
        const int g = idx + start;
        if (g < vm.mpos - 1) Plain(g, b, c);
        else if (g > vm.mpos) Plain(g + vm.moff, b, c);   // also the no-mutation case (mpos = -100)
        else if (g == vm.mpos) { b = vm.mb1; c = vm.mc1; }
        else { b = vm.mb0; c = vm.mc0; }
    }
    __device__ __forceinline__ char Base(int idx) const
    {
        char b; int c;
        At(idx, b, c);
        return b;
    }
    __device__ __forceinline__ int Ctx(int idx) const
    {
        char b; int c;
        At(idx, b, c);
        return c;
    }
};

// The mapped window [ts, te) of read r on its strand's template (no virtual mutation).
__device__ __forceinline__ TplView window_view(const DevBatch& B, int r)
{
    const int z = B.rZmw[r];
    const int L = B.zLen[z];
    const int ts = B.rTs[r], te = B.rTe[r];
    TplView v;
    if (B.rStrand[r] == kFwd) {
        v.T = B.tplPool + B.zFwdOff[z];
        v.start = ts;
    } else {
        v.T = B.tplPool + B.zRevOff[z];
        v.start = L - te;
    }
    v.L = L;
    v.len = te - ts;
    return v;
}

// TemplateParameterPair::ApplyVirtualMutation (TemplateParameterPair.cpp:70-140) on strand template T.
__device__ inline VirtualMut make_virtual(const char* T, int L, int type, int s, char nb)
{
    VirtualMut v;
    v.mpos = s;
    if (type == kSub) {
        v.moff = 0;
        v.mb1 = nb;
        if (s > 0) { v.mb0 = T[s - 1]; v.mc0 = context_index(T[s - 1], nb); }
        if (s + 1 < L) v.mc1 = context_index(nb, T[s + 1]);
    } else if (type == kDel) {
        v.moff = 1;
        const int last = L - 1;
        if (s > 0 && s < last) {
            v.mb0 = T[s - 1];
            v.mb1 = T[s + 1];
            v.mc0 = context_index(T[s - 1], T[s + 1]);
            v.mc1 = (s + 2 < L) ? context_index(T[s + 1], T[s + 2]) : kCtxZero;   // trans_probs[s + 1]
        } else if (s == 0) {
            v.mb1 = T[1];
            v.mc1 = (2 < L) ? context_index(T[1], T[2]) : kCtxZero;
        } else if (s == last) {
            v.mb0 = T[s - 1];
        }
    } else {
        v.moff = -1;
        v.mb1 = nb;
        if (s > 0) { v.mb0 = T[s - 1]; v.mc0 = context_index(T[s - 1], nb); }
        if (s < L) v.mc1 = context_index(nb, T[s]);
    }
    return v;
}

// ---------------------------------------------------------------------------------------------
// Band matrix storage (ScaledSparseMatrixD semantics: cells outside a column's used row range read as
// 0.0).  Alpha columns are stored top-down, beta columns bottom-up, each fill appending its cells in
// the order it computes them.  S is the element stride: 1 for a read's compact band (what scoring
// reads), 64 for the lane-interleaved fill scratch (a fill wave's 64 reads share one region, so each
// wave-wide access stays within a few pages instead of touching 64 separate 2 MB regions).
// ---------------------------------------------------------------------------------------------
template <int S>
struct StridedBand {
    int2* range;
    int* off;
    double* ls;
    double* val;
    long long cap;   // capacity in values
    __device__ __forceinline__ int2& R(int j) const { return range[(long long)j * S]; }
    __device__ __forceinline__ int& O(int j) const { return off[(long long)j * S]; }
    __device__ __forceinline__ double& L(int j) const { return ls[(long long)j * S]; }
    __device__ __forceinline__ double& V(long long k) const { return val[k * S]; }
};
using Band = StridedBand<1>;
using LaneBand = StridedBand<64>;

template <int S>
__device__ __forceinline__ double alpha_at(const StridedBand<S>& m, int i, int j)
{
    const int2 r = m.R(j);
    return (i >= r.x && i < r.y) ? m.V(m.O(j) + (i - r.x)) : 0.0;
}

template <int S>
__device__ __forceinline__ double beta_at(const StridedBand<S>& m, int i, int j)
{
    const int2 r = m.R(j);
    return (i >= r.x && i < r.y) ? m.V(m.O(j) + (r.y - 1 - i)) : 0.0;
}

struct Params {
    const double* ctx;   // 9 x kCtxStride
    double prNot, prThird, sdn;
    __device__ __forceinline__ const double* P(int c) const { return ctx + c * kCtxStride; }
};
// field offsets inside a context slot
constexpr int kM = 0, kS = 1, kB = 2, kD = 3, kS3 = 4;

// ---------------------------------------------------------------------------------------------
// FillAlpha (SimpleRecursor.cpp:60-181).  `guide` (nullable) is the other matrix's used ranges;
// when `selfValid` the matrix's previous used ranges also widen the band (RangeGuide :728-757;
// RowRange :693-726 never trims scaled columns, so only ranges are consulted).  Ranges are updated
// in place column by column, after their old value has been read.  Returns the used-entry count,
// or -1 on value-capacity overflow.
//
// Latency structure: the in-column insertion chain a_i = (M_i + a_{i-1} k_i) + D_i is carried in
// registers; the previous column and the read bases are prefetched kFillChunk rows at a time, so
// a row costs its dependent FP64 chain, not an HBM/L2 round trip.
// ---------------------------------------------------------------------------------------------
constexpr int kFillChunk = 8;

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

template <class View, int S>
__device__ long long fill_alpha(const View& tv, const char* __restrict__ rd, int I, const StridedBand<S>& a,
                                const StridedBand<S>* guide, bool selfValid, const Params& P)
{
    const int J = tv.Length();
    if (a.cap < 1) return -1;
    a.V(0) = 1.0;
    a.R(0) = make_int2(0, 1);
    a.O(0) = 0;
    a.L(0) = 0.0;
    long long used = 1;
    int hb = 1, he = 1;
    int prevCtx = kCtxZero;
    char curBase;
    int curCtx;
    tv.At(0, curBase, curCtx);
    for (int j = 1; j < J; ++j) {
        if (guide) {
            const int2 g = guide->R(j);
            if (g.x < g.y) { hb = min(g.x, hb); he = max(g.y, he); }
        }
        if (selfValid) {
            const int2 o = a.R(j);
            if (o.x < o.y) { hb = min(o.x, hb); he = max(o.y, he); }
        }
        const int reqEnd = min(I, he);
        char nextBase;
        int nextCtx;
        tv.At(j, nextBase, nextCtx);
        const double* cp = P.P(curCtx);
        const double* pp = P.P(prevCtx);
        const double pMatch = pp[kM], pDel = pp[kD];
        const double cBranch = cp[kB], cStick3 = cp[kS3];
        const int2 pr = a.R(j - 1);
        const bool prNonEmpty = pr.x < pr.y;
        const long long pbase = (long long)a.O(j - 1) - pr.x;   // prev column: V(pbase + i), i in [pr.x, pr.y)
        const long long cbase = used - hb;                        // this column:  V(cbase + i), i in [hb, end)
        const int b = hb;
        const long long room = a.cap - used;
        double thr = 0.0, mx = 0.0, score = 0.0, up = 0.0;
        double diag = (prNonEmpty && b - 1 >= pr.x && b - 1 < pr.y) ? a.V(pbase + b - 1) : 0.0;
        int i = b;
        bool go = i < I;   // (score >= thr) holds for the first row
        while (go) {
            double lf[kFillChunk];
            char rbs[kFillChunk];
#pragma unroll
            for (int q = 0; q < kFillChunk; ++q) {
                const int row = i + q;
                const bool in = prNonEmpty && row >= pr.x && row < pr.y;
                const double x = a.V(prNonEmpty ? pbase + clampi(row, pr.x, pr.y - 1) : (long long)a.O(j - 1));
                lf[q] = in ? x : 0.0;
                rbs[q] = rd[clampi(row - 1, 0, I - 1)];
            }
#pragma unroll
            for (int q = 0; q < kFillChunk; ++q) {
                if (i - b >= room) return -1;
                const char rb = rbs[q];
                const double left = lf[q];
                const double mpe = diag * (rb == curBase ? P.prNot : P.prThird);
                double move = 0.0;
                if (i == 1 && j == 1) move = mpe;
                else if (i != 1 && j != 1) move = mpe * pMatch;
                score = 0.0 + move;
                if (i > 1) score = score + up * (rb == nextBase ? cBranch : cStick3);
                if (j > 1) score = score + left * pDel;
                a.V(cbase + i) = score;
                if (score > mx) { mx = score; thr = mx / P.sdn; }
                up = score;
                diag = left;
                ++i;
                go = i < I && (score >= thr || i < reqEnd);
                if (!go) break;
            }
        }
        const int e = i;
        // ScaledMatrix::FinishEditingColumn (ScaledMatrix-inl.hpp:35-60); mx == max(0, cells).  The next
        // column's begin hint is the first row whose *scaled* value reaches the unscaled threshold (:166).
        int nhb = e;
        if (mx != 0.0 && mx != 1.0) {
#pragma unroll 4
            for (int k = b; k < e; ++k) {
                const double v = a.V(cbase + k) / mx;
                a.V(cbase + k) = v;
                if (nhb == e && !(v < thr)) nhb = k;
            }
            a.L(j) = log(mx);
        } else {
            for (int k = b; k < e; ++k)
                if (!(a.V(cbase + k) < thr)) { nhb = k; break; }
            a.L(j) = 0.0;
        }
        a.R(j) = make_int2(b, e);
        a.O(j) = (int)used;
        used += e - b;
        prevCtx = curCtx;
        curBase = nextBase;
        curCtx = nextCtx;
        he = e;
        hb = nhb;
    }
    // last column: pinned final match (:169-179)
    if (used + 1 > a.cap) return -1;
    const char lastBase = tv.Base(J - 1);
    const double em = (rd[I - 1] == lastBase) ? P.prNot : P.prThird;
    const double lik = alpha_at(a, I - 1, J - 1) * em;
    const double c = (0.0 < lik) ? lik : 0.0;
    double v = lik;
    double ls = 0.0;
    if (c != 0.0 && c != 1.0) { v = lik / c; ls = log(c); }
    a.V(used) = v;
    a.R(J) = make_int2(I, I + 1);
    a.O(J) = (int)used;
    a.L(J) = ls;
    used += 1;
    return used;
}

// FillBeta (SimpleRecursor.cpp:183-296).  Same conventions as fill_alpha; values stored bottom-up.
template <class View, int S>
__device__ long long fill_beta(const View& tv, const char* __restrict__ rd, int I, const StridedBand<S>& bm,
                               const StridedBand<S>* guide, bool selfValid, const Params& P)
{
    const int J = tv.Length();
    if (bm.cap < 1) return -1;
    bm.V(0) = 1.0;
    bm.R(J) = make_int2(I, I + 1);
    bm.O(J) = 0;
    bm.L(J) = 0.0;
    long long used = 1;
    int hb = I, he = I;
    char nextBase;
    int nextCtx;
    tv.At(J - 1, nextBase, nextCtx);
    for (int j = J - 1; j > 0; --j) {
        char curBase;
        int curCtx;
        tv.At(j - 1, curBase, curCtx);
        if (guide) {
            const int2 g = guide->R(j);
            if (g.x < g.y) { hb = min(g.x, hb); he = max(g.y, he); }
        }
        if (selfValid) {
            const int2 o = bm.R(j);
            if (o.x < o.y) { hb = min(o.x, hb); he = max(o.y, he); }
        }
        const int reqBegin = max(0, hb);
        const double* cp = P.P(curCtx);
        const double cMatch = cp[kM], cDel = cp[kD], cBranch = cp[kB], cStick3 = cp[kS3];
        const int2 nr = bm.R(j + 1);
        const bool nrNonEmpty = nr.x < nr.y;
        const long long nbase = (long long)bm.O(j + 1) + (nr.y - 1);   // next column: V(nbase - i)
        const int e = he;
        const long long cbase = used + (e - 1);                       // this column: V(cbase - i)
        const long long room = bm.cap - used;
        double thr = 0.0, mx = 0.0, score = 0.0, up = 0.0;
        int i = e - 1;
        double diag = (nrNonEmpty && i + 1 >= nr.x && i + 1 < nr.y) ? bm.V(nbase - (i + 1)) : 0.0;
        bool go = i > 0;
        while (go) {
            double lf[kFillChunk];
            char nbs[kFillChunk];
#pragma unroll
            for (int q = 0; q < kFillChunk; ++q) {
                const int row = i - q;
                const bool in = nrNonEmpty && row >= nr.x && row < nr.y;
                const double x = bm.V(nrNonEmpty ? nbase - clampi(row, nr.x, nr.y - 1) : (long long)bm.O(j + 1));
                lf[q] = in ? x : 0.0;
                nbs[q] = rd[clampi(row, 0, I - 1)];
            }
#pragma unroll
            for (int q = 0; q < kFillChunk; ++q) {
                if (e - 1 - i >= room) return -1;
                const char nb = nbs[q];
                const double left = lf[q];
                const bool same = nb == nextBase;
                const double mpe = diag * (same ? P.prNot : P.prThird);
                score = 0.0;
                if (i < I - 1) score = 0.0 + mpe * cMatch;
                else if (i == I - 1 && j == J - 1) score = 0.0 + mpe;
                if (i < I - 1 && i > 0) score = score + up * (same ? cBranch : cStick3);
                if (j < J - 1 && j > 0) score = score + left * cDel;
                bm.V(cbase - i) = score;
                if (score > mx) { mx = score; thr = mx / P.sdn; }
                up = score;
                diag = left;
                --i;
                go = i > 0 && (score >= thr || i >= reqBegin);
                if (!go) break;
            }
        }
        const int b = i + 1;
        // FinishEditingColumn, then the next column's end hint: scan down from the top while the
        // scaled value stays below the unscaled threshold (:282-285).
        int nhe = b;
        if (mx != 0.0 && mx != 1.0) {
#pragma unroll 4
            for (int k = e - 1; k >= b; --k) {
                const double v = bm.V(cbase - k) / mx;
                bm.V(cbase - k) = v;
                if (nhe == b && !(v < thr)) nhe = k + 1;
            }
            bm.L(j) = log(mx);
        } else {
            for (int k = e - 1; k >= b; --k)
                if (!(bm.V(cbase - k) < thr)) { nhe = k + 1; break; }
            bm.L(j) = 0.0;
        }
        bm.R(j) = make_int2(b, e);
        bm.O(j) = (int)used;
        used += e - b;
        hb = b;
        he = nhe;
        nextBase = curBase;
        nextCtx = curCtx;
    }
    if (used + 1 > bm.cap) return -1;
    const double em = (tv.Base(0) == rd[0]) ? P.prNot : P.prThird;
    const double raw = em * beta_at(bm, 1, 1);
    const double c = (0.0 < raw) ? raw : 0.0;
    double v = raw;
    double ls = 0.0;
    if (c != 0.0 && c != 1.0) { v = raw / c; ls = log(c); }
    bm.V(used) = v;
    bm.R(0) = make_int2(0, 1);
    bm.O(0) = (int)used;
    bm.L(0) = ls;
    used += 1;
    return used;
}

template <int S>
__device__ __forceinline__ double sum_ls(const StridedBand<S>& m, int n)
{
    double s = 0.0;   // std::accumulate from 0.0, left to right
    for (int k = 0; k < n; ++k) s = s + m.L(k);
    return s;
}

}  // namespace pbccs
