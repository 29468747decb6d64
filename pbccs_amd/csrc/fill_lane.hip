// pbccs_amd/csrc/fill_lane.hip -- band fill with one lane per read and an LDS ring per lane.
//
// FillAlphaBeta + flip-flop controller (SimpleRecursor.cpp:60-296, 642-691) for reads whose columns stay
// within H rows -- the typical band (11-27 rows at configs[1]).  One lane owns one
// read and runs the reference's column loop serially, in its exact operation order: the insertion chain
// a_i = (m_i + a_{i-1} k_i) + d_i is then a plain register dependence, and a wave carries 64 reads' cells
// per instruction.  The cooperative fill (fill_coop.hip) spends ~12 wave-instructions per band cell
// resolving that chain across lanes (rocprofv3 SQ_INSTS_VALU, profiles/r2b_pmc_summary.txt); here a cell
// costs one lane-step of ~25 lane-instructions.
//
// Storage: the previous column lives in an LDS ring of H slots per lane, slot = row mod H, laid out
// [slot][lane] so a wave's accesses hit distinct banks whatever rows the lanes are on.  A column is
// computed in place over its predecessor: row i reads the previous column's row i (`left`) and then
// overwrites that slot; the previous row i - 1 (`diag`) is the value read one step earlier.  That is safe
// while the two columns together span at most H rows (checked per column); a read whose band outgrows the
// ring aborts with kFillTall and the host re-runs it on the cooperative paths.  Finished (scaled) columns
// are written to the read's compact band in HBM, where the scoring kernels read them.
#include "arrow_device.hpp"
#include "arrow_kernels.hpp"

#include <cstdlib>
#include <stdexcept>

namespace pbccs {
namespace {

constexpr int kLaneCtxDoubles = 9 * kCtxStride;

// The read's template window (a fill never carries a virtual mutation): TplView::Plain only.
struct LaneWin {
    const char* T;   // strand template
    int L;           // strand template length
    int start;       // window start on the strand
    __device__ __forceinline__ void At(int idx, char& b, int& c) const
    {
        const int g = idx + start;
        b = T[g];
        c = (g + 1 < L) ? context_index(T[g], T[g + 1]) : kCtxZero;
    }
    __device__ __forceinline__ char Base(int idx) const { return T[idx + start]; }
};

struct LaneTask {
    int I, J;
    const char* rd;        // read bases
    LaneWin tv;            // template window
    const double* ctx;     // 9 x kCtxStride transition parameters of the read's ZMW
    double prNot, prThird, sdn;
    double* ring;          // this lane's slot 0; slot s at ring[s * 64]
    // in-kernel band growth (LaneFill::valBump)
    int r;
    double* pool;
    unsigned long long* bump;
    long long limit;
    long long* gA;
    long long* gB;
    long long* gCap;
};

struct LanePass {
    long long used;   // values used by the pass (also when they did not fit)
    double last;      // alpha(I, J) or beta(0, 0)
    double sumL;      // accumulate(logScales, 0.0) in column order
    bool tall;        // a column outgrew the ring
    bool changed;     // some column's [begin, end) differs from the previous pass of this matrix
};

template <int H>
__device__ __forceinline__ double& slot(const LaneTask& T, int row)
{
    static_assert((H & (H - 1)) == 0, "ring rows must be a power of two");
    return T.ring[(row & (H - 1)) * 64];
}

constexpr int kLaneChunk = 8;

// Bytes rd[p .. p + 8) as one little-endian word: two aligned 8-byte loads and a funnel shift, so a lane
// reads its chunk's bases with 2 memory instructions instead of 8 (each one touches 64 lanes' scattered
// lines).  The read pool is padded by 16 bytes before the first read and 32 after the last (ArrowBatch), so
// the p in [-14, I + 7) the loops use stay inside the allocation.
__device__ __forceinline__ unsigned long long load8(const char* rd, int p)
{
    const unsigned long long addr = (unsigned long long)(rd + p);
    const unsigned long long* w = reinterpret_cast<const unsigned long long*>(addr & ~7ull);
    const unsigned sh = (unsigned)(addr & 7) * 8;
    const unsigned long long lo = w[0], hi = w[1];
    return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
}

// The previous column's values (0 outside its rows [pb, pe)) and the read bases of the kLaneChunk rows
// r0, r0 + dir, ...: alpha (dir = +1) uses rd[row - 1], beta (dir = -1) rd[row].  Every row the loops
// compute has its base inside the read (alpha rows are in [1, I), beta rows in [1, I)); prefetched rows
// past the band may read padding or a neighbouring read, and are never used.
template <int H>
__device__ __forceinline__ void fetch_rows(const LaneTask& T, int r0, int dir, int pb, int pe, double* lf,
                                           unsigned long long& bases)
{
#pragma unroll
    for (int q = 0; q < kLaneChunk; ++q) {
        const int row = r0 + dir * q;
        const double x = slot<H>(T, row);
        lf[q] = (row >= pb && row < pe) ? x : 0.0;
    }
    // alpha: bytes rd[r0 - 1 .. r0 + 7), base q at byte q; beta: bytes rd[r0 - 7 .. r0 + 1), base q at byte 7 - q
    bases = dir > 0 ? load8(T.rd, r0 - 1) : load8(T.rd, r0 - 7);
}

__device__ __forceinline__ char base_of(unsigned long long w, int q, int dir)
{
    const int k = dir > 0 ? q : 7 - q;
    return (char)((w >> (8 * k)) & 0xff);
}

// Move the read's alpha/beta region pair to a larger one taken from the pool's free top (as
// fill_coop.hip grow_bands, one lane): keep the running pass's first keepM values and the other matrix's
// last complete pass (keepO values).  False when the mapped headroom is exhausted.
__device__ __forceinline__ bool lane_grow(const LaneTask& T, Band& m, Band& o, bool mIsAlpha, long long need, long long keepM,
                          long long keepO, int done, int total)
{
    if (!T.bump) return false;
    const long long full = (long long)(T.I + 1) * (T.J + 1) + 1;
    const long long proj = need * (long long)total / (long long)max(done, 1);
    long long cap = max(m.cap + m.cap / 2, proj + proj / 8 + 64);
    cap = max(min(cap, full), need);
    const unsigned long long base = atomicAdd(T.bump, (unsigned long long)(2 * cap));
    if (base + 2 * (unsigned long long)cap > (unsigned long long)T.limit) return false;
    double* na = T.pool + base;
    double* nb = na + cap;
    double* nm = mIsAlpha ? na : nb;
    double* no = mIsAlpha ? nb : na;
    for (long long k = 0; k < keepM; ++k) nm[k] = m.val[k];
    for (long long k = 0; k < keepO; ++k) no[k] = o.val[k];
    m.val = nm;
    o.val = no;
    m.cap = cap;
    o.cap = cap;
    T.gA[T.r] = (long long)base;
    T.gB[T.r] = (long long)base + cap;
    T.gCap[T.r] = cap;
    return true;
}

// ---- FillAlpha (SimpleRecursor.cpp:60-181), one lane ------------------------------------------------
template <int H>
__device__ __forceinline__ LanePass lane_alpha(const LaneTask& T, Band& a, Band& o, bool guided, bool selfValid, bool& ovf,
                               long long keepO)
{
    const int I = T.I, J = T.J;
    LanePass out{0, 0.0, 0.0, false, !selfValid};
    if (a.cap < 1) ovf = true;
    if (!ovf) a.V(0) = 1.0;
    a.R(0) = make_int2(0, 1);
    a.O(0) = 0;
    a.L(0) = 0.0;
    slot<H>(T, 0) = 1.0;
    int pb = 0, pe = 1;
    long long used = 1;
    int hb = 1, he = 1;
    int prevCtx = kCtxZero;
    char curBase;
    int curCtx;
    T.tv.At(0, curBase, curCtx);
    char nbNext = 0;   // template base / context of the next column, loaded one column ahead
    int ncNext = kCtxZero;
    if (J > 1) T.tv.At(1, nbNext, ncNext);
    double s = 0.0;   // 0.0 + L(0)
    // column metadata of the next column, loaded one column ahead (the guide's and this matrix's previous
    // ranges of column j + 1 are read before column j + 1 overwrites them)
    int2 gNext = make_int2(0, 0), sNext = make_int2(0, 0);
    if (J > 1) {
        if (guided) gNext = o.R(1);
        if (selfValid) sNext = a.R(1);
    }
    for (int j = 1; j < J; ++j) {
        const int2 gR = gNext, sR = sNext;
        if (j + 1 < J) {
            if (guided) gNext = o.R(j + 1);
            if (selfValid) sNext = a.R(j + 1);
        }
        if (guided && gR.x < gR.y) { hb = min(gR.x, hb); he = max(gR.y, he); }   // RangeGuide (:728-757)
        const int sx = sR.x, sy = sR.y;
        if (selfValid && sx < sy) { hb = min(sx, hb); he = max(sy, he); }
        const int reqEnd = min(I, he);
        const char nextBase = nbNext;
        const int nextCtx = ncNext;
        if (j + 1 < J) T.tv.At(j + 1, nbNext, ncNext);
        const double* cp = T.ctx + curCtx * kCtxStride;
        const double* pp = T.ctx + prevCtx * kCtxStride;
        const double pMatch = pp[kM], pDel = pp[kD];
        const double cBranch = cp[kB], cStick3 = cp[kS3];
        const int b = hb;
        if (pe - b > H) { out.tall = true; return out; }
        double diag = (b - 1 >= pb && b - 1 < pe) ? slot<H>(T, b - 1) : 0.0;
        double mx = 0.0, thr = 0.0, up = 0.0;
        bool thrOk = true;   // thr == mx / sdn (computed lazily: only the loop's continue test past reqEnd reads it)
        int i = b;
        bool go = i < I;
        // rows in chunks of kLaneChunk: the previous column's values and the read bases of the next chunk are
        // loaded while this one computes (its ring slots are distinct mod H, and a row more than H below b
        // aborts as tall before its slot could alias one this column wrote)
        double lf[kLaneChunk];
        unsigned long long rbs;
        fetch_rows<H>(T, i, 1, pb, pe, lf, rbs);
        while (go) {
            double lfN[kLaneChunk];
            unsigned long long rbN;
            fetch_rows<H>(T, i + kLaneChunk, 1, pb, pe, lfN, rbN);
#pragma unroll
            for (int q = 0; q < kLaneChunk; ++q) {
                if (i - b >= H) { out.tall = true; return out; }
                const double left = lf[q];
                const char rb = base_of(rbs, q, 1);
                const double mpe = diag * (rb == curBase ? T.prNot : T.prThird);
                // 0.0 + move == move: every term is a product of non-negative probabilities
                double score = (i == 1 && j == 1) ? mpe : ((i != 1 && j != 1) ? mpe * pMatch : 0.0);
                if (i > 1) score = score + up * (rb == nextBase ? cBranch : cStick3);
                if (j > 1) score = score + left * pDel;
                slot<H>(T, i) = score;
                if (score > mx) { mx = score; thrOk = false; }
                up = score;
                diag = left;
                ++i;
                go = i < I;
                if (go && i >= reqEnd) {
                    if (!thrOk) { thr = mx / T.sdn; thrOk = true; }
                    go = score >= thr;
                }
                if (!go) break;
            }
#pragma unroll
            for (int q = 0; q < kLaneChunk; ++q) lf[q] = lfN[q];
            rbs = rbN;
        }
        const int e = i;
        if (!ovf && used + (e - b) + 1 > a.cap &&
            !lane_grow(T, a, o, true, used + (e - b) + 1, used, keepO, j + 1, J + 1))
            ovf = true;
        // ScaledMatrix::FinishEditingColumn (ScaledMatrix-inl.hpp:35-60) + the next begin hint (:161-167):
        // the first row whose scaled value reaches the unscaled threshold
        if (!thrOk) thr = mx / T.sdn;
        const bool scale = (mx != 0.0 && mx != 1.0);
        int nhb = e;
        const bool store = !ovf && used + (e - b) <= a.cap;
        // in chunks: the chunk's slots are read first, so its divisions are independent and overlap
        for (int k0 = b; k0 < e; k0 += kLaneChunk) {
            double x[kLaneChunk];
#pragma unroll
            for (int q = 0; q < kLaneChunk; ++q) x[q] = slot<H>(T, k0 + q);
#pragma unroll
            for (int q = 0; q < kLaneChunk; ++q) {
                const int k = k0 + q;
                if (k < e) {
                    const double v = scale ? x[q] / mx : x[q];
                    slot<H>(T, k) = v;
                    if (store) a.V(used + (k - b)) = v;
                    if (nhb == e && !(v < thr)) nhb = k;
                }
            }
        }
        if (!store) ovf = true;
        out.changed = out.changed || b != sx || e != sy;
        const double lsj = scale ? log(mx) : 0.0;
        a.R(j) = make_int2(b, e);
        a.O(j) = (int)used;
        a.L(j) = lsj;
        s = s + lsj;
        used += e - b;
        pb = b;
        pe = e;
        prevCtx = curCtx;
        curBase = nextBase;
        curCtx = nextCtx;
        he = e;
        hb = nhb;
    }
    // pinned final match (:169-179)
    const double em = (T.rd[I - 1] == T.tv.Base(J - 1)) ? T.prNot : T.prThird;
    const double lik = ((I - 1 >= pb && I - 1 < pe) ? slot<H>(T, I - 1) : 0.0) * em;
    const double c = (0.0 < lik) ? lik : 0.0;
    double v = lik, ls = 0.0;
    if (c != 0.0 && c != 1.0) { v = lik / c; ls = log(c); }
    if (!ovf && used + 1 > a.cap && !lane_grow(T, a, o, true, used + 1, used, keepO, J + 1, J + 1)) ovf = true;
    if (used + 1 > a.cap) ovf = true;
    if (!ovf) a.V(used) = v;
    a.R(J) = make_int2(I, I + 1);
    a.O(J) = (int)used;
    a.L(J) = ls;
    out.used = used + 1;
    out.last = v;
    out.sumL = s + ls;
    return out;
}

// ---- FillBeta (SimpleRecursor.cpp:183-296), one lane; rows run bottom-up, stored bottom-up ------------
template <int H>
__device__ __forceinline__ LanePass lane_beta(const LaneTask& T, Band& bm, Band& o, bool guided, bool selfValid, bool& ovf,
                              long long keepO)
{
    const int I = T.I, J = T.J;
    LanePass out{0, 0.0, 0.0, false, !selfValid};
    if (bm.cap < 1) ovf = true;
    if (!ovf) bm.V(0) = 1.0;
    bm.R(J) = make_int2(I, I + 1);
    bm.O(J) = 0;
    bm.L(J) = 0.0;
    slot<H>(T, I) = 1.0;
    int pb = I, pe = I + 1;
    long long used = 1;
    int hb = I, he = I;
    char nextBase;
    int nextCtx;
    T.tv.At(J - 1, nextBase, nextCtx);
    char cbNext = 0;   // template base / context of the next column (j - 2 of column j), loaded ahead
    int ccNext = kCtxZero;
    if (J > 1) T.tv.At(J - 2, cbNext, ccNext);
    int2 gNext = make_int2(0, 0), sNext = make_int2(0, 0);
    if (J > 1) {
        if (guided) gNext = o.R(J - 1);
        if (selfValid) sNext = bm.R(J - 1);
    }
    for (int j = J - 1; j > 0; --j) {
        const int2 gR = gNext, sR = sNext;
        if (j - 1 > 0) {
            if (guided) gNext = o.R(j - 1);
            if (selfValid) sNext = bm.R(j - 1);
        }
        const char curBase = cbNext;
        const int curCtx = ccNext;
        if (j - 2 >= 0) T.tv.At(j - 2, cbNext, ccNext);
        if (guided && gR.x < gR.y) { hb = min(gR.x, hb); he = max(gR.y, he); }
        const int sx = sR.x, sy = sR.y;
        if (selfValid && sx < sy) { hb = min(sx, hb); he = max(sy, he); }
        const int reqBegin = max(0, hb);
        const double* cp = T.ctx + curCtx * kCtxStride;
        const double cMatch = cp[kM], cDel = cp[kD], cBranch = cp[kB], cStick3 = cp[kS3];
        const int e = he;
        if (e - pb > H) { out.tall = true; return out; }
        int i = e - 1;
        double diag = (i + 1 >= pb && i + 1 < pe) ? slot<H>(T, i + 1) : 0.0;
        double mx = 0.0, thr = 0.0, up = 0.0;
        bool thrOk = true;
        bool go = i > 0;
        double lf[kLaneChunk];
        unsigned long long nbs;
        fetch_rows<H>(T, i, -1, pb, pe, lf, nbs);
        while (go) {
            double lfN[kLaneChunk];
            unsigned long long nbN;
            fetch_rows<H>(T, i - kLaneChunk, -1, pb, pe, lfN, nbN);
#pragma unroll
            for (int q = 0; q < kLaneChunk; ++q) {
                if (e - 1 - i >= H) { out.tall = true; return out; }
                const double left = lf[q];
                const char nb = base_of(nbs, q, -1);
                const bool same = nb == nextBase;
                const double mpe = diag * (same ? T.prNot : T.prThird);
                double score = 0.0;
                if (i < I - 1) score = mpe * cMatch;   // 0.0 + x == x for the non-negative products
                else if (i == I - 1 && j == J - 1) score = mpe;
                if (i < I - 1 && i > 0) score = score + up * (same ? cBranch : cStick3);
                if (j < J - 1 && j > 0) score = score + left * cDel;
                slot<H>(T, i) = score;
                if (score > mx) { mx = score; thrOk = false; }
                up = score;
                diag = left;
                --i;
                go = i > 0;
                if (go && i < reqBegin) {
                    if (!thrOk) { thr = mx / T.sdn; thrOk = true; }
                    go = score >= thr;
                }
                if (!go) break;
            }
#pragma unroll
            for (int q = 0; q < kLaneChunk; ++q) lf[q] = lfN[q];
            nbs = nbN;
        }
        const int b = i + 1;
        if (!ovf && used + (e - b) + 1 > bm.cap &&
            !lane_grow(T, bm, o, false, used + (e - b) + 1, used, keepO, J - j + 1, J + 1))
            ovf = true;
        // FinishEditingColumn, then the next column's end hint: scan down from the top while the scaled
        // value stays below the unscaled threshold (:282-285)
        if (!thrOk) thr = mx / T.sdn;
        const bool scale = (mx != 0.0 && mx != 1.0);
        int nhe = b;
        const bool store = !ovf && used + (e - b) <= bm.cap;
        for (int k0 = e - 1; k0 >= b; k0 -= kLaneChunk) {
            double x[kLaneChunk];
#pragma unroll
            for (int q = 0; q < kLaneChunk; ++q) x[q] = slot<H>(T, k0 - q);
#pragma unroll
            for (int q = 0; q < kLaneChunk; ++q) {
                const int k = k0 - q;
                if (k >= b) {
                    const double v = scale ? x[q] / mx : x[q];
                    slot<H>(T, k) = v;
                    if (store) bm.V(used + (e - 1 - k)) = v;
                    if (nhe == b && !(v < thr)) nhe = k + 1;
                }
            }
        }
        if (!store) ovf = true;
        out.changed = out.changed || b != sx || e != sy;
        const double lsj = scale ? log(mx) : 0.0;
        bm.R(j) = make_int2(b, e);
        bm.O(j) = (int)used;
        bm.L(j) = lsj;
        used += e - b;
        pb = b;
        pe = e;
        hb = b;
        he = nhe;
        nextBase = curBase;
        nextCtx = curCtx;
    }
    const double em = (T.tv.Base(0) == T.rd[0]) ? T.prNot : T.prThird;
    const double raw = em * ((1 >= pb && 1 < pe) ? slot<H>(T, 1) : 0.0);
    const double c = (0.0 < raw) ? raw : 0.0;
    double v = raw, ls = 0.0;
    if (c != 0.0 && c != 1.0) { v = raw / c; ls = log(c); }
    if (!ovf && used + 1 > bm.cap && !lane_grow(T, bm, o, false, used + 1, used, keepO, J + 1, J + 1)) ovf = true;
    if (used + 1 > bm.cap) ovf = true;
    if (!ovf) bm.V(used) = v;
    bm.R(0) = make_int2(0, 1);
    bm.O(0) = (int)used;
    bm.L(0) = ls;
    // accumulate(logScales, 0.0) in column order 0..J (this lane wrote every L(j) of the pass)
    double s = 0.0 + ls;
    for (int k = 1; k <= J; ++k) s = s + bm.L(k);
    out.used = used + 1;
    out.last = v;
    out.sumL = s;
    return out;
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// k_fill_lane: one lane per read, 64 reads per 64-thread block; LDS = H x 64 doubles (the reads' rings).
// ------------------------------------------------------------------------------------------------
template <int H, int MINW>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MINW, 8))) k_fill_lane(DevBatch B, CoopFill F, const int* __restrict__ reads, int n)
{
    __shared__ double ring[H * 64];
    const int lane = threadIdx.x;
    const int t = blockIdx.x * 64 + lane;
    if (t >= n) return;
    const int r = reads[t];
    const int z = B.rZmw[r];
    const int I = B.rLen[r];
    const TplView tv = window_view(B, r);
    const int J = tv.Length();
    if (I < 1 || J < 1) {
        B.rStatus[r] = kFillBadInput;
        return;
    }
    LaneTask T;
    T.I = I;
    T.J = J;
    T.rd = B.seqPool + B.rSeqOff[r];
    T.tv.T = tv.T;
    T.tv.L = tv.L;
    T.tv.start = tv.start;
    T.ctx = B.zCtx + (long long)z * kLaneCtxDoubles;
    T.prNot = B.prNot;
    T.prThird = B.prThird;
    T.sdn = B.sdn;
    T.ring = ring + lane;
    T.r = r;
    T.pool = B.valPool;
    T.bump = F.valBump;
    T.limit = F.valLimit;
    T.gA = F.rValA;
    T.gB = F.rValB;
    T.gCap = F.rValCap;

    const long long cb = B.rColBase[r];
    Band a, bm;
    a.range = B.aRange + cb;
    a.off = B.aOff + cb;
    a.ls = B.aLs + cb;
    a.val = B.valPool + B.rValA[r];
    a.cap = B.rValCap[r];
    bm.range = B.bRange + cb;
    bm.off = B.bOff + cb;
    bm.ls = B.bLs + cb;
    bm.val = B.valPool + B.rValB[r];
    bm.cap = B.rValCap[r];

    bool ovf = false;
    long long needA = 0, needB = 0;
    unsigned long long cells = 0, passes = 0;
    int flips = 0;
    // FillAlphaBeta (SimpleRecursor.cpp:642-691) as a pass sequencer, with the fixed-point skip of
    // fill_coop.hip (a pass depends only on the other matrix's ranges and its own previous ranges)
    LanePass pa{0, 0.0, 0.0, false, false}, pb{0, 0.0, 0.0, false, false};
    long long ua = 0, ub = 0;
    const int maxSize = (int)(0.5 + kRebandFrac * (I + 1) * (J + 1));
    bool mismatched = false;
    int unchanged = 0;
    for (int step = 0;; ++step) {
        bool doAlpha;
        if (step < 2) doAlpha = step == 0;
        else if (step == 2 && !(ua >= maxSize || ub >= maxSize)) {
            step = 5;   // no reband
            doAlpha = true;
        } else doAlpha = step == 2 || step == 4;
        if (step == 5 && (flips == 0 || flips == 3))   // first entry into the flip-flop loop
            mismatched = fabs((log(pa.last) + pa.sumL) - (log(pb.last) + pb.sumL)) > kAlphaBetaTol;
        if (step >= 5) {
            if (!(mismatched && flips <= kMaxFlipFlops)) break;
            doAlpha = flips % 2 == 0;
        }
        const bool guided = step > 0, self = step > 1;
        LanePass o = doAlpha ? lane_alpha<H>(T, a, bm, guided, self, ovf, ub) : lane_beta<H>(T, bm, a, guided, self, ovf, ua);
        if (o.tall) {
            B.rStatus[r] = kFillTall;
            return;
        }
        cells += o.used;
        passes += 1;
        if (doAlpha) {
            pa = o;
            ua = o.used;
            needA = max(needA, o.used);
        } else {
            pb = o;
            ub = o.used;
            needB = max(needB, o.used);
        }
        if (step >= 2 && step <= 4) ++flips;
        if (step >= 5) {
            ++flips;
            unchanged = o.changed ? 0 : unchanged + 1;
            if (unchanged >= 2) {
                flips = kMaxFlipFlops + 1;
                break;
            }
        }
    }
    const double av = log(pa.last) + pa.sumL;
    const double bv = log(pb.last) + pb.sumL;
    const double mism = fabs(1.0 - av / bv);
    if (ovf) {
        B.rStatus[r] = kFillOverflow;
        F.usedA[r] = (int)needA;
        F.usedB[r] = (int)needB;
        return;
    }
    B.rFlips[r] = flips;
    B.rBaseline[r] = bv;
    F.usedA[r] = (int)ua;
    F.usedB[r] = (int)ub;
    B.rStatus[r] = (mism > kAlphaBetaTol) ? kFillMismatch : kFillOk;
    if (B.stats) {   // algorithmic: 8 B per stored cell + 16 B per column per fill pass
        atomicAdd(&B.stats[2 * kStatFill], cells);
        atomicAdd(&B.stats[2 * kStatFill + 1], 8ull * cells + 16ull * passes * (unsigned long long)(J + 1));
    }
}

void launch_fill_lane(const DevBatch& B, const CoopFill& F, const int* reads, int n, hipStream_t s)
{
    if (n <= 0) return;
    const dim3 grid((n + 63) / 64);
    hipLaunchKernelGGL((k_fill_lane<kFillLaneRows, 2>), grid, dim3(64), 0, s, B, F, reads, n);
}

}  // namespace pbccs
