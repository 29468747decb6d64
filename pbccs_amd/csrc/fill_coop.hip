// pbccs_amd/csrc/fill_coop.hip -- cooperative band fill: G lanes per read.
//
// FillAlphaBeta + flip-flop controller (SimpleRecursor.cpp:60-296, 642-691) with the rows of a column
// spread over the G lanes of a group (G = 16: four reads per wavefront; G = 64: one read per wavefront
// for tall bands).  Per column:
//   1. every lane computes, for its row i, the three terms that do not depend on the in-column chain:
//        m_i = match move (diag * emission * transition), k_i = insertion transition, d_i = deletion move,
//      reading the previous (already scaled) column from an LDS ping-pong buffer;
//   2. the insertion chain a_i = (m_i + a_{i-1} k_i) + d_i is resolved with G shift-by-one DPP steps
//      (lane l holds its final value after step l; each step is the reference's exact operation order,
//      -ffp-contract=off, so every cell is bit-identical to SimpleRecursor);
//   3. a group prefix-max gives each row the running column maximum the reference's loop would hold,
//      hence its threshold maxScore / exp(ScoreDiff) and the loop's continue condition; a ballot finds
//      the row where the reference loop stops (rows past it are discarded);
//   4. the column is scaled by its maximum (ScaledMatrix::FinishEditingColumn), stored to the read's
//      compact band in HBM (coalesced: consecutive rows -> consecutive addresses) and kept in LDS as the
//      next column's input; a second ballot gives the next column's hint row.
// Columns taller than the LDS capacity abort the read with kFillTall (the host re-runs it with G = 64
// and a larger buffer, then on the lane-serial k_fill); value-capacity overflow switches the read to
// count-only mode and reports the exact size it needs (kFillOverflow).
#include "arrow_device.hpp"
#include "arrow_kernels.hpp"
#include "coop_chain.hpp"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>

namespace pbccs {
namespace {

using namespace coop;

// Everything a group needs about its read (group-uniform values) + LDS views.
template <int G>
struct Task {
    Group<G> g;
    int I, J, L, start;
    const unsigned* rdW;   // read bases, nibble-packed (LDS)
    const unsigned* tpW;   // template window bases [0, J], nibble-packed (LDS)
    const double* ctx;     // 9 x kCtxStride transition parameters
    // two ping-pong column buffers: rows [0, hcap) in LDS, rows [hcap, hcap + gRows) in this group's slot of
    // CoopFill::colScratch (gcol: the hybrid 64-lane path, whose columns are never too tall)
    double* lds0;
    double* lds1;
    double* glob0;
    double* glob1;
    int hcap;              // LDS rows per column buffer
    int rowsCap;           // rows a column may hold (hcap, or hcap + gRows for the hybrid path)
    bool gcol;
    int ckK;               // checkpoint interval: 0 keeps every column's values, else only ckpt_col_a/b columns
    bool chainExit;            // G = 64 serial steps with the early exit (insertion_chain64_exit)
    int slackDiv;              // regrow_bands slack: need / slackDiv
    double prNot, prThird, sdn;
    double sdnInvLow;   // a double strictly below 1 / sdn (early-exit test of the 64-lane chain)
    double sdnInvHigh;  // a double strictly above 1 / sdn (thr_ge)
    double devScale;    // SCAN: CoopFill::devScale (test hook: the bounds inflated)
    double sdnInv;      // SCAN: fl(1 / sdn) -- pm * sdnInv is within 2 u of fl(pm / sdn) (the margins hold 8 u)
    // in-kernel band growth (CoopFill::valBump): pool, bump pointer, mapped limit, descriptor arrays
    int r;
    double* pool;
    unsigned long long* bump;
    long long limit;
    long long* gA;
    long long* gB;
    long long* gCap;

    // buffer b (0 / 1), row k (no runtime-indexed pointer arrays: they would live in scratch).  The hybrid
    // path selects an LDS or global address per lane and accesses it through one generic (flat) pointer.
    // (buffer 1 follows buffer 0 in both places: offsets, not a selected pointer member, keep T in registers)
    // R = 2 (split): the LDS rows of a buffer are two planes, even rows then odd rows (row k at (k & 1) hcap / 2 +
    // k / 2).  A lane's rows are k0 + 2 lane + r with k0 + r of one parity across the group, so every LDS access
    // of the group lands in one plane at consecutive doubles -- no bank conflicts (a 16-byte lane stride into one
    // linear buffer put two lanes on each bank: 27% of the tall fill's LDS cycles, profiles/r4h2_pmc_summary.txt).
    bool split;
    __device__ __forceinline__ int lrow(int k) const { return split ? (k & 1) * (hcap >> 1) + (k >> 1) : k; }
    __device__ __forceinline__ double* cptr(int b, int k) const
    {
        if (!gcol) return lds0 + (b ? hcap : 0) + lrow(k);
        return k < hcap ? lds0 + (b ? hcap : 0) + lrow(k) : glob0 + (b ? glob1 - glob0 : 0) + (k - hcap);
    }
    __device__ __forceinline__ double cget(int b, int k) const { return *cptr(b, k); }
    __device__ __forceinline__ void cset(int b, int k, double v) const { *cptr(b, k) = v; }
    // template window base idx (nibble code; past the window or the template: kBaseOther) and its context slot
    __device__ __forceinline__ int TBase(int idx) const
    {
        return nib(tpW, max(idx, 0));
    }
    __device__ __forceinline__ int TCtx(int idx) const
    {
        return (start + idx + 1 < L) ? ctx_code(TBase(idx), TBase(idx + 1)) : kCtxZero;
    }
    // read base x (0 <= x < I)
    __device__ __forceinline__ int RB(int x) const
    {
        return nib(rdW, x);
    }
};

struct PassOut {
    long long used;   // cells the pass computed (the reference's used entries; also when they did not fit)
    long long stored; // values it keeps (= used for a full band; checkpoint columns only otherwise)
    double last;      // alpha(I, J) or beta(0, 0)
    double sumL;      // accumulate(logScales, 0.0) left to right
    bool tall;        // a column exceeded the LDS buffer
    bool changed;     // some column's [begin, end) differs from the previous pass of this matrix
    bool regrow;      // the pass outgrew its region and ran to its end counting only: `used` is its exact need
    int maxH;         // the pass's tallest column (rows)
    double dev;       // SCAN: bound on |log-likelihood - the reference's| of this pass (last + sumL), 0 when exact
    int unc;          // SCAN: decisions that lay within the deviation bound of their threshold (bit 0: a band end,
                      // bit 1: a begin hint)
};

// PBCCS_FILL_WORK diagnostics (CoopFill::work): the group's chunk steps and, per lane, the chunk bodies this lane
// issued as the wave's first active lane (so the lanes' sum is the wave's chunk issues)
struct Work {
    bool on;
    long long steps;
    long long issues;
};
__device__ __forceinline__ void count_issue(Work& W)
{
    if (W.on) {
        const unsigned long long act = __ballot(1);
        if ((int)(threadIdx.x & 63) == __ffsll((long long)act) - 1) W.issues += 1;
    }
}

// Column rows in global memory (the hybrid path's rows past the LDS buffer): a column's rows are written by
// one lane and read by its neighbours in the next column, so the group's stores must have completed before
// the next column's loads.  One workgroup-scope fence after each column that reached global rows (the group
// is one wavefront on one CU, whose L1 its loads and stores share).  LDS rows need nothing: a wavefront's LDS
// operations complete in order.
__device__ __forceinline__ void col_fence(bool gcol)
{
    if (gcol) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
}

// The reference loop's `score >= threshold` with threshold = maxScore / exp(ScoreDiff) (SimpleRecursor.cpp:
// 110-112), i.e. x >= fl(pm / sdn), without the division: for a normal pm, fl(pm * hi) lies above and fl(pm * lo)
// below every rounding of pm / sdn (hi / lo are 1 / sdn widened by 2^-50, three roundings cost at most 3 * 2^-53),
// so both products decide the comparison exactly unless x falls between them -- a band 2^-49 wide around the
// threshold.  `amb` flags that case (and a pm too small for the bound); the caller divides there.
__device__ __forceinline__ bool thr_ge(double x, double pm, double lo, double hi, bool& amb)
{
    const bool ge = x >= pm * hi;
    const bool lt = x < pm * lo;
    amb = pm != 0.0 && (pm < 0x1p-960 || (!ge && !lt));
    return ge || pm == 0.0;
}

// ---- the certified fast path (SCAN) ------------------------------------------------
// With the reassociated chain (scan_chain64) a cell's value is not the reference's bit for bit.  Both are within
// a relative distance of the exact real-arithmetic value of the same recursion (all terms are non-negative: a sum's
// relative error is at most its terms' largest plus u, a product's the sum of its factors' plus u), which a pass
// tracks as D.  Per column: the reference's serial chain adds at most 3 u per row it runs (a mul and two adds on the
// dependent path, propagated with weight <= 1); the scan forms each cell from products of up to a chunk's k's (a
// product of n factors carries at most n - 1 roundings in any order) and sums over six composition levels, so it adds
// at most (rows of the chunk + 40) u per chunk, the carry's error propagating with weight <= 1; the inputs m and d
// add 3 u and the column scale u.  D accumulates over the pass's columns.  A decision (x >= threshold) is certain when
// x and the threshold are further apart than 2 D + 4 u of the larger; otherwise the read is re-run on the exact path
// (kFillUncertain).
__device__ __forceinline__ double scan_col_dev(double D, int chunks, int rowsPerChunk)
{
    return D + (4.0 * (double)chunks * (double)rowsPerChunk + 40.0 * (double)chunks + 8.0) * kUnitRoundoff;
}
// Exact zeros are exact on both paths (a cell is 0 only when every term reaching it is, whatever the association),
// so 0 against a 0 threshold (the running maximum of leading zero rows) is the reference's decision, not an uncertain one.
__device__ __forceinline__ bool near_thr(double x, double t, double margin)
{
    const double mx = fmax(x, t);
    return mx > 0.0 && fabs(x - t) <= margin * mx;
}

// ---- band growth ---------------------------------------------------------------------------------
template <int G>
__device__ __forceinline__ void copy_vals(int lane, double* __restrict__ dst, const double* __restrict__ src, long long n)
{
    long long k = lane;
    for (; k + 3 * G < n; k += 4 * G) {
        const double x0 = src[k], x1 = src[k + G], x2 = src[k + 2 * G], x3 = src[k + 3 * G];
        dst[k] = x0;
        dst[k + G] = x1;
        dst[k + 2 * G] = x2;
        dst[k + 3 * G] = x3;
    }
    for (; k < n; k += G) dst[k] = src[k];
}

// Move the read's alpha/beta region pair to a larger one taken from the pool's free top, for a pass of
// matrix `m` that outgrew it.  That pass ran to its end counting only (no value, range, offset or scale
// stores: its inputs -- the other matrix's ranges and this matrix's previous ranges -- are untouched), so
// `need` is its exact size; the caller re-runs it into the new region.  `o` keeps its first keepO values (its
// last complete pass).  Both regions get max(need, keepO) + 1/slackDiv + 64: an exploded alpha band and the
// beta band after it are the same size to within a few cells.  Returns false when the mapped headroom is
// exhausted (the caller then falls back to count-only mode and the host re-runs the read).
template <int G>
__device__ bool regrow_bands(const Task<G>& T, Band& m, Band& o, bool mIsAlpha, long long need, long long keepO)
{
    if (!T.bump) return false;
    const long long full = (long long)(T.I + 1) * (T.J + 1) + 1;
    long long cap = max(need, keepO);
    cap = max(min(cap + cap / T.slackDiv + 64, full), max(need, keepO));
    unsigned long long base = 0;
    if (T.g.lane == 0) base = atomicAdd(T.bump, (unsigned long long)(2 * cap));
    base = (unsigned long long)__shfl((long long)base, 0, G);
    if (base + 2 * (unsigned long long)cap > (unsigned long long)T.limit) return false;
    __threadfence();   // the group's earlier band stores are visible to every lane's loads below
    double* na = T.pool + base;          // alpha region first, beta region after it
    double* nb = na + cap;
    double* nm = mIsAlpha ? na : nb;
    double* no = mIsAlpha ? nb : na;
    copy_vals<G>(T.g.lane, no, o.val, keepO);
    m.val = nm;
    o.val = no;
    m.cap = cap;
    o.cap = cap;
    if (T.g.lane == 0) {
        T.gA[T.r] = (long long)base;
        T.gB[T.r] = (long long)base + cap;
        T.gCap[T.r] = cap;
    }
    return true;
}

// Log-scale sum of a finished pass.  ScaledMatrix::FinishEditingColumn's log(max) (0.0 for an unscaled
// column, as the reference's `scale ? log(max) : 0`) was taken off the column path: each lane keeps one
// column's scale factor of a G-column block in a register and the block's logs are taken together and stored
// at its end.  Here one lane sums all J + 1 in column order from 0.0 -- accumulate(logScales, 0.0) -- and the
// group gets the sum.
template <int G>
__device__ double finish_log_scales(const Task<G>& T, const Band& m, int J)
{
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");   // the group's stores before lane 0's loads
    double s = 0.0;
    if (T.g.lane == 0) {   // loads batched 8 at a time so the serial adds, not the load latency, set the pace
        int k = 0;
        for (; k + 7 <= J; k += 8) {
            double v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = m.L(k + q);
#pragma unroll
            for (int q = 0; q < 8; ++q) s = s + v[q];
        }
        for (; k <= J; ++k) s = s + m.L(k);
    }
    return T.g.bcast(s, 0);
}

// ---- FillAlpha (SimpleRecursor.cpp:60-181) --------------------------------------------------------
// A column's rows run in chunks of CH = G x R rows, R consecutive rows per lane (lane l: rows i0 + l R ..
// i0 + l R + R - 1); R > 1 hands the chain on once per R rows (insertion_chain_rows).
// SCAN (G = 64, R > 1): the reassociated chain and its certification.
#ifndef PBCCS_TALL_PREFETCH   // A/B builds
#define PBCCS_TALL_PREFETCH 1
#endif
template <int G, int R, bool SCAN, bool GC>
__device__ PassOut coop_alpha(const Task<G>& T, Band& a, Band& o, bool guided, bool selfValid, bool& ovf, long long keepO,
                              Work& W)
{
    constexpr int CH = G * R;
    // loads one chunk ahead (the previous column's rows in the chunk loop, this column's in the scale loop): the
    // hybrid path (global rows) and, with PBCCS_TALL_PREFETCH, the LDS-only tall path too -- its waves spent 35% of
    // their cycles parked on waitcnt (SQ_WAIT_ANY, profiles/r9p_binding_summary.json)
    constexpr bool PF = GC || (G == 64 && PBCCS_TALL_PREFETCH && !SCAN);   // the chunk loop's (no room for it in
                                                                           // the scan kernel's registers)
    constexpr bool PFS = GC || (G == 64 && PBCCS_TALL_PREFETCH);            // the scale loop's
    const Band* guide = guided ? &o : nullptr;
    const int I = T.I, J = T.J, lane = T.g.lane;
    PassOut out{0, 0, 0.0, 0.0, false, !selfValid, false, 1, 0.0, 0};
    bool counting = false;   // outgrew the region: finish the pass without stores (regrow_bands)
    (void)keepO;
    if (a.cap < 1) ovf = true;
    if (lane == 0) {
        if (!ovf) a.V(0) = 1.0;
        a.R(0) = make_int2(0, 1);
        a.O(0) = 0;
        a.L(0) = 0.0;
    }
    int prev = 0, cur = 1;   // column buffers
    if (lane == 0) T.cset(prev, 0, 1.0);
    int pb = 0, pe = 1;
    double D = 0.0;     // SCAN: the pass's relative deviation bound so far (scan_col_dev)
    int unc = 0;   // SCAN: the uncertain decisions met (PassOut::unc)
    long long used = 1, stored = 1;   // cells computed / values kept (column 0 is always kept)
    int hb = 1, he = 1;
    int prevCtx = kCtxZero;
    int curBase = T.TBase(0), curCtx = T.TCtx(0);
    // template bases of the next two columns, loaded one column ahead
    int tA = T.TBase(1), tB = T.TBase(2);
    double myF = 1.0;   // the scale factor of column (block start + lane) of the current G-column block
    // ranges of the guide and of this matrix's previous pass, prefetched one G-column block ahead
    // (a.R(jj) of a later block is read before this pass overwrites it)
    // G = 64: lane l holds column (block + l) and v_readlane hands it out; G = 16 (LDS permutes would sit on
    // the column path): every lane of the group loads the next column's ranges one column ahead
    int2 gR = make_int2(0, 0), sR = make_int2(0, 0), gN = make_int2(0, 0), sN = make_int2(0, 0);
    {
        const int jj = G == 64 ? 1 + lane : 1;
        if (guide && jj < J) gN = guide->R(jj);
        if (selfValid && jj < J) sN = a.R(jj);
    }
    for (int j = 1; j < J; ++j) {
        const int jb = (j - 1) & (G - 1);
        int gx = 0, gy = 0, sx = 0, sy = 0;
        if constexpr (G == 64) {
            if (jb == 0) {
                gR = gN;
                sR = sN;
                const int jj = j + G + lane;
                if (guide && jj < J) gN = guide->R(jj);
                if (selfValid && jj < J) sN = a.R(jj);
            }
            if (guide) { gx = T.g.bcast(gR.x, jb); gy = T.g.bcast(gR.y, jb); }
            if (selfValid) { sx = T.g.bcast(sR.x, jb); sy = T.g.bcast(sR.y, jb); }
        } else {
            gR = gN;
            sR = sN;
            if (guide && j + 1 < J) gN = guide->R(j + 1);
            if (selfValid && j + 1 < J) sN = a.R(j + 1);   // read before this pass writes column j + 1
            gx = gR.x; gy = gR.y; sx = sR.x; sy = sR.y;
        }
        (void)jb;
        if (guide) {   // RangeGuide (SimpleRecursor.cpp:728-757)
            if (gx < gy) { hb = min(gx, hb); he = max(gy, he); }
        }
        if (selfValid) {
            if (sx < sy) { hb = min(sx, hb); he = max(sy, he); }
        }
        const int reqEnd = min(I, he);
        const int nextBase = tA, nextCtx = (T.start + j + 1 < T.L) ? ctx_code(tA, tB) : kCtxZero;   // TBase / TCtx(j)
        const int tC = T.TBase(j + 2);   // for the next column
        const double* cp = T.ctx + curCtx * kCtxStride;
        const double* pp = T.ctx + prevCtx * kCtxStride;
        const double pMatch = pp[kM], pDel = pp[kD];
        const double cBranch = cp[kB], cStick3 = cp[kS3];
        const int b = hb;
        double mx = 0.0, aLast[R];
        int e = b, nc = 0;
        if (b < I) {
            double carry = 0.0;
            // the previous column's rows of a chunk: diag and left of the lane's rows (ibx - 1 .. ibx + R - 1).  GC (the
            // hybrid path, rows past the LDS buffer in global memory): loaded one chunk ahead into pvN, so a global
            // row's latency overlaps the chunk before it (the loads precede the chunk's stores to the other buffer)
            auto load_prev = [&](int ibx, double (&dst)[R + 1]) {
#pragma unroll
                for (int q = 0; q <= R; ++q) {
                    const int row = ibx - 1 + q;
                    dst[q] = (row >= pb && row < pe) ? T.cget(prev, row - pb) : 0.0;
                }
            };
            double pvN[R + 1];
            if constexpr (PF) load_prev(b + lane * R, pvN);
            for (int i0 = b;; i0 += CH) {
                if ((nc + 1) * CH > T.rowsCap) {
                    out.tall = true;
                    out.used = used;
                    W.steps += nc;
                    return out;
                }
                count_issue(W);
                const int ib = i0 + lane * R;   // the lane's first row of the chunk
                double m[R], k[R], d[R], x[R];
                {
                    double pv[R + 1];   // scaled previous column at rows ib - 1 .. ib + R - 1 (diag, left)
                    if constexpr (PF) {
#pragma unroll
                        for (int q = 0; q <= R; ++q) pv[q] = pvN[q];
                        load_prev(ib + CH, pvN);
                    } else {
                        load_prev(ib, pv);
                    }
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const int i = ib + r;
                        const int rb = (i >= 1 && i <= I) ? T.RB(i - 1) : 15;
                        const double mpe = pv[r] * (rb == curBase ? T.prNot : T.prThird);
                        m[r] = (i == 1 && j == 1) ? mpe : ((i != 1 && j != 1) ? mpe * pMatch : 0.0);
                        k[r] = (i > 1) ? (rb == nextBase ? cBranch : cStick3) : 0.0;
                        d[r] = (j > 1) ? pv[r + 1] * pDel : 0.0;
                        x[r] = 0.0;
                    }
                }
                // a chunk whose inputs are all exactly zero stays zero: skip its chain (bit-exact; common
                // in the far rows of tall bands)
                bool nz = false;
#pragma unroll
                for (int r = 0; r < R; ++r) nz = nz || m[r] != 0.0 || d[r] != 0.0;
                const unsigned long long nzb = T.g.bits(nz);
                if (carry != 0.0 || nzb != 0) {
                    // the leading all-zero lanes of a chunk entered with a zero carry are exactly zero
                    const int startLane = ((G == 64 || R > 1) && carry == 0.0) ? __ffsll((long long)nzb) - 1 : 0;
                    if constexpr (R == 1) {
                        const int i = ib;
                        if (G == 64 && T.chainExit) {
                            auto maybe_stop = [&](double xv) {   // x < pm * invLow implies x < pm / sdn
                                const double pmv = fmax(mx, prefix_max<G>(xv));
                                return T.g.bits((i + 1 >= I) || (xv < pmv * T.sdnInvLow && i + 1 >= reqEnd));
                            };
                            x[0] = insertion_chain64_exit(m[0], k[0], d[0], carry, min(reqEnd, I) - 1 - i0, maybe_stop,
                                                          startLane);
                        } else {
                            x[0] = insertion_chain<G>(m[0], k[0], d[0], carry);
                        }
                    } else {
                        auto maybe_stop = [&](const double (&xv)[R]) {   // x < pm * invLow implies x < pm / sdn
                            double lp = xv[0];
#pragma unroll
                            for (int r = 1; r < R; ++r) lp = fmax(lp, xv[r]);
                            const double ex = shift_up<G>(prefix_max<G>(lp), 0.0);   // max over the lanes before
                            double run = fmax(mx, ex);
                            bool st = false;
#pragma unroll
                            for (int r = 0; r < R; ++r) {
                                run = fmax(run, xv[r]);
                                const int i = ib + r;
                                st = st || (i + 1 >= I) || (xv[r] < run * T.sdnInvLow && i + 1 >= reqEnd);
                            }
                            return T.g.bits(st);
                        };
                        const int firstRow = min(reqEnd, I) - 1 - i0;   // the first chunk row the loop may stop at
                        if constexpr (SCAN) {
                            scan_chain64<R>(m, k, d, carry, x);
                        } else {
                            insertion_chain_rows<G, R>(m, k, d, carry, x, firstRow < 0 ? 0 : firstRow / R, T.chainExit,
                                                       startLane, maybe_stop);
                        }
                    }
                }
                // the reference loop's running maximum at each row, its threshold and continue test (:110-112)
                double pmR[R];
                if constexpr (R == 1) {
                    pmR[0] = fmax(mx, prefix_max<G>(x[0]));
                } else {
                    double lp = x[0];
#pragma unroll
                    for (int r = 1; r < R; ++r) lp = fmax(lp, x[r]);
                    double run = fmax(mx, shift_up<G>(prefix_max<G>(lp), 0.0));
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        run = fmax(run, x[r]);
                        pmR[r] = run;
                    }
                }
                bool ge[R], amb = false;   // x >= pm / sdn where the test is read (rows past reqEnd - 1)
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int i = ib + r;
                    bool a;
                    ge[r] = thr_ge(x[r], pmR[r], T.sdnInvLow, T.sdnInvHigh, a);
                    amb = amb || (a && i + 1 < I && i + 1 >= reqEnd);
                }
                if (__ballot(amb) != 0) {   // rare: the quotient itself
#pragma unroll
                    for (int r = 0; r < R; ++r) ge[r] = x[r] >= pmR[r] / T.sdn;
                }
                int fs = R;   // the lane's first row where the loop stops
#pragma unroll
                for (int r = R - 1; r >= 0; --r) {
                    const int i = ib + r;
                    const bool cont = (i + 1 < I) && (ge[r] || i + 1 < reqEnd);
                    if (!cont) fs = r;
                }
                const unsigned long long stop = T.g.bits(fs < R);
                const int lastLane = stop ? (__ffsll((long long)stop) - 1) : (G - 1);
                double pmAt = pmR[R - 1];
#pragma unroll
                for (int r = 0; r < R - 1; ++r)
                    if (r == fs) pmAt = pmR[r];
                // every threshold test up to the stop row, with the chunk's margin (none is read in a chunk that ends
                // before reqEnd: its rows continue unconditionally)
                if (SCAN && i0 + CH >= reqEnd) {
                    const double mg = T.devScale * (2.0 * scan_col_dev(D, nc + 1, CH) + 8.0 * kUnitRoundoff);
                    const int rsStop = stop ? T.g.bcast(fs, lastLane) : R;
                    bool u = false;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const int i = ib + r;
                        const bool matters = (i + 1 < I) && (i + 1 >= reqEnd);
                        const bool upto = !stop || lane < lastLane || (lane == lastLane && r <= rsStop);
                        u = u || (matters && upto && near_thr(x[r], pmR[r] * T.sdnInv, mg));
                    }
                    if (T.g.bits(u) != 0) unc |= 1;
                }
                mx = T.g.bcast(pmAt, lastLane);
                ++nc;
                if (stop) {
                    const int rs = R == 1 ? 0 : T.g.bcast(fs, lastLane);
                    e = i0 + lastLane * R + rs + 1;
#pragma unroll
                    for (int r = 0; r < R; ++r) aLast[r] = x[r];
                    break;
                }
#pragma unroll
                for (int r = 0; r < R; ++r) T.cset(cur, (nc - 1) * CH + lane * R + r, x[r]);
                carry = T.g.bcast_last(x[R - 1]);
            }
        }
        const bool keep = T.ckK == 0 || ckpt_col_a(j, J, T.ckK);
        const long long add = keep ? e - b : 0;
        if (!ovf && !counting && stored + add + 1 > a.cap) {
            if (T.bump) counting = true;
            else ovf = true;
        }
        const bool store = !ovf && !counting && keep;
        // ScaledMatrix::FinishEditingColumn (ScaledMatrix-inl.hpp:35-60) + the next begin hint (:166)
        const double thrF = mx / T.sdn;
        const bool scale = (mx != 0.0 && mx != 1.0);
        int nhb = e;
        bool found = false;
        const double mh = SCAN ? T.devScale * (3.0 * scan_col_dev(D, nc, CH) + 4.0 * kUnitRoundoff) : 0.0;   // hint margin
        // two chunks per iteration: their divisions and LDS round trips overlap (tall columns have many chunks)
        // GC: the next chunk's values are loaded before this chunk's stores (its global rows' latency overlaps)
        auto load_cur = [&](int cx, double (&dst)[R]) {
#pragma unroll
            for (int r = 0; r < R; ++r) dst[r] = (cx == nc - 1) ? aLast[r] : T.cget(cur, cx * CH + lane * R + r);
        };
        double xN[R];
        if constexpr (PFS) load_cur(0, xN);
#pragma unroll 2
        for (int c = 0; c < nc; ++c) {
            int fh = R;   // the lane's first row at or above the scaled threshold
            double vv[R];   // SCAN: the chunk's scaled values (-1: outside the band), for the hint's certification
            double xc[R];
            if constexpr (PFS) {
#pragma unroll
                for (int r = 0; r < R; ++r) xc[r] = xN[r];
                if (c + 1 < nc) load_cur(c + 1, xN);
            } else {
                load_cur(c, xc);
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int kk = c * CH + lane * R + r;
                const bool ok = b + kk < e;
                const double x = xc[r];
                const double v = scale ? x / mx : x;
                if (ok) {
                    T.cset(cur, kk, v);
                    if (store && stored + kk < a.cap) a.V(stored + kk) = v;
                }
                if (fh == R && ok && !(v < thrF)) fh = r;
                vv[r] = ok ? v : -1.0;
            }
            const unsigned long long hit = T.g.bits(fh < R);
            if constexpr (SCAN) {   // the tests up to the hint row (the first hit) decide it
                if (!found) {
                    const int hl = hit ? __ffsll((long long)hit) - 1 : G;
                    const int fhl = hit ? T.g.bcast(fh, hl) : R;
                    bool u = false;
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        u = u || (vv[r] >= 0.0 && (lane < hl || (lane == hl && r <= fhl)) && near_thr(vv[r], thrF, mh));
                    if (T.g.bits(u) != 0) unc |= 2;
                }
            }
            if (!found && hit) {
                const int hl = __ffsll((long long)hit) - 1;
                nhb = b + c * CH + hl * R + (R == 1 ? 0 : T.g.bcast(fh, hl));
                found = true;
            }
        }
        if constexpr (SCAN) D = scan_col_dev(D, nc, CH) + kUnitRoundoff;   // the column's rows and its scale
        if (!counting && stored + add > a.cap) ovf = true;
        out.changed = out.changed || b != sx || e != sy;
        out.maxH = max(out.maxH, e - b);
        if (lane == 0 && !counting) {
            a.R(j) = make_int2(b, e);
            a.O(j) = (int)stored;
        }
        // ScaledMatrix's log(max) off the column path: lane jb keeps this column's factor, and at the end of a
        // G-column block every lane takes the log of its own and stores it (coalesced) -- the factors never
        // reach memory
        if (lane == jb) myF = scale ? mx : 1.0;
        if ((jb == G - 1 || j == J - 1) && !counting && lane <= jb) a.L(j - jb + lane) = (myF != 1.0) ? log(myF) : 0.0;
        used += e - b;
        stored += add;
        W.steps += nc;
        col_fence(T.gcol && nc * CH > T.hcap);   // the next column's lanes read rows this column's lanes wrote
        prev ^= 1;
        cur ^= 1;
        pb = b;
        pe = e;
        prevCtx = curCtx;
        curBase = nextBase;
        curCtx = nextCtx;
        tA = tB;
        tB = tC;
        he = e;
        hb = nhb;
    }
    // pinned final match (:169-179)
    const double em = (T.RB(I - 1) == T.TBase(J - 1)) ? T.prNot : T.prThird;
    const bool lastIn = I - 1 >= pb && I - 1 < pe;
    const double lik = (lastIn ? T.cget(prev, I - 1 - pb) : 0.0) * em;
    const double c = (0.0 < lik) ? lik : 0.0;
    double v = lik, ls = 0.0;
    if (c != 0.0 && c != 1.0) { v = lik / c; ls = log(c); }
    if (!ovf && !counting && stored + 1 > a.cap) {
        if (T.bump) counting = true;
        else ovf = true;
    }
    out.regrow = counting;
    if (lane == 0 && !counting) {
        if (!ovf) a.V(stored) = v;
        a.R(J) = make_int2(I, I + 1);
        a.O(J) = (int)stored;
        a.L(J) = ls;
    }
    out.used = used + 1;
    out.stored = stored + 1;
    out.last = v;
    if (!counting) out.sumL = finish_log_scales<G>(T, a, J);
    if constexpr (SCAN) {   // log(last) + sumL: the mass's deviation plus both sides' log and summation roundings
        out.dev = T.devScale * (1.01 * (D + 4.0 * kUnitRoundoff) +
                                2.0 * (double)(J + 4) * kUnitRoundoff * (fabs(out.sumL) + fabs(log(fmax(v, 1e-300))) + 64.0));
        out.unc = unc | ((lastIn && v == 0.0) ? 1 : 0);   // a zero inside the band: an underflow, not a structure
    }
    return out;
}

// ---- FillBeta (SimpleRecursor.cpp:183-296); rows run bottom-up, stored bottom-up --------------------
template <int G, int R, bool SCAN, bool GC>
__device__ PassOut coop_beta(const Task<G>& T, Band& bm, Band& o, bool guided, bool selfValid, bool& ovf, long long keepO,
                             Work& W)
{
    constexpr int CH = G * R;
    // loads one chunk ahead (the previous column's rows in the chunk loop, this column's in the scale loop): the
    // hybrid path (global rows) and, with PBCCS_TALL_PREFETCH, the LDS-only tall path too -- its waves spent 35% of
    // their cycles parked on waitcnt (SQ_WAIT_ANY, profiles/r9p_binding_summary.json)
    constexpr bool PF = GC || (G == 64 && PBCCS_TALL_PREFETCH && !SCAN);   // the chunk loop's (no room for it in
                                                                           // the scan kernel's registers)
    constexpr bool PFS = GC || (G == 64 && PBCCS_TALL_PREFETCH);            // the scale loop's
    const Band* guide = guided ? &o : nullptr;
    const int I = T.I, J = T.J, lane = T.g.lane;
    PassOut out{0, 0, 0.0, 0.0, false, !selfValid, false, 1, 0.0, 0};
    bool counting = false;   // outgrew the region: finish the pass without stores (regrow_bands)
    (void)keepO;
    if (bm.cap < 1) ovf = true;
    if (lane == 0) {
        if (!ovf) bm.V(0) = 1.0;
        bm.R(J) = make_int2(I, I + 1);
        bm.O(J) = 0;
        bm.L(J) = 0.0;
    }
    // the next column (j + 1) holds rows [pb, pe) at index pe - 1 - row
    int nxt = 0, cur = 1;   // column buffers
    if (lane == 0) T.cset(nxt, 0, 1.0);
    int pb = I, pe = I + 1;
    double D = 0.0;     // SCAN: the pass's relative deviation bound so far (scan_col_dev)
    int unc = 0;   // SCAN: the uncertain decisions met (PassOut::unc)
    long long used = 1, stored = 1;   // cells computed / values kept (column J is always kept)
    int hb = I, he = I;
    int nextBase = T.TBase(J - 1);
    int tA = T.TBase(J - 2), tB = nextBase;   // TBase(j - 1), TBase(j) of the column ahead, loaded one column early
    double myF = 1.0;   // the scale factor of column (block start - lane) of the current G-column block
    int2 gR = make_int2(0, 0), sR = make_int2(0, 0), gN = make_int2(0, 0), sN = make_int2(0, 0);
    {
        const int jj = G == 64 ? J - 1 - lane : J - 1;
        if (guide && jj > 0) gN = guide->R(jj);
        if (selfValid && jj > 0) sN = bm.R(jj);
    }
    for (int j = J - 1; j > 0; --j) {
        const int jb = (J - 1 - j) & (G - 1);
        int gx = 0, gy = 0, sx = 0, sy = 0;
        if constexpr (G == 64) {
            if (jb == 0) {   // block of columns (j - G, j]; prefetch the next one
                gR = gN;
                sR = sN;
                const int jj = j - G - lane;
                if (guide && jj > 0) gN = guide->R(jj);
                if (selfValid && jj > 0) sN = bm.R(jj);
            }
            if (guide) { gx = T.g.bcast(gR.x, jb); gy = T.g.bcast(gR.y, jb); }
            if (selfValid) { sx = T.g.bcast(sR.x, jb); sy = T.g.bcast(sR.y, jb); }
        } else {   // G = 16: the next column's ranges one column ahead (see coop_alpha)
            gR = gN;
            sR = sN;
            if (guide && j - 1 > 0) gN = guide->R(j - 1);
            if (selfValid && j - 1 > 0) sN = bm.R(j - 1);
            gx = gR.x; gy = gR.y; sx = sR.x; sy = sR.y;
        }
        (void)jb;
        const int curBase = tA, curCtx = (T.start + j < T.L) ? ctx_code(tA, tB) : kCtxZero;   // TBase / TCtx(j - 1)
        const int tC = T.TBase(j - 2);   // for the next column
        if (guide) {
            if (gx < gy) { hb = min(gx, hb); he = max(gy, he); }
        }
        if (selfValid) {
            if (sx < sy) { hb = min(sx, hb); he = max(sy, he); }
        }
        const int reqBegin = max(0, hb);
        const double* cp = T.ctx + curCtx * kCtxStride;
        const double cMatch = cp[kM], cDel = cp[kD], cBranch = cp[kB], cStick3 = cp[kS3];
        const int e = he;
        double mx = 0.0, aLast[R];
        int b = e, nc = 0;
        if (e - 1 > 0) {
            double carry = 0.0;
            // the next column's rows of a chunk (rows e - obx .. e - obx - R); GC: one chunk ahead (see coop_alpha)
            auto load_next = [&](int obx, double (&dst)[R + 1]) {
#pragma unroll
                for (int q = 0; q <= R; ++q) {
                    const int row = e - obx - q;
                    dst[q] = (row >= pb && row < pe) ? T.cget(nxt, pe - 1 - row) : 0.0;
                }
            };
            double pvN[R + 1];
            if constexpr (PF) load_next(lane * R, pvN);
            for (int c = 0;; ++c) {
                if ((c + 1) * CH > T.rowsCap) {
                    out.tall = true;
                    out.used = used;
                    W.steps += nc;
                    return out;
                }
                count_issue(W);
                const int ob = c * CH + lane * R;   // the lane's first offset (row e - 1 - ob)
                double m[R], k[R], d[R], x[R];
                {
                    double pv[R + 1];   // scaled next column at rows e - ob .. e - ob - R (diag, left)
                    if constexpr (PF) {
#pragma unroll
                        for (int q = 0; q <= R; ++q) pv[q] = pvN[q];
                        load_next(ob + CH, pvN);
                    } else {
                        load_next(ob, pv);
                    }
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const int i = e - 1 - ob - r;
                        const int nb = (i >= 0 && i < I) ? T.RB(i) : 15;
                        const bool same = nb == nextBase;
                        const double mpe = pv[r] * (same ? T.prNot : T.prThird);
                        m[r] = (i < I - 1) ? mpe * cMatch : ((i == I - 1 && j == J - 1) ? mpe : 0.0);
                        k[r] = (i < I - 1 && i > 0) ? (same ? cBranch : cStick3) : 0.0;
                        d[r] = (j < J - 1 && j > 0) ? pv[r + 1] * cDel : 0.0;
                        x[r] = 0.0;
                    }
                }
                // a chunk whose inputs are all exactly zero stays zero: skip its chain (bit-exact; common
                // in the far rows of tall bands)
                bool nz = false;
#pragma unroll
                for (int r = 0; r < R; ++r) nz = nz || m[r] != 0.0 || d[r] != 0.0;
                const unsigned long long nzb = T.g.bits(nz);
                if (carry != 0.0 || nzb != 0) {
                    const int startLane = ((G == 64 || R > 1) && carry == 0.0) ? __ffsll((long long)nzb) - 1 : 0;
                    if constexpr (R == 1) {
                        const int i = e - 1 - ob;
                        if (G == 64 && T.chainExit) {
                            auto maybe_stop = [&](double xv) {   // x < pm * invLow implies x < pm / sdn
                                const double pmv = fmax(mx, prefix_max<G>(xv));
                                return T.g.bits((i - 1 <= 0) || (xv < pmv * T.sdnInvLow && i - 1 < reqBegin));
                            };
                            x[0] = insertion_chain64_exit(m[0], k[0], d[0], carry, e - 1 - max(1, reqBegin) - c * G,
                                                          maybe_stop, startLane);
                        } else {
                            x[0] = insertion_chain<G>(m[0], k[0], d[0], carry);
                        }
                    } else {
                        auto maybe_stop = [&](const double (&xv)[R]) {   // x < pm * invLow implies x < pm / sdn
                            double lp = xv[0];
#pragma unroll
                            for (int r = 1; r < R; ++r) lp = fmax(lp, xv[r]);
                            const double ex = shift_up<G>(prefix_max<G>(lp), 0.0);
                            double run = fmax(mx, ex);
                            bool st = false;
#pragma unroll
                            for (int r = 0; r < R; ++r) {
                                run = fmax(run, xv[r]);
                                const int i = e - 1 - ob - r;
                                st = st || (i - 1 <= 0) || (xv[r] < run * T.sdnInvLow && i - 1 < reqBegin);
                            }
                            return T.g.bits(st);
                        };
                        const int firstOff = e - 1 - max(1, reqBegin) - c * CH;   // the first chunk offset that may stop
                        if constexpr (SCAN) {
                            scan_chain64<R>(m, k, d, carry, x);
                        } else {
                            insertion_chain_rows<G, R>(m, k, d, carry, x, firstOff < 0 ? 0 : firstOff / R, T.chainExit,
                                                       startLane, maybe_stop);
                        }
                    }
                }
                double pmR[R];
                if constexpr (R == 1) {
                    pmR[0] = fmax(mx, prefix_max<G>(x[0]));
                } else {
                    double lp = x[0];
#pragma unroll
                    for (int r = 1; r < R; ++r) lp = fmax(lp, x[r]);
                    double run = fmax(mx, shift_up<G>(prefix_max<G>(lp), 0.0));
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        run = fmax(run, x[r]);
                        pmR[r] = run;
                    }
                }
                bool ge[R], amb = false;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int i = e - 1 - ob - r;
                    bool a;
                    ge[r] = thr_ge(x[r], pmR[r], T.sdnInvLow, T.sdnInvHigh, a);
                    amb = amb || (a && i - 1 > 0 && i - 1 < reqBegin);
                }
                if (__ballot(amb) != 0) {
#pragma unroll
                    for (int r = 0; r < R; ++r) ge[r] = x[r] >= pmR[r] / T.sdn;
                }
                int fs = R;
#pragma unroll
                for (int r = R - 1; r >= 0; --r) {
                    const int i = e - 1 - ob - r;
                    const bool cont = (i - 1 > 0) && (ge[r] || i - 1 >= reqBegin);
                    if (!cont) fs = r;
                }
                const unsigned long long stop = T.g.bits(fs < R);
                const int lastLane = stop ? (__ffsll((long long)stop) - 1) : (G - 1);
                double pmAt = pmR[R - 1];
#pragma unroll
                for (int r = 0; r < R - 1; ++r)
                    if (r == fs) pmAt = pmR[r];
                // every threshold test up to the stop row (none is read in a chunk whose lowest row is >= reqBegin + 1)
                if (SCAN && e - (c + 1) * CH - 1 < reqBegin) {
                    const double mg = T.devScale * (2.0 * scan_col_dev(D, nc + 1, CH) + 8.0 * kUnitRoundoff);
                    const int rsStop = stop ? T.g.bcast(fs, lastLane) : R;
                    bool u = false;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const int i = e - 1 - ob - r;
                        const bool matters = (i - 1 > 0) && (i - 1 < reqBegin);
                        const bool upto = !stop || lane < lastLane || (lane == lastLane && r <= rsStop);
                        u = u || (matters && upto && near_thr(x[r], pmR[r] * T.sdnInv, mg));
                    }
                    if (T.g.bits(u) != 0) unc |= 1;
                }
                mx = T.g.bcast(pmAt, lastLane);
                ++nc;
                if (stop) {
                    const int rs = R == 1 ? 0 : T.g.bcast(fs, lastLane);
                    b = e - 1 - (c * CH + lastLane * R + rs);
#pragma unroll
                    for (int r = 0; r < R; ++r) aLast[r] = x[r];
                    break;
                }
#pragma unroll
                for (int r = 0; r < R; ++r) T.cset(cur, ob + r, x[r]);
                carry = T.g.bcast_last(x[R - 1]);
            }
        }
        const bool keep = T.ckK == 0 || ckpt_col_b(j, J, T.ckK);
        const long long add = keep ? e - b : 0;
        if (!ovf && !counting && stored + add + 1 > bm.cap) {
            if (T.bump) counting = true;
            else ovf = true;
        }
        const bool store = !ovf && !counting && keep;
        const double thrF = mx / T.sdn;
        const bool scale = (mx != 0.0 && mx != 1.0);
        int nhe = b;
        bool found = false;
        const double mh = SCAN ? T.devScale * (3.0 * scan_col_dev(D, nc, CH) + 4.0 * kUnitRoundoff) : 0.0;   // hint margin
        auto load_cur = [&](int cx, double (&dst)[R]) {   // GC: one chunk ahead (see coop_alpha)
#pragma unroll
            for (int r = 0; r < R; ++r) dst[r] = (cx == nc - 1) ? aLast[r] : T.cget(cur, cx * CH + lane * R + r);
        };
        double xN[R];
        if constexpr (PFS) load_cur(0, xN);
#pragma unroll 2
        for (int c = 0; c < nc; ++c) {
            int fh = R;
            double vv[R];   // SCAN: the chunk's scaled values (-1: outside the band), for the hint's certification
            double xc[R];
            if constexpr (PFS) {
#pragma unroll
                for (int r = 0; r < R; ++r) xc[r] = xN[r];
                if (c + 1 < nc) load_cur(c + 1, xN);
            } else {
                load_cur(c, xc);
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int off = c * CH + lane * R + r;
                const bool ok = e - 1 - off >= b;
                const double x = xc[r];
                const double v = scale ? x / mx : x;
                if (ok) {
                    T.cset(cur, off, v);
                    if (store && stored + off < bm.cap) bm.V(stored + off) = v;
                }
                if (fh == R && ok && !(v < thrF)) fh = r;
                vv[r] = ok ? v : -1.0;
            }
            const unsigned long long hit = T.g.bits(fh < R);
            if constexpr (SCAN) {   // the tests up to the hint row (the first hit) decide it
                if (!found) {
                    const int hl = hit ? __ffsll((long long)hit) - 1 : G;
                    const int fhl = hit ? T.g.bcast(fh, hl) : R;
                    bool u = false;
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        u = u || (vv[r] >= 0.0 && (lane < hl || (lane == hl && r <= fhl)) && near_thr(vv[r], thrF, mh));
                    if (T.g.bits(u) != 0) unc |= 2;
                }
            }
            if (!found && hit) {
                const int hl = __ffsll((long long)hit) - 1;
                nhe = e - (c * CH + hl * R + (R == 1 ? 0 : T.g.bcast(fh, hl)));
                found = true;
            }
        }
        if constexpr (SCAN) D = scan_col_dev(D, nc, CH) + kUnitRoundoff;   // the column's rows and its scale
        if (!counting && stored + add > bm.cap) ovf = true;
        out.changed = out.changed || b != sx || e != sy;
        out.maxH = max(out.maxH, e - b);
        if (lane == 0 && !counting) {
            bm.R(j) = make_int2(b, e);
            bm.O(j) = (int)stored;
        }
        if (lane == jb) myF = scale ? mx : 1.0;   // as in coop_alpha; the block runs down from column j + jb
        if ((jb == G - 1 || j == 1) && !counting && lane <= jb) bm.L(j + jb - lane) = (myF != 1.0) ? log(myF) : 0.0;
        used += e - b;
        stored += add;
        W.steps += nc;
        col_fence(T.gcol && nc * CH > T.hcap);
        nxt ^= 1;
        cur ^= 1;
        pb = b;
        pe = e;
        hb = b;
        he = nhe;
        nextBase = curBase;
        tB = tA;
        tA = tC;
    }
    const double em = (T.TBase(0) == T.RB(0)) ? T.prNot : T.prThird;
    const bool lastIn = 1 >= pb && 1 < pe;
    const double raw = em * (lastIn ? T.cget(nxt, pe - 2) : 0.0);
    const double c = (0.0 < raw) ? raw : 0.0;
    double v = raw, ls = 0.0;
    if (c != 0.0 && c != 1.0) { v = raw / c; ls = log(c); }
    if (!ovf && !counting && stored + 1 > bm.cap) {
        if (T.bump) counting = true;
        else ovf = true;
    }
    out.regrow = counting;
    if (lane == 0 && !counting) {
        if (!ovf) bm.V(stored) = v;
        bm.R(0) = make_int2(0, 1);
        bm.O(0) = (int)stored;
        bm.L(0) = ls;
    }
    out.used = used + 1;
    out.stored = stored + 1;
    out.last = v;
    if (!counting) out.sumL = finish_log_scales<G>(T, bm, J);
    if constexpr (SCAN) {   // as coop_alpha's
        out.dev = T.devScale * (1.01 * (D + 4.0 * kUnitRoundoff) +
                                2.0 * (double)(J + 4) * kUnitRoundoff * (fabs(out.sumL) + fabs(log(fmax(v, 1e-300))) + 64.0));
        out.unc = unc | ((lastIn && v == 0.0) ? 1 : 0);   // a zero inside the band: an underflow, not a structure
    }
    return out;
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// k_fill_coop: one G-lane group per read; 64 / G reads per 64-thread block.
// LDS per group: 2 column buffers (hcap doubles each), the ZMW's transition table, nibble-packed read
// and template window.
// ------------------------------------------------------------------------------------------------
// One listed read's FillAlphaBeta by the G-lane group whose LDS slot starts at gbase (task t of the launch).
template <int G, bool GC, int R, bool SCAN>
__device__ __forceinline__ void fill_read(const DevBatch& B, const CoopFill& F, const int* __restrict__ reads, int n,
                                          int t, unsigned char* gbase)
{
    const int lane = threadIdx.x & (G - 1);
    // LDS: two column buffers of hcap rows, ctx, read, template.  GC (hybrid): rows past hcap go to this
    // slot's part of F.colScratch (2 x gRows doubles)
    double* col = reinterpret_cast<double*>(gbase);
    double* ctx = col + 2 * F.hcap;
    unsigned* rdW = reinterpret_cast<unsigned*>(ctx + kCtxDoubles + 1);
    unsigned* tpW = rdW + F.readWords;

    const bool valid = t < n;
    if (F.trace && valid && lane == 0) {   // start stamps go to memory: nothing stays live across the fill
        F.trace[6LL * t] = (long long)wall_clock64();
        F.trace[6LL * t + 2] = (long long)clock64();
    }
    int r = 0, z = 0, I = 0, J = 0;
    TplView tv{};
    bool bad = true;
    if (valid) {
        r = reads[t];
        z = B.rZmw[r];
        I = B.rLen[r];
        tv = window_view(B, r);
        J = tv.Length();
        bad = I < 1 || J < 1 || (I + 7) / 8 > F.readWords || (J + 8) / 8 > F.tplWords;
        if (!bad) {
            const double* zc = B.zCtx + (long long)z * kCtxDoubles;
            for (int k = lane; k < kCtxDoubles; k += G) ctx[k] = zc[k];
        }
        if (!bad) {
            const char* rd = B.seqPool + B.rSeqOff[r];
            for (int w = lane; w < (I + 7) / 8; w += G) {
                unsigned word = 0;
                for (int q = 0; q < 8; ++q) {
                    const int x = 8 * w + q;
                    word |= (unsigned)(x < I ? base_code(rd[x]) : kBaseOther) << (4 * q);
                }
                rdW[w] = word;
            }
            for (int w = lane; w < (J + 8) / 8; w += G) {
                unsigned word = 0;
                for (int q = 0; q < 8; ++q) {
                    const int x = 8 * w + q;
                    const int g = tv.start + x;
                    word |= (unsigned)((x <= J && g < tv.L) ? base_code(tv.T[g]) : kBaseOther) << (4 * q);
                }
                tpW[w] = word;
            }
        }
    }
    // the group's own LDS slot: its lanes' stores above complete before their loads below (one wavefront; the
    // fence keeps the compiler from moving loads above them)
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    if (!valid) return;
    if (bad) {
        if (lane == 0) B.rStatus[r] = (I < 1 || J < 1) ? kFillBadInput : kFillOverflow;
        return;
    }

    Task<G> T;
    T.g.lane = lane;
    T.g.base = (int)threadIdx.x & ~(G - 1);
    T.I = I;
    T.J = J;
    T.L = tv.L;
    T.start = tv.start;
    T.rdW = rdW;
    T.tpW = tpW;
    T.ctx = ctx;
    T.lds0 = col;
    T.lds1 = col + F.hcap;
    T.glob0 = GC ? F.colScratch + (size_t)t * 2 * F.gRows : nullptr;
    T.glob1 = GC ? T.glob0 + F.gRows : nullptr;
    T.hcap = F.hcap;
    T.split = R == 2;   // launch_fill_coop checks that hcap holds whole chunks (even)
    T.rowsCap = GC ? F.hcap + F.gRows : F.hcap;
    T.gcol = GC;
    T.chainExit = F.chainExit;
    T.ckK = B.rCkpt ? B.rCkpt[r] : 0;
    T.slackDiv = max(1, F.regrowSlackDiv);
    T.prNot = B.prNot;
    T.prThird = B.prThird;
    T.sdn = B.sdn;
    T.sdnInvLow = (1.0 / B.sdn) * (1.0 - F.thrMargin);
    T.sdnInvHigh = (1.0 / B.sdn) * (1.0 + F.thrMargin);
    T.devScale = F.devScale;
    T.sdnInv = 1.0 / B.sdn;
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
    Work W{F.work != nullptr, 0, 0};
    unsigned long long regrowCells = 0, abortCells = 0;
    bool tallAbort = false;
    // MutationScorer ctor -> FillAlphaBeta (SimpleRecursor.cpp:642-691), as a pass sequencer with one
    // call site per matrix (every inlined pass costs registers and instruction cache):
    //   step 0: alpha(Null guide); step 1: beta(alpha guide); if either used >= 4% of the matrix, the
    //   reband steps 2..4 alpha(beta), beta(alpha), alpha(beta) (flip-flops += 3); then the flip-flop loop.
    // NB: alphaV / betaV are evaluated once, after the reband (SimpleRecursor.cpp:667-679).
    // Flip-flop fixed point: a pass depends only on the band ranges of the other matrix (guide) and of
    // its own previous pass (hint), never on previous values.  Once an alpha pass and the beta pass after
    // it both reproduce their predecessors' ranges, every later pass repeats them bit for bit, so the
    // remaining flip-flops are skipped and only the count the reference reports is kept.
    PassOut pa{0, 0, 0.0, 0.0, false, false, false, 0, 0.0, 0}, pb{0, 0, 0.0, 0.0, false, false, false, 0, 0.0, 0};
    int maxH = 0;
    long long ua = 0, ub = 0;   // cells of the last alpha / beta pass (the reband test)
    long long sa = 0, sb = 0;   // values they keep (region sizes)
    const int maxSize = (int)(0.5 + kRebandFrac * (I + 1) * (J + 1));
    bool mismatched = false;
    int uncAny = 0;   // SCAN: the decisions of the fill that could not be certified (kFillUncertain): bits 0-1 a pass's
                      // (PassOut::unc), bit 2 the flip-flop loop's entry test, bit 3 the final mismatch test
    int unchanged = 0;
    int regrows = 0;
    for (int step = 0;; ++step) {
        bool doAlpha;
        if (step < 2) doAlpha = step == 0;
        else if (step == 2 && !(ua >= maxSize || ub >= maxSize)) {
            step = 5;   // no reband
            doAlpha = true;
        } else doAlpha = step == 2 || step == 4;
        if (step == 5) {
            if (flips == 0 || flips == 3) {   // first entry into the flip-flop loop
                const double la = log(pa.last) + pa.sumL, lb = log(pb.last) + pb.sumL;
                mismatched = fabs(la - lb) > kAlphaBetaTol;
                // (an infinite LL is an exact zero final cell -- zeros are exact on both paths -- so its test is
                // certain; only finite LLs within the bound of the tolerance are not)
                if constexpr (SCAN)
                    if (isfinite(la) && isfinite(lb) &&
                        fabs(fabs(la - lb) - kAlphaBetaTol) <= pa.dev + pb.dev + 8.0 * kUnitRoundoff * fmax(fabs(la), fabs(lb)))
                        uncAny |= 4;
            }
        }
        if (step >= 5) {
            if (!(mismatched && flips <= kMaxFlipFlops)) break;
            doAlpha = flips % 2 == 0;
        }
        const bool guided = step > 0, self = step > 1;
        PassOut o;
        if (doAlpha) o = coop_alpha<G, R, SCAN, GC>(T, a, bm, guided, self, ovf, ub, W);
        else o = coop_beta<G, R, SCAN, GC>(T, bm, a, guided, self, ovf, ua, W);
        uncAny |= o.unc;
        if (o.tall) {   // every cell so far is thrown away: the read restarts on the 64-lane path
            tallAbort = true;
            abortCells = cells + (unsigned long long)o.used;
            break;
        }
        if (o.regrow) {   // exact region for this pass, then run it again (count-only if the pool is full)
            regrowCells += (unsigned long long)o.used;
            // (two calls, not a selected reference: the bands then stay in registers)
            const bool moved = ++regrows <= 8 && (doAlpha ? regrow_bands<G>(T, a, bm, true, o.stored, sb)
                                                          : regrow_bands<G>(T, bm, a, false, o.stored, sa));
            if (!moved) ovf = true;
            --step;
            continue;
        }
        cells += o.used;
        passes += 1;
        maxH = max(maxH, o.maxH);
        if (doAlpha) {
            pa = o;
            ua = o.used;
            sa = o.stored;
            needA = max(needA, o.stored);
        } else {
            pb = o;
            ub = o.used;
            sb = o.stored;
            needB = max(needB, o.stored);
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
    if (W.on) {   // PBCCS_FILL_WORK: where this read's computed cells went (every lane: its issue count)
        unsigned long long* w = F.work + (G == 64 ? kFillWorkSlots : 0);
        if (W.issues) atomicAdd(&w[kFillWorkIssues], (unsigned long long)W.issues);
        if (lane == 0) {
            atomicAdd(&w[kFillWorkSteps], (unsigned long long)W.steps);
            atomicAdd(&w[kFillWorkReads], 1ull);
            atomicAdd(&w[kFillWorkRegrow], regrowCells);
            if (tallAbort) atomicAdd(&w[kFillWorkTallAbort], abortCells);
            else {
                atomicAdd(&w[ovf ? kFillWorkOverflow : kFillWorkCells], cells);
                if (!ovf) atomicAdd(&w[kFillWorkPasses], passes);
            }
        }
    }
    if (tallAbort) {
        if (lane == 0) B.rStatus[r] = kFillTall;
        return;
    }
    const double av = log(pa.last) + pa.sumL;
    const double bv = log(pb.last) + pb.sumL;
    const double mism = fabs(1.0 - av / bv);
    if constexpr (SCAN)   // the AlphaBetaMismatch test (SimpleRecursor.cpp:682-688) within the bound of its threshold
        if (isfinite(av) && isfinite(bv) && isfinite(mism) &&
            fabs(mism - kAlphaBetaTol) <= (pa.dev + fabs(av / bv) * pb.dev) / fabs(bv) + 8.0 * kUnitRoundoff)
            uncAny |= 8;
    if (lane == 0) {
        if (ovf) {
            B.rStatus[r] = kFillOverflow;
            F.usedA[r] = (int)needA;
            F.usedB[r] = (int)needB;
        } else if (SCAN && uncAny) {
            B.rStatus[r] = kFillUncertain;   // the host re-runs the read on the exact path
            B.rFlips[r] = uncAny;            // (which decisions: diagnostics)
        } else {
            B.rFlips[r] = flips;
            B.rBaseline[r] = bv;
            B.rDev[r] = SCAN ? fmax(pa.dev, pb.dev) : 0.0;
            F.usedA[r] = (int)sa;   // region sizes: the values the bands keep
            F.usedB[r] = (int)sb;
            if (F.maxH) F.maxH[r] = maxH;
            B.rStatus[r] = (mism > kAlphaBetaTol) ? kFillMismatch : kFillOk;
            if (F.trace) {
                long long* tr = F.trace + 6LL * t;
                tr[1] = (long long)wall_clock64();
                tr[2] = (long long)clock64() - tr[2];
                tr[3] = (long long)cells;
                tr[4] = (long long)passes;
                tr[5] = (long long)J;
            }
            if (B.stats) {   // algorithmic: 8 B per stored cell + 16 B per column per fill pass
                constexpr int kind = G == 64 ? kStatFillTall : kStatFill;
                atomicAdd(&B.stats[2 * kind], cells);
                atomicAdd(&B.stats[2 * kind + 1], 8ull * cells + 16ull * passes * (unsigned long long)(J + 1));
                atomicAdd(&B.stats[G == 64 ? 9 : 8], cells);   // per path (diagnostics: VALU per cell)
            }
        }
    }
}


// ------------------------------------------------------------------------------------------------
// k_fill_coop: one G-lane group per read; 64 / G groups per 64-thread block (one wavefront).
// LDS per group: 2 column buffers (hcap doubles each), the ZMW's transition table, nibble-packed read
// and template window.
// Group g of block b fills task 4b + g (G = 16) / task b (G = 64).  (A dynamic assignment -- a group that finished
// its read taking the launch's next task from a counter, against the 36% idle group slots of lock-step waves,
// profiles/r5c_fill_work.json -- measured no faster, and its second inlined copy of the fill cost 5% of the
// headline in instruction-cache footprint: removed)
// ------------------------------------------------------------------------------------------------
template <int G, int MINW, bool GC, int R, bool SCAN>
__global__ void __launch_bounds__(64, MINW) k_fill_coop(DevBatch B, CoopFill F, const int* __restrict__ reads, int n)
{
    extern __shared__ __align__(16) unsigned char smem[];
    const long long wt0 = wave_t0(B.stats);
    // tall reads are the latency-critical path of every refine round: issue ahead of the 16-lane fills
    // and score waves that share the SIMD (F.prio = 0 leaves the default priority)
    if (F.prio) __builtin_amdgcn_s_setprio(3);
    const int grp = threadIdx.x / G;
    unsigned char* gbase = smem + (size_t)grp * F.groupBytes;
    fill_read<G, GC, R, SCAN>(B, F, reads, n, blockIdx.x * (64 / G) + grp, gbase);
    wave_ticks(B.stats, G == 64 ? kWaveFillTall : kWaveFill, wt0);
}

size_t coop_group_bytes(int hcap, int readWords, int tplWords)
{
    size_t b = (size_t)(2 * hcap + kCtxDoubles + 1) * sizeof(double) + (size_t)(readWords + tplWords) * 4;
    return (b + 15) & ~(size_t)15;
}

#ifndef PBCCS_NARROW_MINW   // A/B builds: waves per SIMD the 16-lane kernels are compiled for
#define PBCCS_NARROW_MINW 2
#endif
void launch_fill_coop(int G, const DevBatch& B, const CoopFill& F, const int* reads, int n, hipStream_t s)
{
    if (n <= 0) return;
    const int per = 64 / G;
    const size_t lds = (size_t)per * F.groupBytes;
    if (lds > 160 * 1024) throw std::runtime_error("fill block needs more than 160 KB of LDS");
    using K = void (*)(DevBatch, CoopFill, const int*, int);
    const bool gc = F.colScratch != nullptr;
    // two waves per SIMD: the register budget that leaves these kernels without spills (higher occupancy
    // was measured slower and needs a private segment, which the resource check in the Makefile forbids)
    // (G, rows per lane, hybrid): the narrow path with four reads per wavefront (16, 1; 2 rows per lane and sixteen
    // reads per wavefront measured slower, profiles/r4i_narrow_rows_ab.txt, r4g_narrow_ab.txt, and were removed), the tall
    // paths one read per wavefront (64, 1 / 2; R = 4 measured slowest, profiles/r4c_tall_rows_ab.txt, and was
    // removed); the hybrid kernel runs R <= 2 (the column buffers hold whole chunks either way).  Four tall reads
    // per wavefront (16, 4) measured half the speed per read (profiles/r4e_tall_grouped_ab.txt) and were removed.
    // (Scaling by a reciprocal and two FMA corrections -- bit-identical -- instead of the division measured 4%
    // slower, profiles/r4h_coldiv_ab.txt, and was removed.)
    const int R = gc ? std::min(F.rows, 2) : F.rows;
    struct Entry {
        int g, r;
        bool gc, scan;
        K k;
        bool attr;
    };
    // the certified fast path (scan) exists for the tall paths with two rows per lane
    static Entry ks[] = {
        {16, 1, false, false, (K)k_fill_coop<16, PBCCS_NARROW_MINW, false, 1, false>, false},
        {64, 1, false, false, (K)k_fill_coop<64, 2, false, 1, false>, false},
        {64, 2, false, false, (K)k_fill_coop<64, 2, false, 2, false>, false},
        {64, 2, false, true, (K)k_fill_coop<64, 2, false, 2, true>, false},
        // (the hybrid kernels -- their loads one chunk ahead -- need more than the 256 registers of two waves per
        // SIMD: one wave per SIMD, where their 60 KB of LDS per read already allows only two reads per CU)
        {64, 1, true, false, (K)k_fill_coop<64, 1, true, 1, false>, false},
        {64, 2, true, false, (K)k_fill_coop<64, 1, true, 2, false>, false},
        {64, 2, true, true, (K)k_fill_coop<64, 1, true, 2, true>, false}};
    const bool scan = F.scan && G == 64 && R == 2;
    Entry* e = nullptr;
    for (Entry& x : ks)
        if (x.g == G && x.r == R && x.gc == gc && x.scan == scan) e = &x;
    if (!e) throw std::runtime_error("no fill kernel for this group size / rows per lane / column buffer");
    if (R > 1 && ((gc ? (F.hcap + F.gRows) : F.hcap) % (G * R) != 0 || F.hcap % 2 != 0))
        throw std::runtime_error("fill column buffers must hold whole chunks of G x rows rows (and even LDS rows)");
    if (!e->attr) {   // dynamic LDS beyond 64 KB must be enabled per kernel
        (void)hipFuncSetAttribute((const void*)e->k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        e->attr = true;
    }
    const dim3 grid((n + per - 1) / per);
    hipLaunchKernelGGL(e->k, grid, dim3(64), lds, s, B, F, reads, n);
}

}  // namespace pbccs
