// pbccs_amd/csrc/arrow_kernels.hip -- HIP kernels of the Arrow polishing engine (gfx950).
//
//   k_fill        one lane per read: FillAlphaBeta with the flip-flop controller
//                 (SimpleRecursor.cpp:642-691) + alpha log-scale prefix + baseline score.
//   k_suffix      one workgroup per read: exact left-to-right beta log-scale suffix sums
//                 GetLogProdScales(k, J+1) for every k (ScaledMatrix-inl.hpp:69-77).
//   k_enumerate   one workgroup per ZMW: UniqueSingleBaseMutationEnumerator order
//                 (MutationEnumerator.cpp:114-145) + per-position offsets (for QVs).
//   k_score       one lane per (mutation, read): MutationScorer::ScoreMutation - Score()
//                 (MutationScorer.cpp:169-272) via register-only recompute sweeps.
//   k_reduce      one lane per mutation: ordered per-read sum with the fast-score break
//                 (MultiReadMutationScorer.cpp:338-368), favourable flag (> 0.04).
//   k_qv          one lane per template position: ConsensusQVs (Consensus-inl.hpp:274-295).
#include "arrow_device.hpp"
#include "arrow_kernels.hpp"

namespace pbccs {

// ------------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ Params params_for(const DevBatch& B, int z)
{
    Params P;
    P.ctx = B.zCtx + (long long)z * 9 * kCtxStride;
    P.prNot = B.prNot;
    P.prThird = B.prThird;
    P.sdn = B.sdn;
    return P;
}

__device__ __forceinline__ Band band_alpha(const DevBatch& B, int r)
{
    const long long cb = B.rColBase[r];
    Band m;
    m.range = B.aRange + cb;
    m.off = B.aOff + cb;
    m.ls = B.aLs + cb;
    m.val = B.valPool + B.rValA[r];
    m.cap = B.rValCap[r];
    return m;
}

__device__ __forceinline__ Band band_beta(const DevBatch& B, int r)
{
    const long long cb = B.rColBase[r];
    Band m;
    m.range = B.bRange + cb;
    m.off = B.bOff + cb;
    m.ls = B.bLs + cb;
    m.val = B.valPool + B.rValB[r];
    m.cap = B.rValCap[r];
    return m;
}

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

// ------------------------------------------------------------------------------------------------
// k_fill: FillAlphaBeta per read (MutationScorer ctor / Template(), MutationScorer.cpp:53-131)
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_fill(DevBatch B, const int* __restrict__ reads, int n)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
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
    const char* rd = B.seqPool + B.rSeqOff[r];
    const Params P = params_for(B, z);
    const Band a = band_alpha(B, r);
    const Band b = band_beta(B, r);

    unsigned long long cells = 0, passes = 0;
    long long ua = fill_alpha(tv, rd, I, a, nullptr, false, P);
    if (ua < 0) { B.rStatus[r] = kFillOverflow; return; }
    long long ub = fill_beta(tv, rd, I, b, a.range, false, P);
    if (ub < 0) { B.rStatus[r] = kFillOverflow; return; }
    cells += ua + ub;
    passes += 2;
    int flips = 0;
    const int maxSize = (int)(0.5 + kRebandFrac * (I + 1) * (J + 1));
    if (ua >= maxSize || ub >= maxSize) {
        ua = fill_alpha(tv, rd, I, a, b.range, true, P);
        if (ua < 0) { B.rStatus[r] = kFillOverflow; return; }
        ub = fill_beta(tv, rd, I, b, a.range, true, P);
        if (ub < 0) { B.rStatus[r] = kFillOverflow; return; }
        const long long ua2 = fill_alpha(tv, rd, I, a, b.range, true, P);
        if (ua2 < 0) { B.rStatus[r] = kFillOverflow; return; }
        cells += ua + ub + ua2;
        passes += 3;
        ua = ua2;
        flips += 3;
    }
    double av = log(alpha_at(a, I, J)) + sum_ls(a.ls, J + 1);
    double bv = log(beta_at(b, 0, 0)) + sum_ls(b.ls, J + 1);
    // NB: the reference does not re-evaluate alphaV/betaV inside this loop (SimpleRecursor.cpp:667-679).
    const bool mismatched = fabs(av - bv) > kAlphaBetaTol;
    while (mismatched && flips <= kMaxFlipFlops) {
        const long long u = (flips % 2 == 0) ? fill_alpha(tv, rd, I, a, b.range, true, P)
                                             : fill_beta(tv, rd, I, b, a.range, true, P);
        if (u < 0) { B.rStatus[r] = kFillOverflow; return; }
        cells += u;
        passes += 1;
        ++flips;
    }
    // alpha prefix sums (exactly GetLogProdScales(0, k) for every k) and its total
    double* pre = B.aPre + B.rColBase[r];
    double s = 0.0;
    pre[0] = 0.0;
    for (int k = 0; k <= J; ++k) {
        s = s + a.ls[k];
        pre[k + 1] = s;
    }
    av = log(alpha_at(a, I, J)) + s;
    bv = log(beta_at(b, 0, 0)) + sum_ls(b.ls, J + 1);
    const double mism = fabs(1.0 - av / bv);
    B.rFlips[r] = flips;
    B.rBaseline[r] = bv;
    B.rStatus[r] = (mism > kAlphaBetaTol) ? kFillMismatch : kFillOk;
    if (B.stats) {   // algorithmic: 8 B per stored cell + 16 B per column per fill pass
        atomicAdd(&B.stats[2 * kStatFill], cells);
        atomicAdd(&B.stats[2 * kStatFill + 1], 8ull * cells + 16ull * passes * (unsigned long long)(J + 1));
    }
}

// ------------------------------------------------------------------------------------------------
// k_suffix: bSuf[k] = accumulate(bLs[k..J], 0.0) for k in [0, J+1] (bSuf[J+1] = 0).  Each lane sums
// its own suffix left to right, reading the shared log-scale column from LDS (broadcast-friendly:
// lanes k, k+1, ... read consecutive words at every step).
// ------------------------------------------------------------------------------------------------
constexpr int kSuffixTile = 2048;

__global__ void __launch_bounds__(256) k_suffix(DevBatch B, const int* __restrict__ reads, int n)
{
    __shared__ double tile[kSuffixTile];
    const int r = reads[blockIdx.x];
    if (B.rStatus[r] != kFillOk && B.rStatus[r] != kFillMismatch) return;
    const long long cb = B.rColBase[r];
    const int J = window_view(B, r).Length();
    const double* ls = B.bLs + cb;
    double* suf = B.bSuf + cb;
    const int ncol = J + 1;
    for (int k0 = 0; k0 <= ncol; k0 += blockDim.x) {
        const int k = k0 + threadIdx.x;
        double s = 0.0;
        // walk the columns [k, ncol) in tiles staged through LDS
        for (int c0 = k0; c0 < ncol; c0 += kSuffixTile) {
            __syncthreads();
            for (int q = threadIdx.x; q < kSuffixTile && c0 + q < ncol; q += blockDim.x) tile[q] = ls[c0 + q];
            __syncthreads();
            const int lo = max(k, c0) - c0;
            const int hi = min(ncol - c0, kSuffixTile);
            if (k <= ncol)
                for (int q = lo; q < hi; ++q) s = s + tile[q];
        }
        if (k <= ncol) suf[k] = s;
    }
}

// ------------------------------------------------------------------------------------------------
// k_enumerate: unique single-base mutations of every position of a ZMW's template, in the
// reference's order; writes codes and per-position offsets (posOff has L+1 entries).
// Templates are validated ACGT on the host, so per-position counts are 8 at p == 0 and
// 6 + [T[p] != T[p-1]] afterwards.
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_enumerate(DevBatch B, const int* __restrict__ zmws,
                                                   const long long* __restrict__ mutBase,
                                                   const long long* __restrict__ posBase, int* __restrict__ codes,
                                                   int* __restrict__ posOff)
{
    __shared__ int waveSums[4];
    __shared__ int carry;
    const int z = zmws[blockIdx.x];
    const char* T = B.tplPool + B.zFwdOff[z];
    const int L = B.zLen[z];
    int* out = codes + mutBase[blockIdx.x];
    int* po = posOff + posBase[blockIdx.x];
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int p0 = 0; p0 < L; p0 += 256) {
        const int p = p0 + threadIdx.x;
        int cnt = 0;
        char cur = 0, prev = '-';
        if (p < L) {
            cur = T[p];
            prev = p > 0 ? T[p - 1] : '-';
            cnt = (p == 0) ? 8 : 6 + (cur != prev ? 1 : 0);
        }
        // block exclusive scan
        int incl = cnt;
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(incl, d, 64);
            if (lane >= d) incl += y;
        }
        if (lane == 63) waveSums[wid] = incl;
        __syncthreads();
        int waveOff = 0;
        for (int w = 0; w < wid; ++w) waveOff += waveSums[w];
        const int excl = carry + waveOff + incl - cnt;
        if (p < L) {
            po[p] = excl;
            int k = excl;
            for (int x = 0; x < 4; ++x)
                if (base_char(x) != cur) out[k++] = mut_code(p, kSub, x);
            for (int x = 0; x < 4; ++x)
                if (base_char(x) != prev) out[k++] = mut_code(p, kIns, x);
            if (cur != prev) out[k++] = mut_code(p, kDel, 0);
        }
        __syncthreads();
        if (threadIdx.x == 255) carry = excl + cnt;
        __syncthreads();
    }
    if (threadIdx.x == 0) po[L] = carry;
}

// ------------------------------------------------------------------------------------------------
// Mutation scoring
// ------------------------------------------------------------------------------------------------
struct ScoreCtx {
    const DevBatch* B;
    Params P;
    const char* rd;
    int I;
    int Jorig;   // unmutated window length (alpha/beta have Jorig + 1 columns)
    TplView tv;
    Band a, b;
    const double* aPre;
    const double* bSuf;
};

// ExtendAlpha (SimpleRecursor.cpp:373-487) over n <= 4 columns starting at `sc`, followed either by
// LinkAlphaBeta (:306-357, n == 2, middle case) or by the at-end read-out (MutationScorer.cpp:219-231).
// ext columns are never stored: sweep t recomputes columns 0..t-1 (scales known) and column t (its
// max = the FinishEditingColumn constant); a final sweep produces the link sum.  Every recomputation
// performs the same operations in the same order, so the values are bit-identical to a stored matrix.
__device__ double extend_alpha_score(const ScoreCtx& S, int sc, int n, bool link, int bc, int absc, TaskStat& st)
{
    const int I = S.I;
    const int Jv = S.tv.Length();
    int cb[kMaxExtCols], ce[kMaxExtCols], jj[kMaxExtCols];
    char cur[kMaxExtCols], nxt[kMaxExtCols];
    double pM[kMaxExtCols], pD[kMaxExtCols], cB[kMaxExtCols], cS3[kMaxExtCols];
#pragma unroll
    for (int c = 0; c < kMaxExtCols; ++c) {
        cb[c] = 0; ce[c] = 0; jj[c] = 0; cur[c] = 0; nxt[c] = 0;
        pM[c] = 0.0; pD[c] = 0.0; cB[c] = 0.0; cS3[c] = 0.0;
        if (c < n) {
            const int j = sc + c;
            jj[c] = j;
            int b, e;
            if (j < Jv) {
                const int2 r0 = S.a.range[j];
                b = r0.x; e = r0.y;
                if (j - 1 >= 0) { const int2 r1 = S.a.range[j - 1]; b = min(b, r1.x); e = max(e, r1.y); }
                if (j + 1 < Jv) { const int2 r2 = S.a.range[j + 1]; b = min(b, r2.x); e = max(e, r2.y); }
            } else {
                b = S.a.range[S.Jorig].x;
                e = I + 1;
            }
            cb[c] = b; ce[c] = e;
            char cbase; int cctx;
            S.tv.At(j - 1, cbase, cctx);
            cur[c] = cbase;
            const double* cp = S.P.P(cctx);
            cB[c] = cp[kB]; cS3[c] = cp[kS3];
            const int pctx = (j > 1) ? S.tv.Ctx(j - 2) : kCtxZero;
            pM[c] = S.P.P(pctx)[kM];
            pD[c] = S.P.P(pctx)[kD];
            if (j != Jv) nxt[c] = S.tv.Base(j);
        }
    }
    // alpha column sc-1 feeds ext column 0
    const int2 ar = S.a.range[sc - 1];
    const double* av = S.a.val + S.a.off[sc - 1] - ar.x;

    // link setup
    int lb = 0, le = 0;
    char linkBase = 0;
    double lM = 0.0, lD = 0.0;
    int2 br = make_int2(0, 0);
    const double* bv = nullptr;
    if (link) {
        lb = min(cb[0], cb[1]); le = max(ce[0], ce[1]);
        const int2 b0 = S.b.range[bc], b1 = S.b.range[bc + 1];
        lb = min(lb, min(b0.x, b1.x));
        le = max(le, max(b0.y, b1.y));
        linkBase = S.tv.Base(absc - 1);
        const int lctx = S.tv.Ctx(absc - 2);
        lM = S.P.P(lctx)[kM];
        lD = S.P.P(lctx)[kD];
        br = b0;
        bv = S.b.val + S.b.off[bc] + (b0.y - 1);   // bv[-i] = beta(i, bc)
    }

    double C[kMaxExtCols], ls[kMaxExtCols];
    bool scl[kMaxExtCols];
#pragma unroll
    for (int c = 0; c < kMaxExtCols; ++c) { C[c] = 0.0; ls[c] = 0.0; scl[c] = false; }
    double rawAtI = 0.0;
    double v = 0.0;
    const int nSweeps = link ? n + 1 : n;
    for (int t = 0; t < nSweeps; ++t) {
        const int top = min(t, n - 1);   // highest column computed in this sweep
        int lo, hi;
        if (t == n) { lo = lb; hi = le; }
        else {
            lo = cb[0]; hi = ce[0];
#pragma unroll
            for (int c = 1; c < kMaxExtCols; ++c)
                if (c <= top) { lo = min(lo, cb[c]); hi = max(hi, ce[c]); }
        }
        double rawPrev[kMaxExtCols], scPrev[kMaxExtCols];
#pragma unroll
        for (int c = 0; c < kMaxExtCols; ++c) { rawPrev[c] = 0.0; scPrev[c] = 0.0; }
        double Ct = 0.0;
        for (int i = lo; i < hi; ++i) {
            const double aD = (i - 1 >= ar.x && i - 1 < ar.y) ? av[i - 1] : 0.0;
            const double aL = (i >= ar.x && i < ar.y) ? av[i] : 0.0;
            const char rb = (i >= 1 && i - 1 < I) ? S.rd[i - 1] : (char)0;
            double rawCur[kMaxExtCols], scCur[kMaxExtCols];
#pragma unroll
            for (int c = 0; c < kMaxExtCols; ++c) {
                rawCur[c] = 0.0;
                scCur[c] = 0.0;
                if (c <= top) {
                    const int j = jj[c];
                    const double pd = (c == 0) ? aD : scPrev[c > 0 ? c - 1 : 0];
                    const double pl = (c == 0) ? aL : scCur[c > 0 ? c - 1 : 0];
                    double raw = 0.0;
                    const bool in = (i >= cb[c] && i < ce[c]);
                    if (in) {
                        double s;
                        if (i > 0 && j > 0) {
                            const double em = (rb == cur[c]) ? S.P.prNot : S.P.prThird;
                            double mv = 0.0;
                            if (i == 1 && j == 1) mv = em;
                            else if (i < I && j < Jv) mv = pd * pM[c] * em;
                            else if (i == I && j == Jv) mv = pd * em;
                            s = mv;
                        } else {
                            s = rawPrev[c];   // the reference's `score` carries over (never taken: i >= 1)
                        }
                        if (i > 1 && i < I && j != Jv) s = s + rawPrev[c] * (nxt[c] == rb ? cB[c] : cS3[c]);
                        if (j > 1 && j < Jv && i != I) s = s + pl * pD[c];
                        raw = s;
                    }
                    rawCur[c] = raw;
                    if (c < t) {
                        scCur[c] = in ? (scl[c] ? raw / C[c] : raw) : 0.0;
                    } else if (in) {   // c == t < n: the column whose scale this sweep determines
                        if (Ct < raw) Ct = raw;
                        if (i == I) rawAtI = raw;
                    }
                }
            }
            if (t == n) {
                const double s1 = scCur[1];
                if (i < I) {
                    const double mprob = lM * (S.rd[i] == linkBase ? S.P.prNot : S.P.prThird);
                    const double bn = (i + 1 >= br.x && i + 1 < br.y) ? bv[-(i + 1)] : 0.0;
                    v = v + s1 * mprob * bn;
                }
                const double bh = (i >= br.x && i < br.y) ? bv[-i] : 0.0;
                v = v + s1 * lD * bh;
            }
#pragma unroll
            for (int c = 0; c < kMaxExtCols; ++c) { rawPrev[c] = rawCur[c]; scPrev[c] = scCur[c]; }
        }
        if (t < n) {
#pragma unroll
            for (int c = 0; c < kMaxExtCols; ++c)
                if (c == t) {
                    C[c] = Ct;
                    scl[c] = (Ct != 0.0 && Ct != 1.0);
                    ls[c] = scl[c] ? log(Ct) : 0.0;
                }
        }
    }
    double E = 0.0;
#pragma unroll
    for (int c = 0; c < kMaxExtCols; ++c)
        if (c < n) {
            E = E + ls[c];
            st.cells += (unsigned long long)max(0, ce[c] - cb[c]);
        }
    st.bytes += 8ull * (unsigned long long)max(0, ar.y - ar.x) + 16ull * (unsigned long long)(n + 2);
    if (link) {
        st.cells += (unsigned long long)max(0, le - lb);
        st.bytes += 8ull * (unsigned long long)max(0, br.y - br.x) + 32ull;
        return ((log(v) + E) + S.bSuf[bc]) + S.aPre[sc];
    }
    // at-end read-out: ext(I, n-1)
    double lastC = 0.0, lastRange = 0.0;
    bool lastScl = false;
    int lastB = 0, lastE = 0;
#pragma unroll
    for (int c = 0; c < kMaxExtCols; ++c)
        if (c == n - 1) { lastC = C[c]; lastScl = scl[c]; lastB = cb[c]; lastE = ce[c]; }
    (void)lastRange;
    double extI = 0.0;
    if (I >= lastB && I < lastE) extI = lastScl ? rawAtI / lastC : rawAtI;
    return (log(extI) + S.aPre[sc]) + E;
}

// ExtendBeta (SimpleRecursor.cpp:509-628) back to column 0 for mutations near the template start,
// read out as in MutationScorer.cpp:233-245.  Columns are filled high to low, rows bottom-up.
__device__ double extend_beta_score(const ScoreCtx& S, int lastCol, int ld, TaskStat& st)
{
    const int I = S.I;
    const int Jv = S.tv.Length();
    const int nExt = ld + lastCol + 1;
    const int firstCol = -ld;
    const int lastExt = nExt - 1;
    int cb[kMaxExtCols], ce[kMaxExtCols], jj[kMaxExtCols], jpv[kMaxExtCols];
    char nxt[kMaxExtCols];
    double cM[kMaxExtCols], cD[kMaxExtCols], cB[kMaxExtCols], cS3[kMaxExtCols];
#pragma unroll
    for (int c = 0; c < kMaxExtCols; ++c) {
        cb[c] = 0; ce[c] = 0; jj[c] = 0; jpv[c] = 0; nxt[c] = 0;
        cM[c] = 0.0; cD[c] = 0.0; cB[c] = 0.0; cS3[c] = 0.0;
        if (c < nExt) {
            const int j = c + firstCol;
            const int jp = j + ld;
            jj[c] = j; jpv[c] = jp;
            int b, e;
            if (j < 0) {
                b = 0;
                e = S.b.range[0].y;
            } else {
                const int2 r0 = S.b.range[j];
                b = r0.x; e = r0.y;
                if (j - 1 >= 0) { const int2 r1 = S.b.range[j - 1]; b = min(b, r1.x); e = max(e, r1.y); }
                if (j + 1 < Jv) { const int2 r2 = S.b.range[j + 1]; b = min(b, r2.x); e = max(e, r2.y); }
            }
            cb[c] = b; ce[c] = e;
            nxt[c] = S.tv.Base(jp);
            const int cctx = (jp > 0) ? S.tv.Ctx(jp - 1) : kCtxZero;
            const double* cp = S.P.P(cctx);
            cM[c] = cp[kM]; cD[c] = cp[kD]; cB[c] = cp[kB]; cS3[c] = cp[kS3];
        }
    }
    // beta column lastCol + 1 feeds ext column lastExt
    const int2 br = S.b.range[lastCol + 1];
    const double* bv = S.b.val + S.b.off[lastCol + 1] + (br.y - 1);   // bv[-i] = beta(i, lastCol+1)

    double C[kMaxExtCols], ls[kMaxExtCols];
    bool scl[kMaxExtCols];
#pragma unroll
    for (int c = 0; c < kMaxExtCols; ++c) { C[c] = 0.0; ls[c] = 0.0; scl[c] = false; }
    double rawAt0 = 0.0;
    for (int t = lastExt; t >= 0; --t) {
        int lo = cb[lastExt], hi = ce[lastExt];
#pragma unroll
        for (int c = 0; c < kMaxExtCols; ++c)
            if (c >= t && c < nExt) { lo = min(lo, cb[c]); hi = max(hi, ce[c]); }
        double rawPrev[kMaxExtCols], scPrev[kMaxExtCols];   // values at row i+1
#pragma unroll
        for (int c = 0; c < kMaxExtCols; ++c) { rawPrev[c] = 0.0; scPrev[c] = 0.0; }
        double Ct = 0.0;
        for (int i = hi - 1; i >= lo; --i) {
            const double bN = (i + 1 >= br.x && i + 1 < br.y) ? bv[-(i + 1)] : 0.0;   // beta(i+1, lastCol+1)
            const double bH = (i >= br.x && i < br.y) ? bv[-i] : 0.0;                 // beta(i, lastCol+1)
            const char nb = (i < I) ? S.rd[i] : 'N';
            double rawCur[kMaxExtCols], scCur[kMaxExtCols];
#pragma unroll
            for (int c = 0; c < kMaxExtCols; ++c) { rawCur[c] = 0.0; scCur[c] = 0.0; }
#pragma unroll
            for (int cc = kMaxExtCols - 1; cc >= 0; --cc) {
                if (cc >= t && cc < nExt) {
                    const int j = jj[cc], jp = jpv[cc];
                    const double nxD = (cc == lastExt) ? bN : scPrev[cc + 1 < kMaxExtCols ? cc + 1 : cc];
                    const double nxH = (cc == lastExt) ? bH : scCur[cc + 1 < kMaxExtCols ? cc + 1 : cc];
                    const bool in = (i >= cb[cc] && i < ce[cc]);
                    double raw = 0.0;
                    if (in) {
                        const bool same = nb == nxt[cc];
                        double s = 0.0;
                        if (i < I && j < Jv) {
                            const double em = same ? S.P.prNot : S.P.prThird;
                            double mv = 0.0;
                            if ((i == I - 1 && jp == Jv - 1) || (i == 0 && j == firstCol)) mv = nxD * em;
                            else if (j > firstCol && i > 0) mv = nxD * cM[cc] * em;
                            s = 0.0 + mv;
                        }
                        if (i < I - 1 && i > 0 && j > firstCol) s = s + rawPrev[cc] * (same ? cB[cc] : cS3[cc]);
                        if (j < Jv - 1 && j > firstCol && i > 0) s = s + nxH * cD[cc];
                        raw = s;
                    }
                    rawCur[cc] = raw;
                    if (cc > t) {
                        scCur[cc] = in ? (scl[cc] ? raw / C[cc] : raw) : 0.0;
                    } else if (in) {
                        if (Ct < raw) Ct = raw;
                        if (i == 0) rawAt0 = raw;
                    }
                }
            }
#pragma unroll
            for (int c = 0; c < kMaxExtCols; ++c) { rawPrev[c] = rawCur[c]; scPrev[c] = scCur[c]; }
        }
#pragma unroll
        for (int c = 0; c < kMaxExtCols; ++c)
            if (c == t) {
                C[c] = Ct;
                scl[c] = (Ct != 0.0 && Ct != 1.0);
                ls[c] = scl[c] ? log(Ct) : 0.0;
            }
    }
    double E = 0.0;
#pragma unroll
    for (int c = 0; c < kMaxExtCols; ++c)
        if (c < nExt) {
            E = E + ls[c];
            st.cells += (unsigned long long)max(0, ce[c] - cb[c]);
        }
    st.bytes += 8ull * (unsigned long long)max(0, br.y - br.x) + 16ull * (unsigned long long)(nExt + 2);
    const double ext00 = (0 >= cb[0] && 0 < ce[0]) ? (scl[0] ? rawAt0 / C[0] : rawAt0) : 0.0;
    return (log(ext00) + S.bSuf[lastCol + 1]) + E;
}

__device__ __forceinline__ bool read_scores(int ts, int te, int type, int ms, int me)
{
    if (type == kIns) return ts <= me && ms <= te;   // MultiReadMutationScorer.cpp:70-80
    return ts < me && ms < te;
}

// MutationScorer::ScoreMutation(OrientedMutation(read, m)) - MutationScorer::Score() for one read.
__device__ double score_mutation(const DevBatch& B, int r, int code, const ScoreScratch& scratch, TaskStat& st)
{
    const int z = B.rZmw[r];
    const int L = B.zLen[z];
    const int ts = B.rTs[r], te = B.rTe[r];
    const int type = mut_type(code);
    const int pos = mut_pos(code);
    const int base = mut_base(code);
    const int mStart = pos;
    const int mEnd = (type == kIns) ? pos : pos + 1;
    const int ld = (type == kIns) ? 1 : (type == kDel ? -1 : 0);

    ScoreCtx S;
    S.B = &B;
    S.P = params_for(B, z);
    S.rd = B.seqPool + B.rSeqOff[r];
    S.I = B.rLen[r];
    S.Jorig = te - ts;
    S.a = band_alpha(B, r);
    S.b = band_beta(B, r);
    const long long cbase = B.rColBase[r];
    S.aPre = B.aPre + cbase;
    S.bSuf = B.bSuf + cbase;
    S.tv = window_view(B, r);
    int os, oe;
    if (B.rStrand[r] == kFwd) {
        S.tv.vm = make_virtual(S.tv.T, L, type, mStart, base_char(base));
        os = mStart - ts;
        oe = mEnd - ts;
    } else {
        S.tv.vm = make_virtual(S.tv.T, L, type, L - mEnd, base_char(complement_index(base)));
        os = te - mEnd;
        oe = te - mStart;
    }
    const int J = S.Jorig;
    const int betaLinkCol = 1 + oe;
    const int absLinkCol = 1 + oe + ld;
    const bool atBegin = os < 3;
    const bool atEnd = oe > (J + 1) - 1 - 2;
    double score;
    if (!atBegin && !atEnd) {
        const int sc = (type == kDel) ? os - 1 : os;
        score = extend_alpha_score(S, sc, 2, true, betaLinkCol, absLinkCol, st);
    } else if (!atBegin && atEnd) {
        const int sc = os - 1;
        const int n = S.tv.Length() - sc + 1;
        score = extend_alpha_score(S, sc, n, false, 0, 0, st);
    } else if (atBegin && !atEnd) {
        score = extend_beta_score(S, oe, ld, st);
    } else {
        // whole fill of the virtually mutated window (MutationScorer.cpp:246-266); tiny windows only
        const int Jv = S.tv.Length();
        const long long ncol = Jv + 1;
        const long long need = ncol * (long long)(S.I + 1) + 4 * ncol + 16;
        const unsigned long long at = atomicAdd(scratch.top, (unsigned long long)need);
        if (at + need > scratch.cap) {
            atomicOr(scratch.overflow, 1);
            return __longlong_as_double(0x7ff8000000000001LL);
        }
        double* base0 = scratch.pool + at;
        Band m;
        m.ls = base0;
        m.range = reinterpret_cast<int2*>(base0 + ncol);
        m.off = reinterpret_cast<int*>(base0 + 2 * ncol);
        m.val = base0 + 4 * ncol;
        m.cap = ncol * (long long)(S.I + 1);
        const long long u = fill_alpha(S.tv, S.rd, S.I, m, nullptr, false, S.P);
        st.cells += (unsigned long long)max(0LL, u);
        st.bytes += 8ull * (unsigned long long)max(0LL, u) + 16ull * (unsigned long long)ncol;
        score = log(alpha_at(m, S.I, Jv)) + sum_ls(m.ls, Jv + 1);
    }
    return score - B.rBaseline[r];
}

// One wave per (work item, read, 64-mutation chunk); lanes take consecutive mutations of one read so
// that a wave walks adjacent template positions of a single read's bands (L1/L2 reuse).
__global__ void __launch_bounds__(256) k_score(DevBatch B, ScoreWork W, ScoreScratch scratch)
{
    const long long wave = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (wave >= W.waveStart[W.nWork]) return;
    // binary search of the work item (wave-uniform)
    int lo = 0, hi = W.nWork;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (W.waveStart[mid] <= wave) lo = mid; else hi = mid;
    }
    const int k = lo;
    const int z = W.zmw[k];
    const int M = W.nMut[k];
    const int chunks = (M + 63) >> 6;
    const long long local = wave - W.waveStart[k];
    const int rr = (int)(local / chunks);
    const int m = (int)(local % chunks) * 64 + lane;
    TaskStat st;
    if (m < M) {
        const int r = B.zReadBegin[z] + rr;
        const int code = W.codes[W.mutBase[k] + m];
        double d = 0.0;
        const int type = mut_type(code), pos = mut_pos(code);
        const int me = (type == kIns) ? pos : pos + 1;
        if (B.rActive[r] && read_scores(B.rTs[r], B.rTe[r], type, pos, me)) d = score_mutation(B, r, code, scratch, st);
        W.delta[W.deltaBase[k] + (long long)rr * M + m] = d;
    }
    if (B.stats) {   // wave-reduce, one atomic per wave
        unsigned long long c = st.cells, b = st.bytes;
        for (int o = 32; o > 0; o >>= 1) {
            c += __shfl_xor(c, o, 64);
            b += __shfl_xor(b, o, 64);
        }
        if (lane == 0) {
            atomicAdd(&B.stats[2 * kStatScore], c);
            atomicAdd(&B.stats[2 * kStatScore + 1], b);
        }
    }
}

// Ordered reduction over reads with the fast-score break (MultiReadMutationScorer.cpp:352-362).
__global__ void __launch_bounds__(256) k_reduce(DevBatch B, ScoreWork W, double fastThr, double* __restrict__ score,
                                                unsigned char* __restrict__ fav)
{
    const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= W.mutStart[W.nWork]) return;
    int lo = 0, hi = W.nWork;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (W.mutStart[mid] <= g) lo = mid; else hi = mid;
    }
    const int k = lo;
    const int z = W.zmw[k];
    const int M = W.nMut[k];
    const int m = (int)(g - W.mutStart[k]);
    const int code = W.codes[W.mutBase[k] + m];
    const int type = mut_type(code), pos = mut_pos(code);
    const int me = (type == kIns) ? pos : pos + 1;
    const int rb = B.zReadBegin[z], nr = B.zNReads[z];
    const double* d = W.delta + W.deltaBase[k] + m;
    double sum = 0.0;
    for (int rr = 0; rr < nr; ++rr) {
        const int r = rb + rr;
        if (B.rActive[r] && read_scores(B.rTs[r], B.rTe[r], type, pos, me)) sum += d[(long long)rr * M];
        if (sum < fastThr) break;
    }
    score[W.mutBase[k] + m] = sum;
    fav[W.mutBase[k] + m] = (sum > 0.04) ? 1 : 0;   // MIN_FAVORABLE_SCOREDIFF, MultiReadMutationScorer.cpp:56
}

// ConsensusQVs + ProbabilityToQV (Consensus-inl.hpp:130-138, 274-295).
__global__ void __launch_bounds__(256) k_qv(DevBatch B, ScoreWork W, const long long* __restrict__ posBase,
                                            const int* __restrict__ posOff, const double* __restrict__ score,
                                            const long long* __restrict__ qvBase, int* __restrict__ qv)
{
    const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= W.posStart[W.nWork]) return;
    int lo = 0, hi = W.nWork;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (W.posStart[mid] <= g) lo = mid; else hi = mid;
    }
    const int k = lo;
    const int p = (int)(g - W.posStart[k]);
    const int* po = posOff + posBase[k];
    const double* sc = score + W.mutBase[k];
    double sum = 0.0;
    for (int m = po[p]; m < po[p + 1]; ++m) {
        const double s = sc[m];
        if (s < 0.0) sum += exp(s);
    }
    double prob = 1.0 - 1.0 / (1.0 + sum);
    if (prob == 0.0) prob = 2.2250738585072014e-308;   // std::numeric_limits<double>::min()
    qv[qvBase[k] + p] = (int)round(-10.0 * log10(prob));
}

// ------------------------------------------------------------------------------------------------
// launch wrappers (host side)
// ------------------------------------------------------------------------------------------------
void launch_fill(const DevBatch& B, const int* reads, int n, hipStream_t s)
{
    if (n <= 0) return;
    hipLaunchKernelGGL(k_fill, dim3((n + 63) / 64), dim3(64), 0, s, B, reads, n);
}

void launch_suffix(const DevBatch& B, const int* reads, int n, hipStream_t s)
{
    if (n <= 0) return;
    hipLaunchKernelGGL(k_suffix, dim3(n), dim3(256), 0, s, B, reads, n);
}

void launch_enumerate(const DevBatch& B, const int* zmws, int n, const long long* mutBase, const long long* posBase,
                      int* codes, int* posOff, hipStream_t s)
{
    if (n <= 0) return;
    hipLaunchKernelGGL(k_enumerate, dim3(n), dim3(256), 0, s, B, zmws, mutBase, posBase, codes, posOff);
}

void launch_score(const DevBatch& B, const ScoreWork& W, long long nWaves, const ScoreScratch& scratch, hipStream_t s)
{
    if (nWaves <= 0) return;
    const long long blocks = (nWaves + 3) / 4;
    hipLaunchKernelGGL(k_score, dim3((unsigned)blocks), dim3(256), 0, s, B, W, scratch);
}

void launch_reduce(const DevBatch& B, const ScoreWork& W, long long nMut, double fastThr, double* score,
                   unsigned char* fav, hipStream_t s)
{
    if (nMut <= 0) return;
    hipLaunchKernelGGL(k_reduce, dim3((unsigned)((nMut + 255) / 256)), dim3(256), 0, s, B, W, fastThr, score, fav);
}

void launch_qv(const DevBatch& B, const ScoreWork& W, long long nPos, const long long* posBase, const int* posOff,
               const double* score, const long long* qvBase, int* qv, hipStream_t s)
{
    if (nPos <= 0) return;
    hipLaunchKernelGGL(k_qv, dim3((unsigned)((nPos + 255) / 256)), dim3(256), 0, s, B, W, posBase, posOff, score,
                       qvBase, qv);
}

}  // namespace pbccs
