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
#include "coop_chain.hpp"

#include <climits>

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


// ------------------------------------------------------------------------------------------------
// k_fill: FillAlphaBeta per read (MutationScorer ctor / Template(), MutationScorer.cpp:53-131), one
// lane per read, into the lane-interleaved scratch of its 64-read group; k_compact then moves the
// final alpha/beta bands into each read's compact layout.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ LaneBand scratch_band(const FillScratch& F, int g, int l, int which)
{
    const long long gm = 2LL * g + which;
    LaneBand m;
    m.range = F.range + gm * F.capCols * 64 + l;
    m.off = F.off + gm * F.capCols * 64 + l;
    m.ls = F.ls + gm * F.capCols * 64 + l;
    m.val = F.val + gm * F.capSlots * 64 + l;
    m.cap = F.capSlots;
    return m;
}

__global__ void __launch_bounds__(64) k_fill(DevBatch B, FillScratch F, const int* __restrict__ reads, int n)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int g = t >> 6, l = t & 63;
    const long long tStart = F.trace ? (long long)wall_clock64() : 0;
    const int r = reads[t];
    const int z = B.rZmw[r];
    const int I = B.rLen[r];
    const TplView tv = window_view(B, r);
    const int J = tv.Length();
    if (I < 1 || J < 1 || J + 2 > F.capCols) {
        B.rStatus[r] = (I < 1 || J < 1) ? kFillBadInput : kFillOverflow;
        return;
    }
    const char* rd = B.seqPool + B.rSeqOff[r];
    const Params P = params_for(B, z);
    const LaneBand a = scratch_band(F, g, l, 0);
    const LaneBand b = scratch_band(F, g, l, 1);

    unsigned long long cells = 0, passes = 0;
    long long ua = fill_alpha(tv, rd, I, a, (const LaneBand*)nullptr, false, P);
    if (ua < 0) { B.rStatus[r] = kFillOverflow; return; }
    long long ub = fill_beta(tv, rd, I, b, &a, false, P);
    if (ub < 0) { B.rStatus[r] = kFillOverflow; return; }
    cells += ua + ub;
    passes += 2;
    int flips = 0;
    const int maxSize = (int)(0.5 + kRebandFrac * (I + 1) * (J + 1));
    if (ua >= maxSize || ub >= maxSize) {
        const long long a1 = fill_alpha(tv, rd, I, a, &b, true, P);
        if (a1 < 0) { B.rStatus[r] = kFillOverflow; return; }
        ub = fill_beta(tv, rd, I, b, &a, true, P);
        if (ub < 0) { B.rStatus[r] = kFillOverflow; return; }
        ua = fill_alpha(tv, rd, I, a, &b, true, P);
        if (ua < 0) { B.rStatus[r] = kFillOverflow; return; }
        cells += a1 + ub + ua;
        passes += 3;
        flips += 3;
    }
    double av = log(alpha_at(a, I, J)) + sum_ls(a, J + 1);
    double bv = log(beta_at(b, 0, 0)) + sum_ls(b, J + 1);
    // NB: the reference does not re-evaluate alphaV/betaV inside this loop (SimpleRecursor.cpp:667-679).
    const bool mismatched = fabs(av - bv) > kAlphaBetaTol;
    while (mismatched && flips <= kMaxFlipFlops) {
        if (flips % 2 == 0) {
            ua = fill_alpha(tv, rd, I, a, &b, true, P);
            if (ua < 0) { B.rStatus[r] = kFillOverflow; return; }
            cells += ua;
        } else {
            ub = fill_beta(tv, rd, I, b, &a, true, P);
            if (ub < 0) { B.rStatus[r] = kFillOverflow; return; }
            cells += ub;
        }
        passes += 1;
        ++flips;
    }
    // alpha prefix sums (exactly GetLogProdScales(0, k) for every k) and its total
    double* pre = F.pre + (long long)g * (F.capCols + 1) * 64 + l;
    double s = 0.0;
    pre[0] = 0.0;
    for (int k = 0; k <= J; ++k) {
        s = s + a.L(k);
        pre[(long long)(k + 1) * 64] = s;
    }
    av = log(alpha_at(a, I, J)) + s;
    bv = log(beta_at(b, 0, 0)) + sum_ls(b, J + 1);
    const double mism = fabs(1.0 - av / bv);
    B.rFlips[r] = flips;
    B.rBaseline[r] = bv;
    B.rDev[r] = 0.0;   // exact path
    F.usedA[r] = (int)ua;
    F.usedB[r] = (int)ub;
    B.rStatus[r] = (mism > kAlphaBetaTol) ? kFillMismatch : kFillOk;
    if (F.trace) {
        long long* tr = F.trace + 8LL * t;
        tr[0] = tStart;
        tr[1] = (long long)wall_clock64();
        tr[2] = (long long)cells;
        tr[3] = (long long)passes;
        tr[4] = J;
        tr[5] = I;
        tr[6] = ua;
        tr[7] = ub;
    }
    if (B.stats) {   // algorithmic: 8 B per stored cell + 16 B per column per fill pass
        atomicAdd(&B.stats[2 * kStatFillTall], cells);   // the lane-serial fallback takes only very tall reads
        atomicAdd(&B.stats[2 * kStatFillTall + 1], 8ull * cells + 16ull * passes * (unsigned long long)(J + 1));
    }
}

// ------------------------------------------------------------------------------------------------
// k_compact: one workgroup per 64-read fill group.  Transposes the group's [slot][lane] scratch through
// LDS into each read's contiguous band (coalesced 512 B rows in, 512 B per-read runs out), and the
// [column][lane] metadata into the per-read column slots the scoring kernels index.
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_compact(DevBatch B, FillScratch F, const int* __restrict__ reads, int n)
{
    __shared__ double tile[64][65];
    __shared__ int rid[64], uA[64], uB[64], ncol[64], ok[64];
    __shared__ long long dA[64], dB[64], cb[64];
    const int g = blockIdx.x;
    const int t = threadIdx.x;
    if (t < 64) {
        const int idx = g * 64 + t;
        int r = -1, good = 0;
        if (idx < n) {
            r = reads[idx];
            good = (B.rStatus[r] == kFillOk || B.rStatus[r] == kFillMismatch) ? 1 : 0;
        }
        rid[t] = r;
        ok[t] = good;
        uA[t] = good ? F.usedA[r] : 0;
        uB[t] = good ? F.usedB[r] : 0;
        ncol[t] = good ? window_view(B, r).Length() + 1 : 0;
        dA[t] = good ? B.rValA[r] : 0;
        dB[t] = good ? B.rValB[r] : 0;
        cb[t] = good ? B.rColBase[r] : 0;
    }
    __syncthreads();
    int maxA = 0, maxB = 0, maxC = 0;
    for (int q = 0; q < 64; ++q) {
        maxA = max(maxA, uA[q]);
        maxB = max(maxB, uB[q]);
        maxC = max(maxC, ncol[q]);
    }
    const int w = t >> 6, ln = t & 63;
    // values: alpha then beta
    for (int which = 0; which < 2; ++which) {
        const int maxU = which ? maxB : maxA;
        const double* src = F.val + (2LL * g + which) * F.capSlots * 64;
        for (int s0 = 0; s0 < maxU; s0 += 64) {
            for (int q = w; q < 64; q += 4) {
                const int slot = s0 + q;
                tile[q][ln] = (slot < maxU) ? src[(long long)slot * 64 + ln] : 0.0;
            }
            __syncthreads();
            for (int q = w; q < 64; q += 4) {   // q = read (lane) of the group, ln = slot within the tile
                const int used = which ? uB[q] : uA[q];
                const int slot = s0 + ln;
                if (ok[q] && slot < used) B.valPool[(which ? dB[q] : dA[q]) + slot] = tile[ln][q];
            }
            __syncthreads();
        }
    }
    // column metadata: ranges, offsets, log-scales of both matrices, and the alpha prefix (J+2 entries)
    for (int c0 = 0; c0 < maxC + 1; c0 += 64) {
        for (int which = 0; which < 2; ++which) {
            const long long gm = (2LL * g + which) * F.capCols * 64;
            // ls (double) through the tile
            for (int q = w; q < 64; q += 4) {
                const int c = c0 + q;
                tile[q][ln] = (c < maxC) ? F.ls[gm + (long long)c * 64 + ln] : 0.0;
            }
            __syncthreads();
            for (int q = w; q < 64; q += 4) {
                const int c = c0 + ln;
                if (ok[q] && c < ncol[q]) (which ? B.bLs : B.aLs)[cb[q] + c] = tile[ln][q];
            }
            __syncthreads();
            // ranges and offsets packed into the tile as raw bits
            for (int q = w; q < 64; q += 4) {
                const int c = c0 + q;
                const int2 rg = (c < maxC) ? F.range[gm + (long long)c * 64 + ln] : make_int2(0, 0);
                tile[q][ln] = __longlong_as_double((long long)(((unsigned long long)(unsigned)rg.y << 32) | (unsigned)rg.x));
            }
            __syncthreads();
            for (int q = w; q < 64; q += 4) {
                const int c = c0 + ln;
                if (ok[q] && c < ncol[q]) {
                    const long long bits = __double_as_longlong(tile[ln][q]);
                    (which ? B.bRange : B.aRange)[cb[q] + c] = make_int2((int)(bits & 0xffffffff), (int)(bits >> 32));
                }
            }
            __syncthreads();
            for (int q = w; q < 64; q += 4) {
                const int c = c0 + q;
                tile[q][ln] = __longlong_as_double((c < maxC) ? (long long)F.off[gm + (long long)c * 64 + ln] : 0LL);
            }
            __syncthreads();
            for (int q = w; q < 64; q += 4) {
                const int c = c0 + ln;
                if (ok[q] && c < ncol[q]) (which ? B.bOff : B.aOff)[cb[q] + c] = (int)__double_as_longlong(tile[ln][q]);
            }
            __syncthreads();
        }
        // alpha prefix: J+2 entries (columns 0..J+1)
        const double* pre = F.pre + (long long)g * (F.capCols + 1) * 64;
        for (int q = w; q < 64; q += 4) {
            const int c = c0 + q;
            tile[q][ln] = (c < maxC + 1) ? pre[(long long)c * 64 + ln] : 0.0;
        }
        __syncthreads();
        for (int q = w; q < 64; q += 4) {
            const int c = c0 + ln;
            if (ok[q] && c < ncol[q] + 1) B.aPre[cb[q] + c] = tile[ln][q];
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------------
// k_suffix: bSuf[k] = accumulate(bLs[k..J], 0.0) for k in [0, J+1] (bSuf[J+1] = 0), and with
// withPrefix the alpha prefixes aPre (the cooperative fill leaves them to this kernel).  Every lane sums
// its own k left to right (the reference's order, so no sharing between k is exact).  A wave owns 64
// consecutive k and walks the log-scale column in wave-uniform order: each LDS read is a broadcast, the
// 64 columns next to the wave's own k are added under a per-lane predicate (the lane's first add is
// 0.0 + ls[k], as in the reference), and every other column is added by all lanes with 8 reads in flight.
// ------------------------------------------------------------------------------------------------
constexpr int kSuffixTile = 2048;

__device__ __forceinline__ double add8(double s, const double* __restrict__ t)
{
    double v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = t[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) s = s + v[i];
    return s;
}

__device__ __forceinline__ void k_suffix_body(DevBatch B, const int* __restrict__ reads, int n, int withPrefix)
{
    __shared__ double tile[kSuffixTile];
    const int r = reads[blockIdx.x];
    if (B.rStatus[r] != kFillOk && B.rStatus[r] != kFillMismatch) return;
    const long long cb = B.rColBase[r];
    const int J = window_view(B, r).Length();
    const double* ls = B.bLs + cb;
    double* suf = B.bSuf + cb;
    const int ncol = J + 1;
    const int lane = threadIdx.x & 63;
    const int wbase = threadIdx.x & ~63;
    for (int k0 = 0; k0 <= ncol; k0 += blockDim.x) {
        const int kb = k0 + wbase;   // the wave's first k
        const int k = kb + lane;
        double s = 0.0;
        for (int c0 = k0; c0 < ncol; c0 += kSuffixTile) {
            __syncthreads();
            for (int q = threadIdx.x; q < kSuffixTile && c0 + q < ncol; q += blockDim.x) tile[q] = ls[c0 + q];
            __syncthreads();
            const int hi = min(ncol - c0, kSuffixTile);
            int q = max(kb - c0, 0);
            const int headEnd = min(hi, kb + 64 - c0);   // columns [kb, kb + 64): lane k starts at k
            for (; q < headEnd; ++q) {
                const double v = tile[q];
                if (c0 + q >= k) s = s + v;
            }
            for (; q + 8 <= hi; q += 8) s = add8(s, tile + q);
            for (; q < hi; ++q) s = s + tile[q];
        }
        if (k <= ncol) suf[k] = s;
    }
    if (!withPrefix) return;
    // aPre[k] = accumulate(aLs[0..k), 0.0) for k in [0, J+1] (GetLogProdScales(0, k)): every prefix is a partial sum
    // of the one left-to-right accumulation, so one thread's running sum gives them all with the reference's
    // roundings (J adds, instead of a separate sum per k), loads batched 8 at a time off the add chain
    if (threadIdx.x != 0) return;
    const double* als = B.aLs + cb;
    double* pre = B.aPre + cb;
    double run = 0.0;
    pre[0] = 0.0;
    int k = 0;
    for (; k + 8 <= ncol; k += 8) {
        double v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = als[k + q];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            run = run + v[q];
            pre[k + q + 1] = run;
        }
    }
    for (; k < ncol; ++k) {
        run = run + als[k];
        pre[k + 1] = run;
    }
}
__global__ void __launch_bounds__(256) k_suffix(DevBatch B, const int* __restrict__ reads, int n, int withPrefix)
{
    const long long wt0 = wave_t0(B.stats);
    k_suffix_body(B, reads, n, withPrefix);
    wave_ticks(B.stats, kWaveSuffix, wt0);
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

// ------------------------------------------------------------------------------------------------
// Middle-case scoring (the ~99% case: 3 <= start, end <= J-2): ExtendAlpha over 2 columns + LinkAlphaBeta
// (MutationScorer.cpp:193-218, SimpleRecursor.cpp:306-357 / :373-487), specialised.  In this case
// absLinkCol == sc + 2 for every mutation type, j0 + 2 < Jv, and every guarded branch of the generic
// ExtendAlpha resolves statically except the per-row ones kept below.
//   av: alpha(i, sc-1) = av[i] for i in ar;  bv: beta(i, bc) = bv[-i] for i in br;  rdp[i] = read base i.
// The pointers address either the wave's LDS stage or HBM (oversized bands).
// ------------------------------------------------------------------------------------------------
struct MidGeom {
    int b0, e0, b1, e1;   // ext column row ranges
    int lb, le;           // link row range
};

__device__ __forceinline__ MidGeom middle_geometry(const Band& a, const Band& b, int sc, int bc)
{
    MidGeom g;
    const int2 r0 = a.range[sc - 1], r1 = a.range[sc], r2 = a.range[sc + 1], r3 = a.range[sc + 2];
    g.b0 = min(min(r1.x, r0.x), r2.x);
    g.e0 = max(max(r1.y, r0.y), r2.y);
    g.b1 = min(min(r2.x, r1.x), r3.x);
    g.e1 = max(max(r2.y, r1.y), r3.y);
    const int2 q0 = b.range[bc], q1 = b.range[bc + 1];
    g.lb = min(min(g.b0, g.b1), min(q0.x, q1.x));
    g.le = max(max(g.e0, g.e1), max(q0.y, q1.y));
    return g;
}

__device__ __forceinline__ double score_middle(const ScoreCtx& S, int sc, int bc, const MidGeom& g,
                                               const double* __restrict__ av, int2 ar,
                                               const double* __restrict__ bv, int2 br,
                                               const char* __restrict__ rdp, TaskStat& st)
{
    const int I = S.I;
    // template positions sc-2 .. sc+1 under the virtual mutation
    char t0, t1, t2, t3;
    int x0, x1, x2, x3;
    S.tv.At(sc - 2, t0, x0);
    S.tv.At(sc - 1, t1, x1);
    S.tv.At(sc, t2, x2);
    S.tv.At(sc + 1, t3, x3);
    (void)t0;
    const double* P0 = S.P.P(sc > 1 ? x0 : kCtxZero);
    const double* P1 = S.P.P(x1);
    const double* P2 = S.P.P(x2);
    // ext column 0 (j = sc):   cur = pos sc-1, prev = pos sc-2, next base = pos sc
    const double pM0 = P0[kM], pD0 = P0[kD], cB0 = P1[kB], cS0 = P1[kS3];
    // ext column 1 (j = sc+1): cur = pos sc, prev = pos sc-1, next base = pos sc+1
    const double pM1 = P1[kM], pD1 = P1[kD], cB1 = P2[kB], cS1 = P2[kS3];
    // link (absLinkCol = sc+2): cur base = pos sc+1, prev params = pos sc
    const double lM = P2[kM], lD = P2[kD];
    const double pn = S.P.prNot, p3 = S.P.prThird;

#define PB_ALPHA(i) (((i) >= ar.x && (i) < ar.y) ? av[(i)] : 0.0)
#define PB_BETA(i) (((i) >= br.x && (i) < br.y) ? bv[-(i)] : 0.0)
    // one ext cell (ExtendAlpha :445-483) with j in (1, Jv): only the row conditions remain
#define PB_CELL(out, i, rb, curB, nxtB, pM, pD, cB, cS, pd, pl, rawPrev)                    \
    {                                                                                     \
        const double em_ = ((rb) == (curB)) ? pn : p3;                                    \
        double s_ = ((i) > 0) ? (((i) < I) ? (pd) * (pM) * em_ : 0.0) : (rawPrev);        \
        if ((i) > 1 && (i) < I) s_ = s_ + (rawPrev) * (((nxtB) == (rb)) ? (cB) : (cS));   \
        if ((i) != I) s_ = s_ + (pl) * (pD);                                              \
        out = s_;                                                                         \
    }

    // sweep 1: column 0 raw values -> its FinishEditingColumn constant C0
    double C0 = 0.0;
    {
        double aD = PB_ALPHA(g.b0 - 1), raw = 0.0;
        for (int i = g.b0; i < g.e0; ++i) {
            const double aL = PB_ALPHA(i);
            const char rb = rdp[i - 1];
            double v;
            PB_CELL(v, i, rb, t1, t2, pM0, pD0, cB0, cS0, aD, aL, raw);
            raw = v;
            if (C0 < v) C0 = v;
            aD = aL;
        }
    }
    const bool s0 = (C0 != 0.0 && C0 != 1.0);
    // sweep 2: column 0 scaled, column 1 raw -> C1
    const int u0 = min(g.b0, g.b1), u1 = max(g.e0, g.e1);
    double C1 = 0.0;
    {
        double aD = PB_ALPHA(u0 - 1), raw0 = 0.0, raw1 = 0.0, sc0p = 0.0;
        for (int i = u0; i < u1; ++i) {
            const double aL = PB_ALPHA(i);
            const char rb = rdp[i - 1];
            double v0 = 0.0, v1 = 0.0, sc0 = 0.0;
            if (i >= g.b0 && i < g.e0) {
                PB_CELL(v0, i, rb, t1, t2, pM0, pD0, cB0, cS0, aD, aL, raw0);
                sc0 = s0 ? v0 / C0 : v0;
            }
            if (i >= g.b1 && i < g.e1) {
                PB_CELL(v1, i, rb, t2, t3, pM1, pD1, cB1, cS1, sc0p, sc0, raw1);
                if (C1 < v1) C1 = v1;
            }
            raw0 = v0;
            raw1 = v1;
            sc0p = sc0;
            aD = aL;
        }
    }
    const bool s1 = (C1 != 0.0 && C1 != 1.0);
    // sweep 3: both columns scaled + LinkAlphaBeta over the union of the four used ranges
    double v = 0.0;
    {
        double aD = PB_ALPHA(g.lb - 1), raw0 = 0.0, raw1 = 0.0, sc0p = 0.0;
        double bH = PB_BETA(g.lb);
        for (int i = g.lb; i < g.le; ++i) {
            const double aL = PB_ALPHA(i);
            const double bN = PB_BETA(i + 1);
            const char rb = (i >= 1) ? rdp[i - 1] : (char)0;
            double v0 = 0.0, v1 = 0.0, sc0 = 0.0, sc1 = 0.0;
            if (i >= g.b0 && i < g.e0) {
                PB_CELL(v0, i, rb, t1, t2, pM0, pD0, cB0, cS0, aD, aL, raw0);
                sc0 = s0 ? v0 / C0 : v0;
            }
            if (i >= g.b1 && i < g.e1) {
                PB_CELL(v1, i, rb, t2, t3, pM1, pD1, cB1, cS1, sc0p, sc0, raw1);
                sc1 = s1 ? v1 / C1 : v1;
            }
            if (i < I) {
                const double mprob = lM * ((rdp[i] == t3) ? pn : p3);
                v = v + sc1 * mprob * bN;
            }
            v = v + sc1 * lD * bH;
            raw0 = v0;
            raw1 = v1;
            sc0p = sc0;
            aD = aL;
            bH = bN;
        }
    }
#undef PB_CELL
#undef PB_BETA
#undef PB_ALPHA
    const double E = (0.0 + (s0 ? log(C0) : 0.0)) + (s1 ? log(C1) : 0.0);
    st.cells += (unsigned long long)(max(0, g.e0 - g.b0) + max(0, g.e1 - g.b1) + max(0, g.le - g.lb));
    st.bytes += 8ull * (unsigned long long)(max(0, ar.y - ar.x) + max(0, br.y - br.x)) + 16ull * 6ull;
    return ((log(v) + E) + S.bSuf[bc]) + S.aPre[sc];
}

// ScoreCtx + oriented mutation for read r (OrientedMutation, MultiReadMutationScorer.cpp:93-139;
// the virtual mutation of MultiReadMutationScorer::Score, :338-348).
struct Oriented {
    int os, oe, ld, type;
};

__device__ __forceinline__ Oriented setup_score(const DevBatch& B, int r, int code, ScoreCtx& S)
{
    const int z = B.rZmw[r];
    const int L = B.zLen[z];
    const int ts = B.rTs[r], te = B.rTe[r];
    Oriented o;
    o.type = mut_type(code);
    const int pos = mut_pos(code);
    const int base = mut_base(code);
    const int mEnd = (o.type == kIns) ? pos : pos + 1;
    o.ld = (o.type == kIns) ? 1 : (o.type == kDel ? -1 : 0);
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
    if (B.rStrand[r] == kFwd) {
        S.tv.vm = make_virtual(S.tv.T, L, o.type, pos, base_char(base));
        o.os = pos - ts;
        o.oe = mEnd - ts;
    } else {
        S.tv.vm = make_virtual(S.tv.T, L, o.type, L - mEnd, base_char(complement_index(base)));
        o.os = te - mEnd;
        o.oe = te - pos;
    }
    return o;
}

// The non-middle cases of MutationScorer::ScoreMutation (MutationScorer.cpp:219-267), from HBM.
__device__ double score_edge(const ScoreCtx& S, const Oriented& o, const ScoreScratch& scratch, TaskStat& st)
{
    const int J = S.Jorig;
    const bool atBegin = o.os < 3;
    const bool atEnd = o.oe > (J + 1) - 1 - 2;
    if (!atBegin && atEnd) {
        const int sc = o.os - 1;
        const int n = S.tv.Length() - sc + 1;
        return extend_alpha_score(S, sc, n, false, 0, 0, st);
    }
    if (atBegin && !atEnd) return extend_beta_score(S, o.oe, o.ld, st);
    if (!atBegin && !atEnd) {   // not reached from k_score (middle case has its own path)
        const int sc = (o.type == kDel) ? o.os - 1 : o.os;
        return extend_alpha_score(S, sc, 2, true, 1 + o.oe, 1 + o.oe + o.ld, st);
    }
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
    const long long u = fill_alpha(S.tv, S.rd, S.I, m, (const Band*)nullptr, false, S.P);
    st.cells += (unsigned long long)max(0LL, u);
    st.bytes += 8ull * (unsigned long long)max(0LL, u) + 16ull * (unsigned long long)ncol;
    return log(alpha_at(m, S.I, Jv)) + sum_ls(m, Jv + 1);
}

__device__ __forceinline__ int wave_min(int v)
{
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ __forceinline__ int wave_max(int v)
{
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}

// LDS stage of one wave: the alpha columns sc-1 and beta columns bc its 64 lanes read (contiguous in
// HBM because fills append columns in order) and the read bases under their rows.
// 448 staged alpha and beta values and 448 read bases per wave: 30.5 KB per 4-wave block, so five blocks
// (five waves per SIMD) fit the CU's 160 KB of LDS.
#ifndef PBCCS_SCORE_STAGE
#define PBCCS_SCORE_STAGE 448
#endif
constexpr int kScoreWaves = 4;
constexpr int kStageA = PBCCS_SCORE_STAGE;
constexpr int kStageB = PBCCS_SCORE_STAGE;
constexpr int kStageR = PBCCS_SCORE_STAGE;
struct WaveStage {
    double a[kStageA];
    double b[kStageB];
    char rd[kStageR];
};

// One wave per (work item, read, 64-mutation chunk): the lanes take consecutive mutations of one read,
// i.e. adjacent template positions, so the wave shares a handful of band columns.
// Occupancy: five waves per SIMD (<= 96 VGPRs; the stage above fits five blocks per CU).  The wave index is
// made wave-uniform (readfirstlane), so the item search and the per-item and per-read loads are scalar and
// the VGPR budget fits without spills (a kernel with a private segment needs scratch allocated at dispatch,
// which fails when the band pools have taken the device memory; check_resources.py refuses any).
#ifndef PBCCS_SCORE_WAVES
#define PBCCS_SCORE_WAVES 5
#endif
#if PBCCS_SCORE_WAVES > 0
#define PBCCS_SCORE_OCC __attribute__((amdgpu_waves_per_eu(PBCCS_SCORE_WAVES)))
#else
#define PBCCS_SCORE_OCC
#endif
__global__ void __launch_bounds__(256) PBCCS_SCORE_OCC k_score(DevBatch B, ScoreWork W, ScoreScratch scratch)
{
    // the start stamp waits in LDS: k_score sits at its register budget
    __shared__ long long wt0[kScoreWaves];
    if (PBCCS_WAVE_STAMPS && (threadIdx.x & 63) == 0) wt0[threadIdx.x >> 6] = wave_t0(B.stats);
    __shared__ WaveStage stage[kScoreWaves];
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: the item search and per-item loads go scalar
    const long long wave = (long long)blockIdx.x * kScoreWaves + wid;
    const int lane = threadIdx.x & 63;
    const bool waveLive = wave < W.waveStart[W.nWork];
    int k = 0;
    if (waveLive) {   // binary search of the work item (wave-uniform)
        int lo = 0, hi = W.nWork;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (W.waveStart[mid] <= wave) lo = mid; else hi = mid;
        }
        k = lo;
    }
    const int z = waveLive ? W.zmw[k] : 0;
    const int M = waveLive ? W.nMut[k] : 0;
    // mutations this phase scores: all of the item's, or its surviving ones (W.sel)
    const int Mc = (waveLive && W.sel) ? W.nSel[k] : M;
    const int chunks = max(1, (Mc + 63) >> 6);
    const long long local = waveLive ? wave - W.waveStart[k] : 0;
    const int rr = W.readLo + (int)(local / chunks);
    const int mc = (int)(local % chunks) * 64 + lane;
    const int r = waveLive ? B.zReadBegin[z] + rr : 0;
    // checkpointed reads are k_score_ckpt's (their non-checkpoint columns hold no values)
    const bool valid = waveLive && mc < Mc && !(B.rCkpt && B.rCkpt[r] != 0);
    const int m = (valid && W.sel) ? (int)(W.sel[W.selBase[k] + mc] - W.mutStart[k]) : mc;

    // classify this lane's task
    int code = 0;
    bool scored = false;
    if (valid) {
        code = W.codes[W.mutBase[k] + m];
        const int type = mut_type(code), pos = mut_pos(code);
        const int me = (type == kIns) ? pos : pos + 1;
        scored = B.rActive[r] && read_scores(B.rTs[r], B.rTe[r], type, pos, me);
    }
    ScoreCtx S;
    Oriented o;
    o.os = o.oe = o.ld = o.type = 0;
    bool middle = false;
    int sc = 0, bc = 0;
    MidGeom g;
    g.b0 = g.e0 = g.b1 = g.e1 = g.lb = g.le = 0;
    if (scored) {
        o = setup_score(B, r, code, S);
        const int J = S.Jorig;
        middle = !(o.os < 3) && !(o.oe > J - 2);
        if (middle) {
            sc = (o.type == kDel) ? o.os - 1 : o.os;
            bc = 1 + o.oe;
            g = middle_geometry(S.a, S.b, sc, bc);
        }
    }
    // wave-wide stage extents (only over middle lanes)
    const int aLo = wave_min(middle ? sc - 1 : INT_MAX), aHi = wave_max(middle ? sc - 1 : -1);
    const int bLo = wave_min(middle ? bc : INT_MAX), bHi = wave_max(middle ? bc : -1);
    const int rLo = wave_min(middle ? g.lb - 1 : INT_MAX), rHi = wave_max(middle ? g.le + 1 : -1);
    WaveStage& ws = stage[wid];
    bool staged = false;
    long long aBase = 0, bBase = 0;
    int rBase = 0;
    if (aHi >= 0) {
        const long long cb = B.rColBase[r];
        const int2 rah = B.aRange[cb + aHi];
        const int offLo = B.aOff[cb + aLo], offHi = B.aOff[cb + aHi];
        const int spanA = offHi + (rah.y - rah.x) - offLo;
        const int2 rbl = B.bRange[cb + bLo];
        const int boLo = B.bOff[cb + bLo], boHi = B.bOff[cb + bHi];
        const int spanB = boLo + (rbl.y - rbl.x) - boHi;
        const int I = B.rLen[r];
        const int r0 = max(0, rLo), r1 = min(I, rHi);
        const int spanR = r1 - r0;
        staged = spanA <= kStageA && spanB <= kStageB && spanR <= kStageR;
        if (staged) {
            const double* ga = B.valPool + B.rValA[r] + offLo;
            const double* gb = B.valPool + B.rValB[r] + boHi;
            const char* gr = B.seqPool + B.rSeqOff[r] + r0;
            for (int q = lane; q < spanA; q += 64) ws.a[q] = ga[q];
            for (int q = lane; q < spanB; q += 64) ws.b[q] = gb[q];
            for (int q = lane; q < spanR; q += 64) ws.rd[q] = gr[q];
            aBase = offLo;
            bBase = boHi;
            rBase = r0;
        }
    }
    __syncthreads();   // every wave of the block reaches this point exactly once

    TaskStat st;
    double d = 0.0;
    if (scored) {
        if (middle) {
            const int2 ar = S.a.range[sc - 1];
            const int2 br = S.b.range[bc];
            const int ao = S.a.off[sc - 1], bo = S.b.off[bc];
            double score;
            if (staged) {
                const double* av = ws.a + (ao - aBase) - ar.x;
                const double* bv = ws.b + (bo - bBase) + (br.y - 1);
                const char* rdp = ws.rd - rBase;
                score = score_middle(S, sc, bc, g, av, ar, bv, br, rdp, st);
            } else {
                const double* av = S.a.val + ao - ar.x;
                const double* bv = S.b.val + bo + (br.y - 1);
                score = score_middle(S, sc, bc, g, av, ar, bv, br, S.rd, st);
            }
            d = score - B.rBaseline[r];
        } else {
            // rare: mutations within 3 columns of a read's window ends -> k_score_edge
            const int slot = atomicAdd(W.edgeCount, 1);
            if (slot < W.edgeCap) {
                W.edgeList[3 * slot + 0] = k;
                W.edgeList[3 * slot + 1] = rr;
                W.edgeList[3 * slot + 2] = m;
            } else {
                atomicOr(scratch.overflow, 2);
            }
        }
    }
    if (valid && !(scored && !middle)) W.delta[W.deltaBase[k] + (long long)rr * M + m] = d;
    if (B.stats) {   // wave-reduce, one atomic per wave
        unsigned long long c = st.cells, b = st.bytes;
        for (int q = 32; q > 0; q >>= 1) {
            c += __shfl_xor(c, q, 64);
            b += __shfl_xor(b, q, 64);
        }
        if (lane == 0 && waveLive) {
            atomicAdd(&B.stats[2 * kStatScore], c);
            atomicAdd(&B.stats[2 * kStatScore + 1], b);
        }
        if (PBCCS_WAVE_STAMPS && lane == 0)
            atomicAdd(&B.stats[kWaveScore], (unsigned long long)((long long)__builtin_amdgcn_s_memrealtime() - wt0[wid]));
    }
}


// Edge cases of ScoreMutation (ExtendAlpha to the end, ExtendBeta to the start, whole refill), listed
// by k_score.  A separate kernel keeps their 4-column register state out of k_score's budget.
__device__ __forceinline__ void k_score_edge_body(DevBatch B, ScoreWork W, ScoreScratch scratch)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= *W.edgeCount || t >= W.edgeCap) return;
    const int k = W.edgeList[3 * t + 0], rr = W.edgeList[3 * t + 1], m = W.edgeList[3 * t + 2];
    const int z = W.zmw[k];
    const int M = W.nMut[k];
    const int r = B.zReadBegin[z] + rr;
    const int code = W.codes[W.mutBase[k] + m];
    ScoreCtx S;
    const Oriented o = setup_score(B, r, code, S);
    TaskStat st;
    const double d = score_edge(S, o, scratch, st) - B.rBaseline[r];
    W.delta[W.deltaBase[k] + (long long)rr * M + m] = d;
    if (B.stats) {
        atomicAdd(&B.stats[2 * kStatScore], st.cells);
        atomicAdd(&B.stats[2 * kStatScore + 1], st.bytes);
    }
}
__global__ void __launch_bounds__(64) k_score_edge(DevBatch B, ScoreWork W, ScoreScratch scratch)
{
    k_score_edge_body(B, W, scratch);   // (no wave stamp: roofline.occupancy's score family is k_score's)
}

// ------------------------------------------------------------------------------------------------
// k_score_ckpt: ScoreMutation for reads with checkpointed bands.  Such a read keeps the
// values of every K-th column only (ckpt_col_a / ckpt_col_b); a wave replays the columns its mutations
// read -- alpha forward from the kept column at or before them, beta backward from the kept column at or
// after them -- into its slot of C.slots, with the 64-lane insertion chain of the fill and each column's
// stored row range, so every replayed value is the fill's value bit for bit (a column depends only on the
// scaled column before it, the template, the read and its own range).  Then each lane scores its mutation
// with score_middle against the replayed columns, exactly as k_score does against stored ones.
// Persistent grid: each wave owns one slot and pulls 64-mutation chunks (tasks) from C.counter until none
// are left.  Lanes are scored block by block (alpha column / K), so a sparse chunk of a later scoring phase
// replays only the blocks it touches.  A block whose columns do not fit the slot is skipped and its size
// reported (C.need): the host grows the slots and reruns the launch.
// ------------------------------------------------------------------------------------------------
constexpr int kCkptCols = 3 * kCkptMaxK + 8;   // alpha <= K columns, beta <= 2K + 4 per block

// One replayed column's inputs that are uniform over the wave.
struct ReplayRead {
    const char* rd;   // read bases
    const char* T;    // strand template
    int I, J, L, start;
    const double* ctx;
    double prNot, prThird;
    __device__ __forceinline__ int TB(int idx) const   // TBase of fill_coop (nibble code of window base idx)
    {
        const int g = start + idx;
        return (idx <= J && g < L) ? coop::base_code(T[g]) : coop::kBaseOther;
    }
    __device__ __forceinline__ int TC(int idx) const   // TCtx of fill_coop
    {
        return (start + idx + 1 < L) ? coop::ctx_code(TB(idx), TB(idx + 1)) : kCtxZero;
    }
    __device__ __forceinline__ int RB(int i) const { return (i >= 0 && i < I) ? coop::base_code(rd[i]) : 15; }
};

// Rows per lane of the replay chain: the fill's 64-lane chain with R consecutive rows per lane and one DPP
// hand-off per R rows (coop_chain.hpp insertion_chain_rows; 17.6 against 29.3 cycles per row at R = 4 / 1,
// tools/ubench/chain_step.hip), each row in the reference's operation order.
constexpr int kReplayRows = 4;

// the insertion chain over the first n (>= 1) rows of a 64 R-row chunk; lanes holding only rows >= n are left
// unfinished
template <int R>
__device__ __forceinline__ void replay_chain(const double (&m)[R], const double (&k)[R], const double (&d)[R],
                                             double carry, int n, double (&x)[R])
{
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = 0.0;
    double up = carry;
    const int phases = (n + R - 1) / R;   // lanes [0, phases) hold the rows below n
#pragma unroll
    for (int p = 0; p < 64; p += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            up = coop::shift_up<64>(x[R - 1], up);
            x[0] = (m[0] + up * k[0]) + d[0];
#pragma unroll
            for (int r = 1; r < R; ++r) x[r] = (m[r] + x[r - 1] * k[r]) + d[r];
        }
        if (p + 4 >= phases) break;
    }
}

__device__ __forceinline__ double lane63(double x)   // the chunk-to-chunk carry (wave-uniform)
{
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), 63),
                            __builtin_amdgcn_readlane(__double2loint(x), 63));
}

__device__ __forceinline__ double wave_max_d(double x)
{
    for (int o = 32; o > 0; o >>= 1) x = fmax(x, __shfl_xor(x, o, 64));
    return x;
}

// Alpha column j (j >= 1) over its stored rows [b, e) from the scaled column j-1 (rows [pb, pe) at prev),
// scaled into cur (top-down): coop_alpha's column step (fill_coop.hip) without the band-end logic; lane l
// takes rows i0 + l R .. i0 + l R + R - 1 of each 64 R-row chunk.
__device__ void replay_alpha(const ReplayRead& X, int j, const double* prev, int pb, int pe, double* cur, int b, int e)
{
    constexpr int R = kReplayRows;
    const int lane = threadIdx.x & 63;
    const int curBase = X.TB(j - 1), nextBase = X.TB(j);
    const double* cp = X.ctx + X.TC(j - 1) * kCtxStride;
    const double* pp = X.ctx + (j >= 2 ? X.TC(j - 2) : kCtxZero) * kCtxStride;
    const double pMatch = pp[kM], pDel = pp[kD], cBranch = cp[kB], cStick3 = cp[kS3];
    double carry = 0.0, mx = 0.0;
    for (int i0 = b; i0 < e; i0 += 64 * R) {
        const int ib = i0 + lane * R;
        double pv[R + 1], m[R], k[R], d[R], x[R];
#pragma unroll
        for (int q = 0; q <= R; ++q) {
            const int row = ib - 1 + q;
            pv[q] = (row >= pb && row < pe) ? prev[row - pb] : 0.0;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int i = ib + r;
            const int rb = (i >= 1 && i <= X.I) ? X.RB(i - 1) : 15;
            const double mpe = pv[r] * (rb == curBase ? X.prNot : X.prThird);
            m[r] = (i == 1 && j == 1) ? mpe : ((i != 1 && j != 1) ? mpe * pMatch : 0.0);
            k[r] = (i > 1) ? (rb == nextBase ? cBranch : cStick3) : 0.0;
            d[r] = (j > 1) ? pv[r + 1] * pDel : 0.0;
        }
        replay_chain<R>(m, k, d, carry, e - i0, x);
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (ib + r < e) {
                cur[ib + r - b] = x[r];
                mx = fmax(mx, x[r]);
            }
        carry = lane63(x[R - 1]);
    }
    mx = wave_max_d(mx);
    if (mx != 0.0 && mx != 1.0)   // ScaledMatrix::FinishEditingColumn, each row by the lane that stored it
        for (int i0 = b; i0 < e; i0 += 64 * R)
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int i = i0 + lane * R + r;
                if (i < e) cur[i - b] = cur[i - b] / mx;
            }
}

// Beta column j (0 < j < J) over its stored rows [b, e), bottom-up, from the scaled column j+1 (rows [pb, pe)
// at nxt, stored bottom-up), scaled into cur (bottom-up): coop_beta's column step, R offsets per lane.
__device__ void replay_beta(const ReplayRead& X, int j, const double* nxt, int pb, int pe, double* cur, int b, int e)
{
    constexpr int R = kReplayRows;
    const int lane = threadIdx.x & 63;
    const int nextBase = X.TB(j);
    const double* cp = X.ctx + X.TC(j - 1) * kCtxStride;
    const double cMatch = cp[kM], cDel = cp[kD], cBranch = cp[kB], cStick3 = cp[kS3];
    const int I = X.I, J = X.J;
    double carry = 0.0, mx = 0.0;
    for (int o0 = 0; o0 < e - b; o0 += 64 * R) {
        const int ob = o0 + lane * R;
        double pv[R + 1], m[R], k[R], d[R], x[R];
#pragma unroll
        for (int q = 0; q <= R; ++q) {   // rows e - ob - q: diag of offset q, left of offset q - 1
            const int row = e - ob - q;
            pv[q] = (row >= pb && row < pe) ? nxt[pe - 1 - row] : 0.0;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int i = e - 1 - ob - r;
            const int nb = X.RB(i);
            const bool same = nb == nextBase;
            const double mpe = pv[r] * (same ? X.prNot : X.prThird);
            m[r] = (i < I - 1) ? mpe * cMatch : ((i == I - 1 && j == J - 1) ? mpe : 0.0);
            k[r] = (i < I - 1 && i > 0) ? (same ? cBranch : cStick3) : 0.0;
            d[r] = (j < J - 1 && j > 0) ? pv[r + 1] * cDel : 0.0;
        }
        replay_chain<R>(m, k, d, carry, e - b - o0, x);
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (e - 1 - ob - r >= b) {
                cur[ob + r] = x[r];
                mx = fmax(mx, x[r]);
            }
        carry = lane63(x[R - 1]);
    }
    mx = wave_max_d(mx);
    if (mx != 0.0 && mx != 1.0)   // each offset by the lane that stored it
        for (int o0 = 0; o0 < e - b; o0 += 64 * R)
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int off = o0 + lane * R + r;
                if (off < e - b) cur[off] = cur[off] / mx;
            }
}

__device__ __forceinline__ void k_score_ckpt_body(DevBatch B, ScoreWork W, CkptWork C)
{
    __shared__ int sOff[kCkptCols];
    const int lane = threadIdx.x;
    double* slot = C.slots + (long long)blockIdx.x * C.slotCap;
    for (;;) {
        unsigned long long tt = 0;
        if (lane == 0) tt = atomicAdd(C.counter, 1ull);
        const unsigned hi32 = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(tt >> 32));
        const unsigned lo32 = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)tt);
        const long long t = (long long)(((unsigned long long)hi32 << 32) | lo32);
        if (t >= C.nTasks) break;   // every wave leaves once the task list is drained
        int lo = 0, hi = C.nPairs;   // pair of task t (wave-uniform binary search)
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (C.taskStart[mid] <= t) lo = mid; else hi = mid;
        }
        const int k = C.pairs[lo].x, rr = C.pairs[lo].y;
        const int chunk = (int)(t - C.taskStart[lo]);
        const int z = W.zmw[k];
        const int M = W.nMut[k];
        const int Mc = W.sel ? W.nSel[k] : M;
        const int mc = chunk * 64 + lane;
        const bool valid = mc < Mc;
        const int m = (valid && W.sel) ? (int)(W.sel[W.selBase[k] + mc] - W.mutStart[k]) : mc;
        const int r = B.zReadBegin[z] + rr;
        int code = 0;
        bool scored = false;
        if (valid) {
            code = W.codes[W.mutBase[k] + m];
            const int type = mut_type(code), pos = mut_pos(code);
            const int me = (type == kIns) ? pos : pos + 1;
            scored = B.rActive[r] && read_scores(B.rTs[r], B.rTe[r], type, pos, me);
        }
        ScoreCtx S;
        Oriented o;
        o.os = o.oe = o.ld = o.type = 0;
        bool middle = false;
        int sc = 0, bc = 0;
        MidGeom g;
        g.b0 = g.e0 = g.b1 = g.e1 = g.lb = g.le = 0;
        if (scored) {
            o = setup_score(B, r, code, S);
            const int J = S.Jorig;
            middle = !(o.os < 3) && !(o.oe > J - 2);
            if (middle) {
                sc = (o.type == kDel) ? o.os - 1 : o.os;
                bc = 1 + o.oe;
                g = middle_geometry(S.a, S.b, sc, bc);
            } else {   // ends of the window: k_score_edge (the kept tail columns hold their values)
                const int es = atomicAdd(W.edgeCount, 1);
                if (es < W.edgeCap) {
                    W.edgeList[3 * es + 0] = k;
                    W.edgeList[3 * es + 1] = rr;
                    W.edgeList[3 * es + 2] = m;
                }
            }
        }
        if (valid && !scored) W.delta[W.deltaBase[k] + (long long)rr * M + m] = 0.0;
        // replay + score, one alpha block (column / K) at a time
        const int K = B.rCkpt[r];
        const int J = B.rTe[r] - B.rTs[r];
        const long long cbase = B.rColBase[r];
        const int2* aR = B.aRange + cbase;
        const int2* bR = B.bRange + cbase;
        const int* aO = B.aOff + cbase;
        const int* bO = B.bOff + cbase;
        const double* aV = B.valPool + B.rValA[r];
        const double* bV = B.valPool + B.rValB[r];
        ReplayRead X;
        {
            const TplView tv = window_view(B, r);
            X.rd = B.seqPool + B.rSeqOff[r];
            X.T = tv.T;
            X.I = B.rLen[r];
            X.J = J;
            X.L = tv.L;
            X.start = tv.start;
            X.ctx = B.zCtx + (long long)z * 9 * kCtxStride;
            X.prNot = B.prNot;
            X.prThird = B.prThird;
        }
        bool pending = middle;
        TaskStat st;
        while (__ballot(pending) != 0) {
            const int ja = sc - 1;
            const int q = wave_min(pending ? ja / K : INT_MAX);
            const bool mine = pending && ja / K == q;
            const int aHi = wave_max(mine ? ja : -1);
            const int jbLo = wave_min(mine ? bc : INT_MAX), jbHi = wave_max(mine ? bc : -1);
            const int ckA = q * K;                 // kept (j % K == 0)
            int ckB = jbHi;
            while (!ckpt_col_b(ckB, J, K)) ++ckB;   // <= the next multiple of K, or J
            const int nA = aHi - ckA + 1, nB = ckB - jbLo + 1;
            // slot layout: alpha columns ckA..aHi, then beta columns ckB down to jbLo, each compact
            long long need = 0;
            if (nA + nB <= kCkptCols) {
                long long hsum = 0;
                for (int c = lane; c < nA + nB; c += 64) {
                    const int2 rg = c < nA ? aR[ckA + c] : bR[ckB - (c - nA)];
                    hsum += max(0, rg.y - rg.x);
                }
                for (int w = 32; w > 0; w >>= 1) hsum += __shfl_xor(hsum, w, 64);
                need = hsum;
            }
            if (nA + nB > kCkptCols || need > C.slotCap) {   // rerun with larger slots (or a bad geometry)
                if (lane == 0) atomicMax(C.need, nA + nB > kCkptCols ? kCkptBadGeometry : (unsigned long long)need);
                pending = pending && !mine;
                continue;
            }
            if (lane == 0) {
                int o2 = 0;
                for (int c = 0; c < nA + nB; ++c) {
                    const int2 rg = c < nA ? aR[ckA + c] : bR[ckB - (c - nA)];
                    sOff[c] = o2;
                    o2 += max(0, rg.y - rg.x);
                }
            }
            __syncthreads();
            // alpha: the kept column, then forward
            {
                const int2 r0 = aR[ckA];
                const double* src = aV + aO[ckA];
                for (int i = lane; i < r0.y - r0.x; i += 64) slot[sOff[0] + i] = src[i];
                for (int j = ckA + 1; j <= aHi; ++j) {
                    const int2 pr = aR[j - 1], rg = aR[j];
                    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
                    replay_alpha(X, j, slot + sOff[j - 1 - ckA], pr.x, pr.y, slot + sOff[j - ckA], rg.x, rg.y);
                }
            }
            // beta: the kept column, then backward
            {
                const int2 r0 = bR[ckB];
                const double* src = bV + bO[ckB];
                for (int i = lane; i < r0.y - r0.x; i += 64) slot[sOff[nA] + i] = src[i];
                for (int j = ckB - 1; j >= jbLo; --j) {
                    const int2 nr = bR[j + 1], rg = bR[j];
                    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
                    replay_beta(X, j, slot + sOff[nA + (ckB - (j + 1))], nr.x, nr.y, slot + sOff[nA + (ckB - j)], rg.x,
                                rg.y);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
            if (mine) {
                const int2 ar = aR[ja];
                const int2 br = bR[bc];
                const double* av = slot + sOff[ja - ckA] - ar.x;
                const double* bv = slot + sOff[nA + (ckB - bc)] + (br.y - 1);
                const double score = score_middle(S, sc, bc, g, av, ar, bv, br, S.rd, st);
                W.delta[W.deltaBase[k] + (long long)rr * M + m] = score - B.rBaseline[r];
            }
            pending = pending && !mine;
            __syncthreads();   // sOff and the slot are reused by the next block
        }
        if (B.stats) {
            unsigned long long c2 = st.cells, b2 = st.bytes;
            for (int w = 32; w > 0; w >>= 1) {
                c2 += __shfl_xor(c2, w, 64);
                b2 += __shfl_xor(b2, w, 64);
            }
            if (lane == 0) {
                atomicAdd(&B.stats[2 * kStatScore], c2);
                atomicAdd(&B.stats[2 * kStatScore + 1], b2);
            }
        }
    }
}
__global__ void __launch_bounds__(64) k_score_ckpt(DevBatch B, ScoreWork W, CkptWork C)
{
    k_score_ckpt_body(B, W, C);
}

// Ordered reduction over reads with the fast-score break (MultiReadMutationScorer.cpp:352-362).
__device__ __forceinline__ void k_reduce_body(DevBatch B, ScoreWork W, double fastThr, double* __restrict__ score,
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
    const double e = W.dev ? W.dev[k] : 0.0;   // certified fast path: the bound of this item's sums
    bool amb = false;
    for (int rr = 0; rr < nr; ++rr) {
        const int r = rb + rr;
        if (B.rActive[r] && read_scores(B.rTs[r], B.rTe[r], type, pos, me)) sum += d[(long long)rr * M];
        if (e > 0.0) amb = amb || fabs(sum - fastThr) <= e + 1e-12 * fabs(fastThr);
        if (sum < fastThr) break;
    }
    score[W.mutBase[k] + m] = sum;
    fav[W.mutBase[k] + m] = (sum > 0.04) ? 1 : 0;   // MIN_FAVORABLE_SCOREDIFF, MultiReadMutationScorer.cpp:56
    if (e > 0.0 && (amb || fabs(sum - 0.04) <= e)) W.amb[k] = 1;   // the item's round is re-scored on exact bands
}
__global__ void __launch_bounds__(256) k_reduce(DevBatch B, ScoreWork W, double fastThr, double* __restrict__ score,
                                                unsigned char* __restrict__ fav)
{
    const long long wt0 = wave_t0(B.stats);
    k_reduce_body(B, W, fastThr, score, fav);
    wave_ticks(B.stats, kWaveReduce, wt0);
}

// The reduction's ordered prefix over the first readHi reads only (same sums, same break).
__global__ void __launch_bounds__(256) k_alive(DevBatch B, ScoreWork W, double fastThr, int readHi,
                                               unsigned char* __restrict__ alive)
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
    const int rb = B.zReadBegin[z], nr = min(B.zNReads[z], readHi);
    const double* d = W.delta + W.deltaBase[k] + m;
    double sum = 0.0;
    bool live = true;
    for (int rr = 0; rr < nr; ++rr) {
        const int r = rb + rr;
        if (B.rActive[r] && read_scores(B.rTs[r], B.rTe[r], type, pos, me)) sum += d[(long long)rr * M];
        if (sum < fastThr) {
            live = false;
            break;
        }
    }
    alive[g] = live ? 1 : 0;
}

// selBase[k] / nSel[k]: the entries of the ascending selected list that fall in item k's mutation range.
__global__ void __launch_bounds__(256) k_sel_ranges(ScoreWork W, const long long* __restrict__ sel,
                                                    const long long* __restrict__ count, long long* __restrict__ selBase,
                                                    int* __restrict__ nSel)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= W.nWork) return;
    const long long n = *count;
    auto lower = [&](long long v) {
        long long lo = 0, hi = n;
        while (lo < hi) {
            const long long mid = (lo + hi) >> 1;
            if (sel[mid] < v) lo = mid + 1; else hi = mid;
        }
        return lo;
    };
    const long long b = lower(W.mutStart[k]), e = lower(W.mutStart[k + 1]);
    selBase[k] = b;
    nSel[k] = (int)(e - b);
}

// BestSubset (Consensus-inl.hpp:98-118) per work item, on its favourable list compacted in list order:
// greedily the first maximum of the float-cast scores, then every entry whose Start lies within
// [best - sep, best + sep] leaves the list; again until it is empty.  One wavefront per work item; lane l
// owns entries q = l mod 64 (kept in LDS up to ldsCap <= kBestLds entries, read from HBM beyond), so the per-entry
// state needs no cross-lane ordering.  rank[q] = k for the k-th pick (1-based), 0 for a removed entry.
// sep = 0 keeps the whole list in order (the reference returns its input).
constexpr int kBestLds = 2048;

__device__ inline unsigned order_key(float f)   // float order as unsigned order (no NaN reaches here)
{
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ void __launch_bounds__(64) k_best_subset(const long long* __restrict__ selBase, const int* __restrict__ nSel,
                                                    const int* __restrict__ code, const double* __restrict__ score,
                                                    int sep, int ldsCap, int* __restrict__ rank)
{
    __shared__ unsigned sKey[kBestLds];
    __shared__ int sPos[kBestLds];
    __shared__ int sRank[kBestLds];
    const int k = blockIdx.x, lane = threadIdx.x;
    const long long b = selBase[k];
    const int m = nSel[k];
    const int* c = code + b;
    const double* sc = score + b;
    int* rk = rank + b;
    if (sep == 0) {
        for (int q = lane; q < m; q += 64) rk[q] = q + 1;
        return;
    }
    const int ml = m < ldsCap ? m : ldsCap;
    for (int q = lane; q < ml; q += 64) {
        sKey[q] = order_key((float)sc[q]);
        sPos[q] = mut_pos(c[q]);
        sRank[q] = -1;   // alive
    }
    for (int q = ml + lane; q < m; q += 64) rk[q] = -1;
    for (int picks = 1;; ++picks) {
        // first maximum: the highest key, then the lowest index (the key's low word is ~q)
        unsigned long long best = 0;
        for (int q = lane; q < ml; q += 64)
            if (sRank[q] < 0) {
                const unsigned long long v = ((unsigned long long)sKey[q] << 32) | (0xFFFFFFFFu - (unsigned)q);
                best = v > best ? v : best;
            }
        for (int q = ml + lane; q < m; q += 64)
            if (rk[q] < 0) {
                const unsigned long long v = ((unsigned long long)order_key((float)sc[q]) << 32) |
                                             (0xFFFFFFFFu - (unsigned)q);
                best = v > best ? v : best;
            }
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long o = __shfl_xor(best, off, 64);
            best = o > best ? o : best;
        }
        if (best == 0) break;   // order_key is never 0 for a finite score: the list is empty
        const int bq = (int)(0xFFFFFFFFu - (unsigned)(best & 0xFFFFFFFFu));
        const int bp = mut_pos(c[bq]);
        const int lo = bp - sep, hi = bp + sep;
        for (int q = lane; q < ml; q += 64)
            if (sRank[q] < 0 && lo <= sPos[q] && sPos[q] <= hi) sRank[q] = q == bq ? picks : 0;
        for (int q = ml + lane; q < m; q += 64)
            if (rk[q] < 0) {
                const int pq = mut_pos(c[q]);
                if (lo <= pq && pq <= hi) rk[q] = q == bq ? picks : 0;
            }
    }
    for (int q = lane; q < ml; q += 64) rk[q] = sRank[q];
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
void launch_fill(const DevBatch& B, const FillScratch& F, const int* reads, int n, hipStream_t s)
{
    if (n <= 0) return;
    hipLaunchKernelGGL(k_fill, dim3((n + 63) / 64), dim3(64), 0, s, B, F, reads, n);
}

void launch_compact(const DevBatch& B, const FillScratch& F, const int* reads, int n, hipStream_t s)
{
    if (n <= 0) return;
    hipLaunchKernelGGL(k_compact, dim3((n + 63) / 64), dim3(256), 0, s, B, F, reads, n);
}

void launch_suffix(const DevBatch& B, const int* reads, int n, hipStream_t s, bool withPrefix)
{
    if (n <= 0) return;
    hipLaunchKernelGGL(k_suffix, dim3(n), dim3(256), 0, s, B, reads, n, withPrefix ? 1 : 0);
}

void launch_enumerate(const DevBatch& B, const int* zmws, int n, const long long* mutBase, const long long* posBase,
                      int* codes, int* posOff, hipStream_t s)
{
    if (n <= 0) return;
    hipLaunchKernelGGL(k_enumerate, dim3(n), dim3(256), 0, s, B, zmws, mutBase, posBase, codes, posOff);
}

void launch_score(const DevBatch& B, const ScoreWork& W, long long nWaves, const ScoreScratch& scratch, hipStream_t s,
                  const CkptWork* ck)
{
    if (nWaves <= 0) return;
    const long long blocks = (nWaves + kScoreWaves - 1) / kScoreWaves;
    hipLaunchKernelGGL(k_score, dim3((unsigned)blocks), dim3(64 * kScoreWaves), 0, s, B, W, scratch);
    if (ck && ck->nTasks > 0 && ck->nSlots > 0)
        hipLaunchKernelGGL(k_score_ckpt, dim3((unsigned)ck->nSlots), dim3(64), 0, s, B, W, *ck);
    if (W.edgeCap > 0)
        hipLaunchKernelGGL(k_score_edge, dim3((W.edgeCap + 63) / 64), dim3(64), 0, s, B, W, scratch);
}

void launch_reduce(const DevBatch& B, const ScoreWork& W, long long nMut, double fastThr, double* score,
                   unsigned char* fav, hipStream_t s)
{
    if (nMut <= 0) return;
    hipLaunchKernelGGL(k_reduce, dim3((unsigned)((nMut + 255) / 256)), dim3(256), 0, s, B, W, fastThr, score, fav);
}

void launch_alive(const DevBatch& B, const ScoreWork& W, long long nMut, double fastThr, int readHi,
                  unsigned char* alive, hipStream_t s)
{
    if (nMut <= 0) return;
    hipLaunchKernelGGL(k_alive, dim3((unsigned)((nMut + 255) / 256)), dim3(256), 0, s, B, W, fastThr, readHi, alive);
}

void launch_sel_ranges(const ScoreWork& W, const long long* sel, const long long* count, long long* selBase,
                       int* nSel, hipStream_t s)
{
    if (W.nWork <= 0) return;
    hipLaunchKernelGGL(k_sel_ranges, dim3((W.nWork + 255) / 256), dim3(256), 0, s, W, sel, count, selBase, nSel);
}

void launch_best_subset(int nWork, const long long* selBase, const int* nSel, const int* code, const double* score,
                        int sep, int ldsCap, int* rank, hipStream_t s)
{
    if (nWork <= 0) return;
    ldsCap = ldsCap < 0 || ldsCap > kBestLds ? kBestLds : ldsCap;
    hipLaunchKernelGGL(k_best_subset, dim3(nWork), dim3(64), 0, s, selBase, nSel, code, score, sep, ldsCap, rank);
}

void launch_qv(const DevBatch& B, const ScoreWork& W, long long nPos, const long long* posBase, const int* posOff,
               const double* score, const long long* qvBase, int* qv, hipStream_t s)
{
    if (nPos <= 0) return;
    hipLaunchKernelGGL(k_qv, dim3((unsigned)((nPos + 255) / 256)), dim3(256), 0, s, B, W, posBase, posOff, score,
                       qvBase, qv);
}

}  // namespace pbccs
