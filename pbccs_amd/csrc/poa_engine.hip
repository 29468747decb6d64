// pbccs_amd/csrc/poa_engine.hip -- the POA draft step: read-vs-graph DP and traceback kernels for
// gfx950, and the host loop that threads reads into the graphs.
//
// Reference: ConsensusCore/src/C++/Poa/PoaGraphImpl.cpp:177-447 (alignment columns, TryAddRead,
// CommitAdd), PoaGraphTraversals.cpp:227-369 (traceback), pbccs src/SparsePoa.cpp:95-201.
//
// The DP (makeAlignmentColumn, PoaGraphImpl.cpp:236-352) scores with DefaultPoaConfig's integers
// (match 3, mismatch -5, insert -4, delete -4) in float; every cell is an integer far below 2^24, so
// the float sums are exact and the device runs them in int32 -- the same values, bit for bit.  A cell
//     S(v, i) = max( [LOCAL, i > 0] 0,
//                    max over predecessors u:  S(u, i-1) + (read[i-1] == base(v) ? 3 : -5),  S(u, i) - 4,
//                    S(v, i-1) - 4 )
// is a column recurrence whose only serial term is the last one (the Extra move).  With
// g(i) = ne(i) + 4 i, where ne is the max of the other terms, S(v, i) = max_{k <= i} g(k) - 4 i: a prefix
// maximum, which the wavefront takes with DPP.  So one wavefront fills a column 1024 rows at a time
// (16 contiguous rows per lane), columns in the graph's topological order.
//
// Layout in HBM: each alignment owns nCols x colStride score cells (colStride = rows padded to 1024),
// row-major per column so a lane's 16 rows are one or two 16-byte accesses and a wave's are contiguous.
// LOCAL scores are >= 0 and at most 3 * rows, so they are stored as uint16 when that fits (half the
// traffic); other modes and longer reads use int32.  The traceback does not store moves: it recomputes
// the reaching move of each visited cell from the scores with the reference's candidate order and strict
// '>' ties, which is what tracebackAndThread reads from AlignmentColumn::ReachingMove / PreviousVertex.
#include "poa_engine.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstring>
#include <memory>
#include <thread>

namespace pbccs {
namespace poa {

namespace {

constexpr int kMatchScore = 3, kMismatchScore = -5, kInsertScore = -4, kDeleteScore = -4;   // DefaultPoaConfig
constexpr int kNeg = -(1 << 29);   // stands in for -FLT_MAX: every real candidate beats it

template <int CTRL, int ROWMASK>
__device__ __forceinline__ int dpp_i(int old, int x)
{
    return __builtin_amdgcn_update_dpp(old, x, CTRL, ROWMASK, 0xF, false);
}

// inclusive prefix maximum over the wavefront's 64 lanes
__device__ __forceinline__ int wave_prefix_max(int x)
{
    x = max(x, dpp_i<0x111, 0xF>(kNeg, x));   // row_shr:1
    x = max(x, dpp_i<0x112, 0xF>(kNeg, x));   // row_shr:2
    x = max(x, dpp_i<0x114, 0xF>(kNeg, x));   // row_shr:4
    x = max(x, dpp_i<0x118, 0xF>(kNeg, x));   // row_shr:8
    x = max(x, dpp_i<0x142, 0xA>(kNeg, x));   // row_bcast:15
    x = max(x, dpp_i<0x143, 0xC>(kNeg, x));   // row_bcast:31
    return x;
}

// (value, key) maximum over the wave: larger value, then smaller key
__device__ __forceinline__ void wave_argmax(int& v, int& key)
{
    for (int off = 32; off > 0; off >>= 1) {
        const int ov = __shfl_xor(v, off);
        const int ok = __shfl_xor(key, off);
        if (ov > v || (ov == v && ok < key)) {
            v = ov;
            key = ok;
        }
    }
}

template <class ST>
struct Rows16;

template <>
struct Rows16<uint16_t> {
    static __device__ __forceinline__ void load(const uint16_t* p, int* v)
    {
        const uint4 a = reinterpret_cast<const uint4*>(p)[0], b = reinterpret_cast<const uint4*>(p)[1];
        const unsigned w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = (int)((w[r >> 1] >> ((r & 1) * 16)) & 0xFFFFu);
    }
    static __device__ __forceinline__ void store(uint16_t* p, const int* v)
    {
        unsigned w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = (unsigned)(v[2 * k] & 0xFFFF) | ((unsigned)v[2 * k + 1] << 16);
        reinterpret_cast<uint4*>(p)[0] = make_uint4(w[0], w[1], w[2], w[3]);
        reinterpret_cast<uint4*>(p)[1] = make_uint4(w[4], w[5], w[6], w[7]);
    }
};

template <>
struct Rows16<int> {
    static __device__ __forceinline__ void load(const int* p, int* v)
    {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int4 a = reinterpret_cast<const int4*>(p)[k];
            v[4 * k] = a.x;
            v[4 * k + 1] = a.y;
            v[4 * k + 2] = a.z;
            v[4 * k + 3] = a.w;
        }
    }
    static __device__ __forceinline__ void store(int* p, const int* v)
    {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            reinterpret_cast<int4*>(p)[k] = make_int4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    }
};

// TryAddRead's alignment columns (PoaGraphImpl.cpp:384-435): one wavefront per job, columns in the
// program's topological order.  Also the $ column (makeAlignmentColumnForExit, :177-233): its score
// and the column it is reached from.
template <class ST>
__global__ __launch_bounds__(64) void k_poa_fill(const PoaJob* __restrict__ jobs, int jobBase, PoaPools P,
                                                 ST* __restrict__ pool, int* __restrict__ outScore,
                                                 int* __restrict__ outExitCol)
{
    const int j = jobBase + blockIdx.x;
    const PoaJob J = jobs[j];
    const int lane = threadIdx.x;
    ST* S = pool + J.scoreOff;
    const uint8_t* rb = P.rowBase + J.readOff;
    const int I = J.I, stride = J.colStride, mode = J.mode;
    const int* predStart = P.predStart + J.predStartOff;
    int bestVal = kNeg, bestVid = INT_MAX, bestCol = 0;
    for (int k = 0; k < J.nCols; ++k) {
        const int base = P.base[J.progOff + k];
        const int vid = P.vertexOfCol[J.progOff + k];
        const int ps = predStart[k], pe = predStart[k + 1];
        ST* col = S + (long long)k * stride;
        int carry = kNeg, colBest = kNeg;
        for (int c0 = 0; c0 <= I; c0 += kChunkRows) {
            const int i0 = c0 + lane * 16;
            const uint4 rw = *reinterpret_cast<const uint4*>(rb + i0);
            const unsigned rbw[4] = {rw.x, rw.y, rw.z, rw.w};
            int ne[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) ne[r] = mode == kLocal ? 0 : kNeg;
            // row 0: ^ has no reaching move (0); LOCAL/SEMIGLOBAL start there (0); GLOBAL deletes into it
            if (i0 == 0) ne[0] = (ps == pe || mode != kGlobal) ? 0 : kNeg;
            for (int p = ps; p < pe; ++p) {
                const ST* q = S + (long long)P.predCol[p] * stride;
                int qv[16];
                Rows16<ST>::load(q + i0, qv);
                int up = i0 > 0 ? (int)q[i0 - 1] : kNeg;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int b = (rbw[r >> 2] >> ((r & 3) * 8)) & 0xFF;
                    const int diag = up + (b == base ? kMatchScore : kMismatchScore);
                    ne[r] = max(ne[r], max(diag, qv[r] + kDeleteScore));
                    up = qv[r];
                }
            }
            // Extra moves: S(i) = max_{k<=i} (ne(k) - k * insert) + i * insert
            int run = kNeg;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                run = max(run, ne[r] - (i0 + r) * kInsertScore);
                ne[r] = run;
            }
            const int incl = wave_prefix_max(run);
            const int excl = max(dpp_i<0x138, 0xF>(kNeg, incl), carry);   // wave_shr:1
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int i = i0 + r;
                ne[r] = max(ne[r], excl) + i * kInsertScore;
                if (i <= I && (mode == kLocal || (mode == kSemiGlobal && i == I))) colBest = max(colBest, ne[r]);
            }
            Rows16<ST>::store(col + i0, ne);
            carry = __builtin_amdgcn_readlane(max(incl, carry), 63);
        }
        if (colBest > bestVal || (colBest == bestVal && vid < bestVid)) {
            bestVal = colBest;
            bestVid = vid;
            bestCol = k;
        }
        // the next columns' lanes read rows this column's lanes wrote
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    }
    if (mode == kGlobal) {
        // regular predecessors of $ in in-edge order, strict '>' (PoaGraphImpl.cpp:214-227)
        bestVal = kNeg;
        bestCol = 0;
        for (int e = 0; e < J.nExit; ++e) {
            const int c = P.exitPred[J.exitOff + e];
            const int v = (int)S[(long long)c * stride + I];
            if (v > bestVal) {
                bestVal = v;
                bestCol = c;
            }
        }
    } else {
        int key = bestVid;
        const int v0 = bestVal;
        wave_argmax(bestVal, key);
        // the lane holding the winner publishes its column
        const unsigned long long m = __ballot(v0 == bestVal && bestVid == key);
        bestCol = __shfl(bestCol, (int)__builtin_ctzll(m));
    }
    if (lane == 0) {
        outScore[j] = bestVal;
        outExitCol[j] = bestCol;
    }
}

// LDS-ring variant (LOCAL uint16 jobs of up to 64 * RMAX rows).  A lane owns R = ceil(rows / 64)
// consecutive rows, so a column is one wave pass with no row padding beyond 64; the last K columns stay in
// an LDS ring, and the global copy (for the traceback and for predecessors further back) is stored
// lane-interleaved -- row i of a column at (i % R) * 64 + i / R -- so every store instruction writes 64
// consecutive uint16.  Predecessors within the ring are read from LDS; the workgroup fence that makes the
// global stores visible to the wave's own loads is paid only for a predecessor older than the ring.
template <int R, int K>
__global__ __launch_bounds__(64) void k_poa_fill_lds(const PoaJob* __restrict__ jobs, int jobBase, PoaPools P,
                                                     uint16_t* __restrict__ pool, int* __restrict__ outScore,
                                                     int* __restrict__ outExitCol)
{
    extern __shared__ uint16_t ring[];   // K columns x 64 * R
    const int j = jobBase + blockIdx.x;
    const PoaJob J = jobs[j];
    const int lane = threadIdx.x;
    uint16_t* S = pool + J.scoreOff;
    const int I = J.I, stride = J.colStride, mode = J.mode;   // stride == 64 * R
    const int* predStart = P.predStart + J.predStartOff;
    const int i0 = lane * R;
    // the lane's read bases (row i holds read[i - 1]), 4 per word
    unsigned rbw[R / 4];
#pragma unroll
    for (int w = 0; w < R / 4; ++w) {
        unsigned x = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b)
            x |= (unsigned)P.rowBase[J.readOff + i0 + 4 * w + b] << (8 * b);
        rbw[w] = x;
    }
    bool dirty = false;
    int bestVal = kNeg, bestVid = INT_MAX, bestCol = 0;
    for (int k = 0; k < J.nCols; ++k) {
        const int base = P.base[J.progOff + k];
        const int vid = P.vertexOfCol[J.progOff + k];
        const int ps = predStart[k], pe = predStart[k + 1];
        int ne[R];
#pragma unroll
        for (int r = 0; r < R; ++r) ne[r] = mode == kLocal ? 0 : kNeg;
        if (lane == 0) ne[0] = 0;   // row 0: ^ has no reaching move, everything else starts there (LOCAL)
        // one predecessor column, streamed row by row from LDS (ring) or HBM
        auto absorb = [&](auto col) {
            int up = lane > 0 ? (int)col[(R - 1) * 64 + lane - 1] : kNeg;
            const auto c = col + lane;   // rows at constant offsets r * 64 from one base
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int qr = (int)c[r * 64];
                const int b = (rbw[r >> 2] >> ((r & 3) * 8)) & 0xFF;
                ne[r] = max(ne[r], max(up + (b == base ? kMatchScore : kMismatchScore), qr + kDeleteScore));
                up = qr;
            }
        };
        for (int p = ps; p < pe; ++p) {
            const int pc = P.predCol[p];
            if (k - pc < K) {
                absorb(ring + (pc % K) * stride);
            } else {
                if (dirty) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
                    dirty = false;
                }
                absorb(S + (long long)pc * stride);
            }
        }
        int run = kNeg;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            run = max(run, ne[r] - (i0 + r) * kInsertScore);
            ne[r] = run;
        }
        const int incl = wave_prefix_max(run);
        const int excl = dpp_i<0x138, 0xF>(kNeg, incl);   // wave_shr:1
        int colBest = kNeg;
        uint16_t* slot = ring + (k % K) * stride + lane;
        uint16_t* out = S + (long long)k * stride + lane;
        __syncthreads();   // the slot's previous column (k - K) has been read by every lane
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int i = i0 + r;
            const int v = max(ne[r], excl) + i * kInsertScore;
            if (i <= I) colBest = max(colBest, v);
            slot[r * 64] = (uint16_t)v;
            out[r * 64] = (uint16_t)v;
        }
        __syncthreads();   // the column is in the ring before the next column reads it
        dirty = true;
        if (colBest > bestVal || (colBest == bestVal && vid < bestVid)) {
            bestVal = colBest;
            bestVid = vid;
            bestCol = k;
        }
    }
    int key = bestVid;
    const int v0 = bestVal;
    wave_argmax(bestVal, key);
    const unsigned long long m = __ballot(v0 == bestVal && bestVid == key);
    bestCol = __shfl(bestCol, (int)__builtin_ctzll(m));
    if (lane == 0) {
        outScore[j] = bestVal;
        outExitCol[j] = bestCol;
    }
}

// tracebackAndThread's walk (PoaGraphTraversals.cpp:252-347) for the jobs whose reads are committed:
// the End move into $, then each visited cell with the move that reached it, recomputed as
// makeAlignmentColumn chose it (candidates in order Start, per predecessor Match/Mismatch then Delete,
// then Extra; strict '>').
// The walk is one lane's chain of dependent loads (a column's predecessor list, then their cells); the job's
// column program -- predStart, predCol and the column bases -- is staged in LDS first (ldsInts ints of dynamic
// LDS; a larger program stays in HBM), so only the score cells are HBM/L2 loads on the chain.
template <class ST>
__global__ __launch_bounds__(64) void k_poa_trace(const PoaJob* __restrict__ jobs, const int* __restrict__ traceJobs,
                                                  int traceBase, PoaPools P, const ST* __restrict__ pool,
                                                  const int* __restrict__ exitCol, uint32_t* __restrict__ steps,
                                                  TraceHeader* __restrict__ heads, int ldsInts)
{
    extern __shared__ int tprog[];
    const int t = traceBase + blockIdx.x;
    const int j = traceJobs[t];
    const PoaJob J = jobs[j];
    const int lane = threadIdx.x;
    const ST* S = pool + J.scoreOff;
    const int I = J.I, stride = J.colStride, mode = J.mode, R = J.rowsPerLane;
    const int ec = exitCol[j];
    const int* vtx = P.vertexOfCol + J.progOff;
    const int nC = J.nCols;
    const int* psG = P.predStart + J.predStartOff;
    const int p0 = psG[0], nPred = psG[nC] - p0;
    const bool staged = nC + 1 + nPred + (nC + 3) / 4 <= ldsInts;
    const int* predStartT = psG;      // absolute indices into predColT
    const int* predColT = P.predCol;
    const uint8_t* baseT = P.base + J.progOff;
    if (staged) {   // rebased: predStart[c] - p0 indexes the staged predCol
        int* ps = tprog;
        int* pc = tprog + nC + 1;
        uint8_t* bs = reinterpret_cast<uint8_t*>(pc + nPred);
        for (int c = lane; c <= nC; c += 64) ps[c] = psG[c] - p0;
        for (int q = lane; q < nPred; q += 64) pc[q] = P.predCol[p0 + q];
        for (int c = lane; c < nC; c += 64) bs[c] = P.base[J.progOff + c];
        predStartT = ps;
        predColT = pc;
        baseT = bs;
    }
    __syncthreads();
    // cell (column c, row i): linear rows, or lane-interleaved for the ring variants
    auto cell = [&](int c, int i) -> int {
        const int x = R ? (i % R) * 64 + i / R : i;
        return (int)S[(long long)c * stride + x];
    };
    // LOCAL: the End move comes from ArgMax of that column (first maximum, VectorL.hpp:66-69)
    int prevRow = I;
    if (mode == kLocal) {
        int bv = kNeg, br = INT_MAX;
        for (int i = lane; i <= I; i += 64) {
            const int v = cell(ec, i);
            if (v > bv) {
                bv = v;
                br = i;
            }
        }
        wave_argmax(bv, br);
        prevRow = br;
    }
    if (lane != 0) return;
    uint32_t* out = steps + J.stepOff;
    const int cap = I + J.nCols + 2;
    int n = 0;
    out[n++] = pack_step(kExit, kEnd);
    int k = ec, i = mode == kLocal ? prevRow : I;
    const uint8_t* rb = P.rowBase + J.readOff;
    const int* predStart = predStartT;
    while (!(k == 0 && i == 0)) {
        if (n >= cap) {
            n = -1;
            break;
        }
        const int ps = predStart[k], pe = predStart[k + 1];
        int best, mv, pv;
        if (i == 0) {
            if (mode != kGlobal) {
                mv = kStart;
                pv = 0;
            } else {
                best = kNeg;
                mv = kInvalid;
                pv = -1;
                for (int p = ps; p < pe; ++p) {
                    const int c = predColT[p];
                    const int cand = cell(c, 0) + kDeleteScore;
                    if (cand > best) {
                        best = cand;
                        pv = c;
                        mv = kDelete;
                    }
                }
            }
        } else {
            if (mode == kLocal) {
                best = 0;
                mv = kStart;
                pv = 0;
            } else {
                best = kNeg;
                mv = kInvalid;
                pv = -1;
            }
            const bool isMatch = rb[i] == baseT[k];
            for (int p = ps; p < pe; ++p) {
                const int c = predColT[p];
                int cand = cell(c, i - 1) + (isMatch ? kMatchScore : kMismatchScore);
                if (cand > best) {
                    best = cand;
                    pv = c;
                    mv = isMatch ? kMatch : kMismatch;
                }
                cand = cell(c, i) + kDeleteScore;
                if (cand > best) {
                    best = cand;
                    pv = c;
                    mv = kDelete;
                }
            }
            const int cand = cell(k, i - 1) + kInsertScore;
            if (cand > best) {
                pv = k;
                mv = kExtra;
            }
        }
        if (mv == kInvalid) {
            n = -1;
            break;
        }
        out[n++] = pack_step(vtx[k], mv);
        if (mv == kStart) i = 0;
        else if (mv != kDelete) i--;
        k = pv;
    }
    heads[t] = TraceHeader{n, prevRow, vtx[ec], 0};
}

// ConsensusCore Sequence.cpp:44-105 (ComplementArray; note N <-> M)
char complement(char c)
{
    switch (c) {
        case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C'; case 'T': return 'A';
        case 'a': return 't'; case 'c': return 'g'; case 'g': return 'c'; case 't': return 'a';
        case 'N': return 'M'; case 'M': return 'N'; case 'n': return 'm'; case 'm': return 'n';
        case '-': return '-';
        case 0: return 3; case 1: return 2; case 2: return 1; case 3: return 0;
    }
    return (char)127;
}

std::string reverse_complement(const std::string& s)
{
    std::string r(s.size(), 0);
    for (size_t k = 0; k < s.size(); ++k) r[s.size() - 1 - k] = complement(s[k]);
    return r;
}

double ms_since(std::chrono::steady_clock::time_point t0)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// k_poa_fill variants: 0 = chunked, linear rows, memory-resident predecessors (any length and width);
// v = 1..12 = LDS ring, lane-interleaved rows, uint16 (LOCAL), R = 4 v rows per lane (at most 3072 rows)
constexpr int kRingVariants = 12;
int fill_variant(int rows, bool wide)
{
    if (wide || rows > 64 * 4 * kRingVariants) return 0;
    return (rows + 255) / 256;
}
int rows_per_lane(int variant, int rows) { return 4 * variant; }
int variant_stride(int variant, int rows)
{
    return variant == 0 ? (rows + kChunkRows - 1) / kChunkRows * kChunkRows : 64 * rows_per_lane(variant, rows);
}
constexpr int kRing = 4;   // columns kept in LDS by the ring variants

template <class ST>
void launch_fill(int variant, int n, int base, hipStream_t s, const PoaJob* jobs, const PoaPools& P, ST* pool,
                 int* score, int* exitCol)
{
    if (n <= 0) return;
    switch (variant) {
        default: hipLaunchKernelGGL(k_poa_fill<ST>, dim3(n), dim3(64), 0, s, jobs, base, P, pool, score, exitCol); break;
    }
}

// the ring variants; lds = the launch's largest ring (kRing columns of 64 * R uint16)
void launch_fill_lds(int variant, int n, int base, size_t lds, hipStream_t s, const PoaJob* jobs, const PoaPools& P,
                     uint16_t* pool, int* score, int* exitCol)
{
    if (n <= 0) return;
#define POA_RING_CASE(V)                                                                                         \
    case V:                                                                                                    \
        hipLaunchKernelGGL((k_poa_fill_lds<4 * V, kRing>), dim3(n), dim3(64), lds, s, jobs, base, P, pool, score, \
                           exitCol);                                                                           \
        break;
    switch (variant) {
        POA_RING_CASE(1) POA_RING_CASE(2) POA_RING_CASE(3) POA_RING_CASE(4) POA_RING_CASE(5) POA_RING_CASE(6)
        POA_RING_CASE(7) POA_RING_CASE(8) POA_RING_CASE(9) POA_RING_CASE(10) POA_RING_CASE(11) POA_RING_CASE(12)
        default: break;
    }
#undef POA_RING_CASE
}

constexpr long long kTraceLdsBytes = 48 * 1024;   // k_poa_trace: staged column program per wave

void check(hipError_t e, const char* what)
{
    if (e != hipSuccess) {
        (void)hipGetLastError();
        throw DeviceError(std::string("POA: ") + what + ": " + hipGetErrorString(e));
    }
}

template <class T>
void upload(DevVec<T>& d, const std::vector<T>& h, hipStream_t s)
{
    d.reserve(std::max<size_t>(h.size(), 1), false);
    if (!h.empty()) check(hipMemcpyAsync(d.ptr, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, s), "upload");
}

}  // namespace

PoaRunner::PoaRunner(int device, int hostThreads) : device_(device)
{
    const int hw = (int)std::thread::hardware_concurrency();
    threads_ = hostThreads > 0 ? hostThreads : std::max(1, std::min(16, hw));
    workers_.reset(new WorkerPool(threads_));
    check(hipSetDevice(device_), "hipSetDevice");
    check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
    for (auto& e : ev_) check(hipEventCreate(&e), "hipEventCreate");
    dPool_.allowVmm = true;
}

PoaRunner::~PoaRunner()
{
    (void)hipSetDevice(device_);
    if (stream_) (void)hipStreamSynchronize(stream_);
    for (auto& e : ev_)
        if (e) (void)hipEventDestroy(e);
    if (stream_) (void)hipStreamDestroy(stream_);
}

void PoaRunner::Align(std::vector<AlignRequest>& reqs, std::vector<AlignResult>* out)
{
    check(hipSetDevice(device_), "hipSetDevice");
    const StreamScope bound(stream_);   // the runner's buffers grow stream-ordered (no device-wide sync)
    const int n = (int)reqs.size();
    out->assign(n, AlignResult());
    if (n == 0) return;

    // ---- host: column programs, then the job layout (sizes -> prefix offsets -> parallel fill)
    auto t0 = std::chrono::steady_clock::now();
    if ((int)prog_.size() < n) prog_.resize(n);
    std::vector<ColumnProgram>& prog = prog_;
    std::vector<std::string> rcRead(n);
    ParallelFor(n, [&](int r) {
        reqs[r].graph->Program(&prog[r]);
        if (reqs[r].orient) rcRead[r] = reverse_complement(reqs[r].read);
    });
    std::vector<int> firstJob(n + 1, 0);
    for (int r = 0; r < n; ++r) firstJob[r + 1] = firstJob[r] + (reqs[r].orient ? 2 : 1);
    const int nJobs = firstJob[n];
    hJobs_.reserve(2 * (size_t)nJobs);   // [0, nJobs): by request; [nJobs, 2 nJobs): a group in launch order
    PoaJob* jobs = hJobs_.ptr;
    std::vector<int> jobReq(nJobs), jobOri(nJobs);
    long long nBase = 0, nPredStart = 0, nPredCol = 0, nExit = 0, nRow = 0;
    for (int r = 0; r < n; ++r) {
        const ColumnProgram& C = prog[r];
        const int nCols = (int)C.vertexOfCol.size();
        for (int o = 0; o < (reqs[r].orient ? 2 : 1); ++o) {
            const int j = firstJob[r] + o;
            PoaJob& J = jobs[j];
            J = PoaJob{};
            J.nCols = nCols;
            J.I = (int)(o ? rcRead[r] : reqs[r].read).size();
            J.mode = reqs[r].mode;
            // uint16 holds LOCAL scores (>= 0, at most 3 per row) of every row up to the padded stride
            J.wide = !(J.mode == kLocal && 3LL * (J.I + 1 + kChunkRows) < 65536);
            J.variant = fill_variant(J.I + 1, J.wide);
            J.rowsPerLane = rows_per_lane(J.variant, J.I + 1);
            J.colStride = variant_stride(J.variant, J.I + 1);
            J.progOff = (int)nBase;
            J.predStartOff = (int)nPredStart;
            J.exitOff = (int)nExit;
            J.nExit = (int)C.exitPredCol.size();
            J.readOff = nRow;
            J.traceSlot = -1;
            nRow += J.colStride + 16;
            jobReq[j] = r;
            jobOri[j] = o;
        }
        nBase += nCols;
        nPredStart += nCols + 1;
        nPredCol += (long long)C.predCol.size();
        nExit += (long long)C.exitPredCol.size();
    }
    hBase_.reserve(nBase);
    hVertex_.reserve(nBase);
    hPredStart_.reserve(nPredStart);
    hPredCol_.reserve(std::max(1LL, nPredCol));
    hExit_.reserve(std::max(1LL, nExit));
    hRowBase_.reserve(nRow);
    std::vector<long long> predColOff(n + 1, 0);
    for (int r = 0; r < n; ++r) predColOff[r + 1] = predColOff[r] + (long long)prog[r].predCol.size();
    ParallelFor(n, [&](int r) {
        const ColumnProgram& C = prog[r];
        const PoaJob& J = jobs[firstJob[r]];
        memcpy(hBase_.ptr + J.progOff, C.base.data(), C.base.size());
        memcpy(hVertex_.ptr + J.progOff, C.vertexOfCol.data(), C.vertexOfCol.size() * sizeof(int));
        for (size_t c = 0; c < C.predStart.size(); ++c)
            hPredStart_.ptr[J.predStartOff + c] = (int)(C.predStart[c] + predColOff[r]);
        if (!C.predCol.empty())
            memcpy(hPredCol_.ptr + predColOff[r], C.predCol.data(), C.predCol.size() * sizeof(int));
        if (!C.exitPredCol.empty())
            memcpy(hExit_.ptr + J.exitOff, C.exitPredCol.data(), C.exitPredCol.size() * sizeof(int));
        for (int o = 0; o < (reqs[r].orient ? 2 : 1); ++o) {
            const PoaJob& Jo = jobs[firstJob[r] + o];
            const std::string& s = o ? rcRead[r] : reqs[r].read;
            uint8_t* rb = hRowBase_.ptr + Jo.readOff;
            rb[0] = 0;
            memcpy(rb + 1, s.data(), s.size());
            memset(rb + 1 + s.size(), 0, Jo.colStride + 16 - 1 - s.size());
        }
    });
    auto upload = [&](auto& d, const auto& h, long long count) {
        d.reserve(std::max(1LL, count), false);
        if (count > 0)
            check(hipMemcpyAsync(d.ptr, h.ptr, count * sizeof(*h.ptr), hipMemcpyHostToDevice, stream_), "upload");
    };
    stats.progMs += ms_since(t0);
    t0 = std::chrono::steady_clock::now();
    upload(dBase_, hBase_, nBase);
    upload(dVertexOfCol_, hVertex_, nBase);
    upload(dPredStart_, hPredStart_, nPredStart);
    upload(dPredCol_, hPredCol_, nPredCol);
    upload(dExitPred_, hExit_, nExit);
    upload(dRowBase_, hRowBase_, nRow);
    const PoaPools pools{dBase_.ptr, dVertexOfCol_.ptr, dPredStart_.ptr, dPredCol_.ptr, dExitPred_.ptr, dRowBase_.ptr};

    size_t budget = 0;
    {
        size_t fr = 0, tot = 0;
        check(hipMemGetInfo(&fr, &tot), "hipMemGetInfo");
        budget = std::min<size_t>((size_t)(0.6 * (double)fr) + dPool_.mapped_bytes(), budget_ ? budget_ : 64ull << 30);
        budget = std::max<size_t>(budget, 64ull << 20);
    }
    auto jobBytes = [&](const PoaJob& J) {
        return ((size_t)J.nCols * J.colStride * (J.wide ? 4 : 2) + 255) / 256 * 256;
    };

    // ---- launch groups: consecutive requests whose jobs fit the score-pool budget together
    std::vector<uint32_t*> stepPtr(n, nullptr);
    std::vector<TraceHeader> heads(n);
    dScore_.reserve(nJobs, false);
    dExitCol_.reserve(nJobs, false);
    hScore_.reserve(nJobs);
    hExitCol_.reserve(nJobs);
    std::vector<std::vector<uint32_t>> keepSteps;   // a group's steps outlive the pinned buffer's next use
    int r0 = 0;
    while (r0 < n) {
        size_t bytes = 0;
        int r1 = r0;
        while (r1 < n) {
            size_t b = 0;
            for (int j = firstJob[r1]; j < firstJob[r1 + 1]; ++j) b += jobBytes(jobs[j]);
            if (r1 > r0 && bytes + b > budget) break;
            bytes += b;
            r1++;
        }
        const int j0 = firstJob[r0], j1 = firstJob[r1], gn = j1 - j0;
        // launch order: uint16 jobs, then int32 jobs, each by fill variant (one range per kernel instantiation)
        std::vector<int> order;
        order.reserve(gn);
        for (int w = 0; w < 2; ++w)
            for (int v = 0; v <= kRingVariants; ++v)
                for (int j = j0; j < j1; ++j)
                    if (jobs[j].wide == w && jobs[j].variant == v) order.push_back(j);
        int nNarrow = 0;
        while (nNarrow < gn && !jobs[order[nNarrow]].wide) nNarrow++;
        size_t off16 = 0, off32 = 0;
        for (int k = 0; k < gn; ++k) {
            PoaJob& J = jobs[order[k]];
            size_t& off = k < nNarrow ? off16 : off32;
            J.scoreOff = (long long)(off / (J.wide ? 4 : 2));
            off += jobBytes(J);
        }
        dPool_.reserve((off16 + off32 + 256 + 7) / 8, false);
        // the group's jobs in launch order: [nJobs, nJobs + gn) of the pinned job array
        PoaJob* gj = hJobs_.ptr + nJobs;
        for (int k = 0; k < gn; ++k) gj[k] = jobs[order[k]];
        dJobs_.reserve(gn, false);
        check(hipMemcpyAsync(dJobs_.ptr, gj, gn * sizeof(PoaJob), hipMemcpyHostToDevice, stream_), "upload jobs");
        uint16_t* pool16 = reinterpret_cast<uint16_t*>(dPool_.ptr);
        int* pool32 = reinterpret_cast<int*>(reinterpret_cast<uint8_t*>(dPool_.ptr) + off16);
        if (profiling) check(hipEventRecord(ev_[0], stream_), "event");
        for (int k = 0; k < gn;) {   // one launch per (width, variant) run
            int e = k;
            while (e < gn && gj[e].wide == gj[k].wide && gj[e].variant == gj[k].variant) e++;
            if (gj[k].wide) {
                launch_fill<int>(0, e - k, k, stream_, dJobs_.ptr, pools, pool32, dScore_.ptr, dExitCol_.ptr);
            } else if (gj[k].variant == 0) {
                launch_fill<uint16_t>(0, e - k, k, stream_, dJobs_.ptr, pools, pool16, dScore_.ptr, dExitCol_.ptr);
            } else {
                size_t lds = 0;
                for (int x = k; x < e; ++x) lds = std::max(lds, (size_t)kRing * gj[x].colStride * sizeof(uint16_t));
                launch_fill_lds(gj[k].variant, e - k, k, lds, stream_, dJobs_.ptr, pools, pool16, dScore_.ptr,
                                dExitCol_.ptr);
            }
            stats.launches++;
            k = e;
        }
        check(hipGetLastError(), "k_poa_fill launch");
        if (profiling) check(hipEventRecord(ev_[1], stream_), "event");
        check(hipMemcpyAsync(hScore_.ptr, dScore_.ptr, gn * sizeof(int), hipMemcpyDeviceToHost, stream_), "d2h");
        check(hipStreamSynchronize(stream_), "k_poa_fill");
        if (profiling) {
            float ms = 0.f;
            check(hipEventElapsedTime(&ms, ev_[0], ev_[1]), "event");
            stats.fillMs += ms;
        }
        for (int k = 0; k < gn; ++k) {
            const PoaJob& J = gj[k];
            (*out)[jobReq[order[k]]].score[jobOri[order[k]]] = (float)hScore_.ptr[k];
            stats.alignments++;
            stats.cells += (long long)J.nCols * (J.I + 1);
            stats.bytes += (double)J.nCols * (J.I + 1) * (J.wide ? 4 : 2);
        }
        // SparsePoa's choice (src/SparsePoa.cpp:112-131) / AddRead's unconditional commit (PoaGraphImpl.cpp:354-369)
        for (int r = r0; r < r1; ++r) {
            AlignResult& R = (*out)[r];
            if (!reqs[r].orient) R.chosen = 0;
            else if (R.score[0] >= R.score[1] && R.score[0] >= reqs[r].minScore) R.chosen = 0;
            else if (R.score[1] >= R.score[0] && R.score[1] >= reqs[r].minScore) R.chosen = 1;
        }
        // traceback of the committed jobs (positions in the group's launch order), uint16 first
        std::vector<int> traceNarrow, traceWide;
        for (int k = 0; k < gn; ++k)
            if ((*out)[jobReq[order[k]]].chosen == jobOri[order[k]]) (k < nNarrow ? traceNarrow : traceWide).push_back(k);
        const int tn = (int)traceNarrow.size(), tw = (int)traceWide.size(), nt = tn + tw;
        if (nt > 0) {
            hTraceJobs_.reserve(nt);
            long long stepTotal = 0;
            std::vector<long long> stepOff(nt);
            for (int t = 0; t < nt; ++t) {
                const int k = t < tn ? traceNarrow[t] : traceWide[t - tn];
                hTraceJobs_.ptr[t] = k;
                gj[k].stepOff = stepTotal;
                stepOff[t] = stepTotal;
                stepTotal += gj[k].I + gj[k].nCols + 2;
            }
            check(hipMemcpyAsync(dJobs_.ptr, gj, gn * sizeof(PoaJob), hipMemcpyHostToDevice, stream_), "upload jobs");
            dTraceJobs_.reserve(nt, false);
            check(hipMemcpyAsync(dTraceJobs_.ptr, hTraceJobs_.ptr, nt * sizeof(int), hipMemcpyHostToDevice, stream_),
                  "upload");
            dSteps_.reserve(stepTotal, false);
            dHeads_.reserve(nt, false);
            if (profiling) check(hipEventRecord(ev_[2], stream_), "event");
            // LDS for the traced jobs' column programs (k_poa_trace), up to kTraceLdsBytes; larger ones walk from HBM
            auto progInts = [&](const std::vector<int>& ks) {
                long long m = 0;
                for (int k : ks) {
                    const PoaJob& Jk = gj[k];
                    const long long np = hPredStart_.ptr[Jk.predStartOff + Jk.nCols] - hPredStart_.ptr[Jk.predStartOff];
                    m = std::max(m, Jk.nCols + 1 + np + (Jk.nCols + 3) / 4);
                }
                return (int)std::min<long long>(m, kTraceLdsBytes / 4);
            };
            if (tn > 0) {
                const int li = progInts(traceNarrow);
                hipLaunchKernelGGL(k_poa_trace<uint16_t>, dim3(tn), dim3(64), (size_t)li * 4, stream_, dJobs_.ptr,
                                   dTraceJobs_.ptr, 0, pools, pool16, dExitCol_.ptr, dSteps_.ptr, dHeads_.ptr, li);
            }
            if (tw > 0) {
                const int li = progInts(traceWide);
                hipLaunchKernelGGL(k_poa_trace<int>, dim3(tw), dim3(64), (size_t)li * 4, stream_, dJobs_.ptr,
                                   dTraceJobs_.ptr, tn, pools, pool32, dExitCol_.ptr, dSteps_.ptr, dHeads_.ptr, li);
            }
            check(hipGetLastError(), "k_poa_trace launch");
            if (profiling) check(hipEventRecord(ev_[3], stream_), "event");
            hSteps_.reserve(stepTotal);
            hHeads_.reserve(nt);
            check(hipMemcpyAsync(hHeads_.ptr, dHeads_.ptr, nt * sizeof(TraceHeader), hipMemcpyDeviceToHost, stream_),
                  "d2h");
            check(hipMemcpyAsync(hSteps_.ptr, dSteps_.ptr, stepTotal * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                 stream_), "d2h");
            check(hipStreamSynchronize(stream_), "k_poa_trace");
            if (profiling) {
                float ms = 0.f;
                check(hipEventElapsedTime(&ms, ev_[2], ev_[3]), "event");
                stats.traceMs += ms;
            }
            const bool last = r1 == n;
            if (!last) keepSteps.emplace_back(hSteps_.ptr, hSteps_.ptr + stepTotal);
            const uint32_t* base = last ? hSteps_.ptr : keepSteps.back().data();
            for (int t = 0; t < nt; ++t) {
                const int k = t < tn ? traceNarrow[t] : traceWide[t - tn];
                const int r = jobReq[order[k]];
                if (hHeads_.ptr[t].nSteps < 1) throw DeviceError("POA traceback did not reach the start vertex");
                heads[r] = hHeads_.ptr[t];
                stepPtr[r] = const_cast<uint32_t*>(base) + stepOff[t];
                stats.traceSteps += heads[r].nSteps;
            }
        }
        r0 = r1;
    }

    stats.deviceMs += ms_since(t0);
    // ---- host: thread the committed reads into their graphs (CommitAdd)
    t0 = std::chrono::steady_clock::now();
    ParallelFor(n, [&](int r) {
        AlignResult& R = (*out)[r];
        if (R.chosen < 0) return;
        const std::string& s = R.chosen ? rcRead[r] : reqs[r].read;
        reqs[r].graph->ThreadTraceback(s, reqs[r].mode, stepPtr[r], heads[r], &R.path);
    });
    stats.threadMs += ms_since(t0);
}

std::string ZmwPoa::FindConsensus(int minCoverage, std::vector<int>* extents, std::vector<int>* cssPath)
{
    const std::vector<int> path = graph.ConsensusPath(kLocal, minCoverage);
    if (cssPath) *cssPath = path;
    if (extents) {
        std::vector<int> pos(graph.NumVertices(), -1);
        for (size_t k = 0; k < path.size(); ++k) pos[path[k]] = (int)k;
        extents->clear();
        for (const std::vector<int>& rp : readPaths) {
            int rs = 0, re = 0, cs = 0, ce = 0;
            bool found = false;
            for (size_t p = 0; p < rp.size(); ++p) {
                const int x = pos[rp[p]];
                if (x < 0) continue;
                if (!found) {
                    cs = x;
                    rs = (int)p;
                    found = true;
                }
                ce = x + 1;
                re = (int)p + 1;
            }
            extents->insert(extents->end(), {rs, re, cs, ce});
        }
    }
    return graph.Sequence(path);
}

namespace {

// One slice [z0, z1) of a PoaBatch on one runner: lock-step read rounds over the slice's ZMWs.
void PoaSlice(PoaRunner& R, const std::vector<std::vector<const std::string*>>& reads, int z0, int z1, long long maxCov,
              int minCov, std::vector<std::string>* consensus, std::vector<std::vector<int>>* keys,
              std::vector<std::vector<char>>* rc, std::vector<std::vector<int>>* extents)
{
    const auto tStart = std::chrono::steady_clock::now();
    const int nz = z1 - z0;
    std::vector<std::unique_ptr<ZmwPoa>> Z(nz);
    for (auto& p : Z) p.reset(new ZmwPoa());
    std::vector<int> next(nz, 0);
    std::vector<long long> cov(nz, 0);
    std::vector<char> done(nz, 0);
    for (int z = 0; z < nz; ++z) (*keys)[z0 + z].assign(reads[z0 + z].size(), -2);
    auto record = [&](int z, int key) {
        (*keys)[z0 + z][next[z]++] = key;
        if (key >= 0 && ++cov[z] >= maxCov) done[z] = 1;
        if (next[z] >= (int)reads[z0 + z].size()) done[z] = 1;
    };
    for (int z = 0; z < nz; ++z)
        if (reads[z0 + z].empty()) done[z] = 1;
    for (;;) {
        std::vector<AlignRequest> reqs;
        std::vector<int> reqZ;
        for (int z = 0; z < nz; ++z) {
            while (!done[z]) {
                const std::string* s = reads[z0 + z][next[z]];
                if (s == nullptr || s->empty()) {   // a dropped or empty read is never added (key -1)
                    record(z, -1);
                } else if (Z[z]->graph.NumReads() == 0) {
                    std::vector<int> path;
                    Z[z]->graph.AddFirstRead(*s, &path);
                    Z[z]->readPaths.push_back(std::move(path));
                    Z[z]->rc.push_back(0);
                    record(z, 0);
                } else {
                    reqs.push_back(AlignRequest{&Z[z]->graph, *s, kLocal, true, 0.0f});
                    reqZ.push_back(z);
                    break;
                }
            }
        }
        if (reqs.empty()) break;
        std::vector<AlignResult> res;
        R.Align(reqs, &res);
        for (size_t q = 0; q < reqs.size(); ++q) {
            const int z = reqZ[q];
            if (res[q].chosen < 0) {
                record(z, -1);
                continue;
            }
            Z[z]->readPaths.push_back(std::move(res[q].path));
            Z[z]->rc.push_back((char)res[q].chosen);
            record(z, (int)Z[z]->readPaths.size() - 1);
        }
    }
    const auto t0 = std::chrono::steady_clock::now();
    R.ParallelFor(nz, [&](int z) {
        const int mc = minCov >= 0 ? minCov : (cov[z] < 5 ? 1 : (int)((cov[z] + 1) / 2 - 1));
        (*consensus)[z0 + z] = Z[z]->readPaths.empty() ? std::string() : Z[z]->FindConsensus(mc, &(*extents)[z0 + z]);
        (*rc)[z0 + z] = Z[z]->rc;
        Z[z].reset();   // the graphs' many small blocks are freed on all host threads
    });
    R.stats.consensusMs += ms_since(t0);
    R.stats.totalMs += ms_since(tStart);
}

}  // namespace

void PoaBatch(const std::vector<PoaRunner*>& runners, const std::vector<std::vector<const std::string*>>& reads,
              long long maxCov, int minCov, std::vector<std::string>* consensus, std::vector<std::vector<int>>* keys,
              std::vector<std::vector<char>>* rc, std::vector<std::vector<int>>* extents)
{
    const int nz = (int)reads.size();
    consensus->assign(nz, std::string());
    keys->assign(nz, std::vector<int>());
    rc->assign(nz, std::vector<char>());
    extents->assign(nz, std::vector<int>());
    // slices of about equal read-base totals, one per runner; small batches use one runner
    const int ns = std::max(1, std::min((int)runners.size(), nz / 64));
    std::vector<long long> pre(nz + 1, 0);
    for (int z = 0; z < nz; ++z) {
        long long b = 0;
        for (const std::string* s : reads[z]) b += s ? (long long)s->size() : 0;
        pre[z + 1] = pre[z] + b;
    }
    std::vector<int> cut(ns + 1, nz);
    cut[0] = 0;
    for (int k = 1; k < ns; ++k)
        cut[k] = (int)(std::lower_bound(pre.begin(), pre.end(), pre[nz] * k / ns) - pre.begin());
    std::vector<std::thread> th;
    std::vector<std::exception_ptr> err(ns);
    for (int k = 0; k < ns; ++k)
        th.emplace_back([&, k] {
            try {
                PoaSlice(*runners[k], reads, cut[k], std::max(cut[k], cut[k + 1]), maxCov, minCov, consensus, keys, rc,
                         extents);
            } catch (...) {
                err[k] = std::current_exception();
            }
        });
    for (auto& t : th) t.join();
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
}

}  // namespace poa
}  // namespace pbccs
