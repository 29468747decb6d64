// pbccs_amd/csrc/coop_chain.hpp -- wavefront primitives of the cooperative band recursions, shared by the
// fill (fill_coop.hip) and the checkpoint-replay scorer (k_score_ckpt, arrow_kernels.hip): nibble-packed bases, the gfx9 DPP
// shift / prefix-max / broadcast helpers of a G-lane group, and the in-column insertion chain
// x_i = (m_i + x_{i-1} k_i) + d_i in the reference's operation order (SimpleRecursor.cpp:117-150).
#pragma once

#include "arrow_device.hpp"

namespace pbccs {
namespace coop {

constexpr int kCtxDoubles = 9 * kCtxStride;   // 45
constexpr int kBaseOther = 4;                 // nibble code of a non-ACGT read base (never matches)

__device__ __forceinline__ int base_code(char c)
{
    return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : c == 'T' ? 3 : kBaseOther;
}

__device__ __forceinline__ int nib(const unsigned* w, int x) { return (w[x >> 3] >> ((x & 7) << 2)) & 15; }

// ContextParameters::GetParametersForContext slot from two template base codes (ACGT only).
__device__ __forceinline__ int ctx_code(int b1, int b2) { return b1 == b2 ? b2 : 4 + b2; }

// --- cross-lane primitives (gfx9 DPP) -------------------------------------------------------------
template <int CTRL, int ROWMASK, bool BOUND>
__device__ __forceinline__ double dpp_d(double old, double x)
{
    const int xl = __double2loint(x), xh = __double2hiint(x);
    const int ol = __double2loint(old), oh = __double2hiint(old);
    const int rl = __builtin_amdgcn_update_dpp(ol, xl, CTRL, ROWMASK, 0xF, BOUND);
    const int rh = __builtin_amdgcn_update_dpp(oh, xh, CTRL, ROWMASK, 0xF, BOUND);
    return __hiloint2double(rh, rl);
}

// value of lane l-1 of the group; lane 0 receives `first`
template <int G>
__device__ __forceinline__ double shift_up(double x, double first)
{
    if constexpr (G == 16) {
        return dpp_d<0x111, 0xF, false>(first, x);   // row_shr:1
    } else {
        return dpp_d<0x138, 0xF, false>(first, x);   // wave_shr:1
    }
}

// inclusive prefix maximum over the group's lanes (values >= 0)
template <int G>
__device__ __forceinline__ double prefix_max(double x)
{
    x = fmax(x, dpp_d<0x111, 0xF, true>(0.0, x));
    x = fmax(x, dpp_d<0x112, 0xF, true>(0.0, x));
    x = fmax(x, dpp_d<0x114, 0xF, true>(0.0, x));
    x = fmax(x, dpp_d<0x118, 0xF, true>(0.0, x));
    if constexpr (G == 64) {
        x = fmax(x, dpp_d<0x142, 0xA, false>(0.0, x));   // row_bcast:15
        x = fmax(x, dpp_d<0x143, 0xC, false>(0.0, x));   // row_bcast:31
    }
    return x;
}

template <int G>
struct Group {
    int lane;   // lane within the group
    int base;   // first wavefront lane of the group
    __device__ __forceinline__ unsigned long long bits(bool p) const
    {
        const unsigned long long m = __ballot(p);
        if constexpr (G == 64) return m;
        else return (m >> base) & ((1ull << G) - 1);
    }
    // value of group lane `src` (uniform across the group).  G = 64: the group is the wavefront and src is
    // wave-uniform at every call site (a loop counter, a ballot's first set bit, a constant), so the value
    // moves through an SGPR (v_readlane, a few cycles) instead of an LDS permute (ds_bpermute) -- this sits
    // on the insertion chain's critical path once per 64-row chunk.
    __device__ __forceinline__ double bcast(double x, int src) const
    {
        if constexpr (G == 64) {
            const int lo = __builtin_amdgcn_readlane(__double2loint(x), src);
            const int hi = __builtin_amdgcn_readlane(__double2hiint(x), src);
            return __hiloint2double(hi, lo);
        } else {
            return __shfl(x, src, G);
        }
    }
    __device__ __forceinline__ int bcast(int x, int src) const
    {
        if constexpr (G == 64) {
            return __builtin_amdgcn_readlane(x, src);
        } else {
            return __shfl(x, src, G);
        }
    }
    // value of the group's last lane: G = 16 is one DPP row, whose lane 15 a single v_mov_b64 row_newbcast:15
    // hands to the whole row (instead of two LDS permutes on the chunk-to-chunk carry path)
    __device__ __forceinline__ double bcast_last(double x) const
    {
        if constexpr (G == 64) {
            return bcast(x, 63);
        } else {
            const long long r = __builtin_amdgcn_update_dpp(0ll, __double_as_longlong(x), 0x15F, 0xF, 0xF, false);
            return __longlong_as_double(r);
        }
    }
};

// The in-column insertion chain x_i = (m_i + x_{i-1} k_i) + d_i over the G rows of a chunk (lane l = row
// l; lane 0's predecessor is `carry`), in the reference's operation order (SimpleRecursor.cpp:117-150):
// G serial shift-by-one DPP steps; after step q lanes <= q hold their final value.  (Jacobi sweeps for
// G = 64 -- exact by fixed-point uniqueness -- measured 157 ms against 67 ms per tall fill and were
// removed)
template <int G>
__device__ __forceinline__ double insertion_chain(double m, double k, double d, double carry)
{
    double x = 0.0, up = carry;   // lane 0's `up` stays the carry: DPP leaves it untouched
#pragma unroll
    for (int q = 0; q < G; ++q) {
        up = shift_up<G>(x, up);
        x = (m + up * k) + d;
    }
    return x;
}

// The chain over a chunk of G x R rows, R consecutive rows per lane (lane l holds rows l R .. l R + R - 1):
// in phase p lane p takes its predecessor from lane p - 1 with one DPP hand-off and runs its R rows in
// registers, so the dependent path per row is mul + add + add without a DPP move (tools/ubench/chain_step.hip,
// 29.3 cycles per row with a hand-off per row, 17.6 / 15.6 with one per 4 / 8 rows).  Every
// row keeps the reference's operation order.  After phase p lanes <= p hold their final values.  From
// `firstLane` on (the first lane whose rows the reference loop may stop at; >= G: none) every kCheckPhases
// phases `maybe_stop(x)` -- a conservative form of the loop's stop test over the final lanes -- may end the
// chain early; the caller's exact test then finds the same stop row.  Blocks of phases below `startLane` are
// skipped: the caller passes the first lane with a non-zero input when the carry is zero (every row before it
// is exactly zero, and so is its predecessor), 0 otherwise -- the leading zero rows of tall bands, a quarter of
// their cells at 2 kb (oracle), at 16-row granularity instead of whole chunks.
// G < 64 (several reads per wavefront, one per G-lane group): the skip and the exit are wave decisions -- a
// block is skipped when every active group's startLane passes it, the chain ends when every active group has a
// final stop (a group that keeps running past its own stop recomputes its final lanes to the same values).
template <int G, int R, class MaybeStop>
__device__ __forceinline__ void insertion_chain_rows(const double (&m)[R], const double (&k)[R], const double (&d)[R],
                                                     double carry, double (&x)[R], int firstLane, bool exitOn,
                                                     int startLane, MaybeStop maybe_stop)
{
    constexpr int kCheckPhases = R >= 16 ? 1 : 16 / R;   // a check every 16 rows
    double up = carry;   // lane 0's `up` stays the carry: DPP leaves it untouched
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = 0.0;
    const int check0 = exitOn ? max(firstLane, 0) : G;
#pragma unroll
    for (int p = 0; p < G; p += kCheckPhases) {
        if (G == 64 ? p + kCheckPhases <= startLane : __ballot(p + kCheckPhases > startLane) == 0)
            continue;   // every lane of the block is exactly zero
#pragma unroll
        for (int u = 0; u < kCheckPhases; ++u) {
            up = shift_up<G>(x[R - 1], up);
            x[0] = (m[0] + up * k[0]) + d[0];
#pragma unroll
            for (int r = 1; r < R; ++r) x[r] = (m[r] + x[r - 1] * k[r]) + d[r];
        }
        const int last = p + kCheckPhases - 1;   // lanes <= last are final
        if (G == 64) {
            if (last >= check0 && last < G - 1) {
                const unsigned long long st = maybe_stop(x) & ((2ull << last) - 1);
                if (st) return;
            }
        } else if (last < G - 1 && __ballot(last >= check0) != 0) {
            const unsigned long long sb = maybe_stop(x);   // cross-lane: every active lane takes part
            const bool done = last >= check0 && (sb & ((2ull << last) - 1)) != 0;
            if (__ballot(!done) == 0) return;
        }
    }
}

// G = 64 serial chain with an early exit: after step q, lanes <= q hold their final value.  From lane
// `first` on (the first lane the reference loop may stop at; >= G: none in this chunk) the chain is checked
// every 8 steps with `maybe_stop`, a conservative form of the loop's stop test (it never reports a lane the
// exact test continues at).  Once a lane <= q would stop, every lane past it is discarded by the caller, so
// the remaining steps are skipped; the caller's exact test then finds the same stop lane among the final
// lanes.  Narrow passes of tall reads (the first alpha / beta, bands of ~15-30 rows) and the last chunk of a
// tall column no longer pay the full 64 steps.
template <class MaybeStop>
__device__ __forceinline__ double insertion_chain64_exit(double m, double k, double d, double carry, int first,
                                                         MaybeStop maybe_stop, int startLane = 0)
{
    double x = 0.0, up = carry;
    int q = 0;
    const int check0 = max(first, 0) + 3;   // first check: a few rows past the first possible stop
    if (check0 < 63 || startLane >= 8) {
        // fully unrolled like the check-free path below (a rolled block loop measured 4% slower end to end,
        // profiles/r2h17_code_size_ab): the checks sit at fixed positions and only their branch is dynamic
        // (blocks below startLane: all-zero rows, see insertion_chain_rows)
#pragma unroll
        for (q = 0; q < 64; q += 8) {
            if (q + 8 <= startLane) continue;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                up = shift_up<64>(x, up);
                x = (m + up * k) + d;
            }
            const int last = q + 7;   // lanes <= last are final
            if (last >= check0 && last < 63) {
                const unsigned long long st = maybe_stop(x) & ((2ull << last) - 1);
                if (st) return x;
            }
        }
        return x;
    }
#pragma unroll
    for (int s = 0; s < 64; ++s) {
        up = shift_up<64>(x, up);
        x = (m + up * k) + d;
    }
    return x;
}

// ---- reassociated chain (the certified fast path of the tall fills) -----------------------
// x_i = k_i x_{i-1} + c_i with c_i = m_i + d_i is an affine recurrence: each lane folds its R rows into one map
// x -> A x + B, a Kogge-Stone scan over the 64 lanes composes the maps of the lanes below (6 DPP levels: row_shr
// 1/2/4/8, row_bcast 15/31, as prefix_max), and each lane applies the exclusive prefix to the chunk's carry and
// then runs its own R rows.  A chunk costs ~6 dependent levels instead of 64 hand-offs.  The sums are
// reassociated, so the values are not the reference's bit for bit: every value is within a tracked relative
// bound of it (all terms are non-negative), and the caller certifies each decision against that bound.
// compose (A, B) := (A, B) o (Av, Bv), i.e. x -> A (Av x + Bv) + B; lanes without a source see the identity (1, 0)
template <int CTRL, int ROWMASK>
__device__ __forceinline__ void affine_step(double& A, double& B)
{
    const double Av = dpp_d<CTRL, ROWMASK, false>(1.0, A);
    const double Bv = dpp_d<CTRL, ROWMASK, false>(0.0, B);
    B = A * Bv + B;
    A = A * Av;
}
// inclusive scan over the wavefront's 64 lanes: lane l ends with the composition of lanes 0..l
__device__ __forceinline__ void affine_scan64(double& A, double& B)
{
    affine_step<0x111, 0xF>(A, B);   // row_shr:1
    affine_step<0x112, 0xF>(A, B);   // row_shr:2
    affine_step<0x114, 0xF>(A, B);   // row_shr:4
    affine_step<0x118, 0xF>(A, B);   // row_shr:8
    affine_step<0x142, 0xA>(A, B);   // row_bcast:15 (rows 1, 3)
    affine_step<0x143, 0xC>(A, B);   // row_bcast:31 (rows 2, 3)
}
// The chunk's R x 64 rows by the scan: x[r] of lane l is row l R + r; lane 0's predecessor is `carry`.
template <int R>
__device__ __forceinline__ void scan_chain64(const double (&m)[R], const double (&k)[R], const double (&d)[R],
                                             double carry, double (&x)[R])
{
    double c[R];
#pragma unroll
    for (int r = 0; r < R; ++r) c[r] = m[r] + d[r];
    double A = k[0], B = c[0];
#pragma unroll
    for (int r = 1; r < R; ++r) {
        B = k[r] * B + c[r];
        A = k[r] * A;
    }
    affine_scan64(A, B);
    // exclusive prefix: the map of the lanes below (lane 0: the identity)
    const double Ae = dpp_d<0x138, 0xF, false>(1.0, A);   // wave_shr:1
    const double Be = dpp_d<0x138, 0xF, false>(0.0, B);
    double up = Ae * carry + Be;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        x[r] = k[r] * up + c[r];
        up = x[r];
    }
}

}  // namespace coop
}  // namespace pbccs
