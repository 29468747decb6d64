// pbccs_amd/csrc/quiver_device.hpp -- device side of the Quiver engine.
//
// ConsensusCore's Quiver family scores reads in log space (FP32) with per-base QV features.  ccs never
// calls it; it is the second kernel family the north_star names.  Execution model: one
// lane owns one read's FillAlphaBeta, or one (mutation, read) ScoreMutation, column-serial in the
// reference's operation order (-ffp-contract=off), so every cell is bit-identical to the SSE recursor:
// each _mm_*_ps of the reference is an IEEE single-precision operation per lane.
//
// Band storage: a matrix keeps, per column, its used row range and an offset into a float arena; cells
// outside the used range read -FLT_MAX, which is exactly what the reference's SparseVector<lvalue<float>>
// returns (columns are cleared on StartEditingColumn and only used rows are ever set).  Each matrix has
// two arenas: a pass writes one while its self-hint (RangeGuide on the previous pass) reads the other.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pbccs {
namespace quiver {

constexpr float kNegInf = -3.402823466e+38f;   // -FLT_MAX (QvEvaluator.hpp:64)
constexpr int kMerge = 8;                     // Move::MERGE (QuiverConfig.hpp:50-59)
constexpr int kMaxFlipFlops = 5;              // detail/RecursorBase.cpp:51
// ALPHA_BETA_MISMATCH_TOLERANCE 0.2 and REBANDING_THRESHOLD 0.04 (detail/RecursorBase.cpp:52-53) are
// double literals in the reference; quiver_kernels.hip uses them as such.

// kQTall: a column outgrew k_qfill_coop's band-height LDS ring; the host reruns the read with a full-height ring
enum QFillStatus : int { kQOk = 0, kQMismatch = 1, kQOverflow = 2, kQBad = 3, kQMemFail = 4, kQTall = 5 };

// QvModelParams + QuiverConfig fields the recursion reads (QuiverConfig.hpp:79-176)
struct QParams {
    float Match, Mismatch, MismatchS, Branch, BranchS, DeletionN, DeletionWithTag, DeletionWithTagS, Nce, NceS;
    float Merge[4], MergeS[4];
    float scoreDiff, fastThreshold, addThreshold;
    int moves;
    int sumProduct;
    int simple;   // SimpleRecursor fills / extend / link (else SseRecursor)
    int dense;    // DenseMatrixF storage: column j at j * (I + 1), AllocatedEntries = (I + 1)(J + 1)
};

// ---- Cephes exp_ps / log_ps (detail/sse_mathfun.h:167-350), one lane -----------------------------------
__device__ __forceinline__ float maxps(float a, float b) { return a > b ? a : b; }   // MAXPS operand rule
__device__ __forceinline__ float minps(float a, float b) { return a < b ? a : b; }

__device__ __forceinline__ float cephes_log(float x)
{
    const bool invalid = x <= 0.0f;
    const bool zero = x == 0.0f;
    x = maxps(x, __uint_as_float(0x00800000u));
    int e0 = (int)(__float_as_uint(x) >> 23);
    x = __uint_as_float(__float_as_uint(x) & ~0x7f800000u);
    x = __uint_as_float(__float_as_uint(x) | __float_as_uint(0.5f));
    e0 = e0 - 0x7f;
    float e = (float)e0;
    e = e + 1.0f;
    const bool lt = x < 0.707106781186547524f;
    const float t0 = lt ? x : 0.0f;
    x = x - 1.0f;
    e = e - (lt ? 1.0f : 0.0f);
    x = x + t0;
    const float z = x * x;
    float y = 7.0376836292E-2f;
    y = y * x; y = y + -1.1514610310E-1f;
    y = y * x; y = y + 1.1676998740E-1f;
    y = y * x; y = y + -1.2420140846E-1f;
    y = y * x; y = y + 1.4249322787E-1f;
    y = y * x; y = y + -1.6668057665E-1f;
    y = y * x; y = y + 2.0000714765E-1f;
    y = y * x; y = y + -2.4999993993E-1f;
    y = y * x; y = y + 3.3333331174E-1f;
    y = y * x;
    y = y * z;
    float t = e * -2.12194440e-4f;
    y = y + t;
    t = z * 0.5f;
    y = y - t;
    t = e * 0.693359375f;
    x = x + y;
    x = x + t;
    if (invalid) x = __uint_as_float(0xffffffffu);
    if (zero) x = -__builtin_inff();
    return x;
}

__device__ __forceinline__ float cephes_exp(float x)
{
    x = minps(x, 88.3762626647949f);
    x = maxps(x, -88.3762626647949f);
    float fx = x * 1.44269504088896341f;
    fx = fx + 0.5f;
    int e0 = (int)fx;   // cvttps: truncation
    float t = (float)e0;
    fx = t - ((t > fx) ? 1.0f : 0.0f);
    t = fx * 0.693359375f;
    float z = fx * -2.12194440e-4f;
    x = x - t;
    x = x - z;
    z = x * x;
    float y = 1.9875691500E-4f;
    y = y * x; y = y + 1.3981999507E-3f;
    y = y * x; y = y + 8.3334519073E-3f;
    y = y * x; y = y + 4.1665795894E-2f;
    y = y * x; y = y + 1.6666665459E-1f;
    y = y * x; y = y + 5.0000001201E-1f;
    y = y * z;
    y = y + x;
    y = y + 1.0f;
    e0 = (int)fx;
    e0 = e0 + 0x7f;
    const float pow2n = __uint_as_float((unsigned)e0 << 23);
    return y * pow2n;
}

// logAdd4 / logAdd (detail/SseMath.hpp:66-88)
__device__ __forceinline__ float log_add(float a, float b)
{
    const float mx = maxps(a, b), mn = minps(a, b);
    const float d = mn - mx;
    return mx + cephes_log(1.0f + cephes_exp(d));
}

// Combiner::Combine (std::max / logAdd) and Combine4 (_mm_max_ps / logAdd4), detail/Combiner.hpp:53-81
__device__ __forceinline__ float comb(bool sp, float x, float y) { return sp ? log_add(x, y) : (x < y ? y : x); }
__device__ __forceinline__ float comb4(bool sp, float x, float y) { return sp ? log_add(x, y) : maxps(x, y); }

// ---- read features + evaluator (QvEvaluator.hpp:150-207) ------------------------------------------------
struct QRead {
    const char* seq;
    const float* ins;
    const float* subs;
    const float* del;
    const float* tag;     // DelTag as float(char)
    const float* merge;
    int I;
};

// The template seen by a recursion: `len` bases of the strand template starting at `base`, optionally with
// one edit (the mutated window of ScoreMutation; the reference materialises newTpl, MutationScorer.cpp:117).
struct QTpl {
    const char* base;
    int len;             // length of the (possibly edited) template
    int editPos = -1;    // position of the edit in the unedited template (-1: none)
    int editType = 0;    // 0 insertion, 1 deletion, 2 substitution (single base)
    int editBase = 0;    // a char (int: byte-sized members of a by-value struct were kept in scratch)
    __device__ __forceinline__ char at(int j) const   // std::string semantics: '\0' at j == len
    {
        if (j >= len) return '\0';
        if (editPos < 0 || j < editPos) return base[j];
        if (editType == 2) return j == editPos ? (char)editBase : base[j];
        if (editType == 0) return j == editPos ? (char)editBase : base[j - 1];
        return base[j + 1];
    }
};

__device__ __forceinline__ int tpl_code(char b) { return b == 'A' ? 0 : b == 'C' ? 1 : b == 'G' ? 2 : 3; }

struct QEval {
    QRead r;   // by value: a pointer to a kernel-local QRead would keep it in scratch
    const QParams* p;
    QTpl t;
    __device__ __forceinline__ int I() const { return r.I; }
    __device__ __forceinline__ int J() const { return t.len; }
    __device__ __forceinline__ float Inc(int i, int j) const
    {
        return (r.seq[i] == t.at(j)) ? p->Match : p->Mismatch + p->MismatchS * r.subs[i];
    }
    __device__ __forceinline__ float Del(int i, int j) const   // pinStart = pinEnd = true
    {
        const float tb = (float)t.at(j);
        return (i < r.I && tb == r.tag[i]) ? p->DeletionWithTag + p->DeletionWithTagS * r.del[i] : p->DeletionN;
    }
    __device__ __forceinline__ float Extra(int i, int j) const
    {
        return (j < t.len && r.seq[i] == t.at(j)) ? p->Branch + p->BranchS * r.ins[i] : p->Nce + p->NceS * r.ins[i];
    }
    __device__ __forceinline__ float Merge(int i, int j) const
    {
        const char a = t.at(j), b = t.at(j + 1), s = r.seq[i];
        if (!(s == a && s == b)) return kNegInf;
        const int k = tpl_code(a);
        return p->Merge[k] + p->MergeS[k] * r.merge[i];
    }
};

// ---- band matrix --------------------------------------------------------------------------------------
// One pass of one matrix lives in one arena: per column range[j] = used rows, off[j] = arena offset of
// row range[j].x.  Get outside the used range = -FLT_MAX.
struct QBand {
    int2* range;
    int* off;
    float* val;
    long long cap;   // floats in the arena
    int cols;
    __device__ __forceinline__ float Get(int i, int j) const
    {
        const int2 r = range[j];
        if (i < r.x || i >= r.y) return kNegInf;
        const long long k = (long long)off[j] + (i - r.x);
        return k < cap ? val[k] : kNegInf;   // past the arena only in overflow (count-only) mode
    }
    __device__ __forceinline__ bool Empty(int j) const { const int2 r = range[j]; return r.x >= r.y; }
};

// SparseVector<float> allocation bookkeeping (SparseVector-inl.hpp:48-141, 171-186, 250-255) for
// AllocatedEntries = storage_.capacity(), as libstdc++'s vector grows it: resize(n) above the capacity
// allocates max(2 * size, n); vector(n).swap() gives capacity n.  Only the AddRead memory gate reads it.
struct QAlloc {
    int ab, ae, size, capacity;
};

__device__ __forceinline__ void vec_resize(QAlloc& a, int n)
{
    if (n > a.capacity) a.capacity = max(2 * a.size, n);
    a.size = n;
}

__device__ __forceinline__ void alloc_start(QAlloc& a, bool exists, int hb, int he, int rows)
{
    const int nb = max(hb - 8, 0), ne = min(he + 8, rows);
    if (!exists) {
        a.size = a.capacity = ne - nb;
    } else if ((ne - nb) > (a.ae - a.ab)) {
        vec_resize(a, ne - nb);
    } else if ((ne - nb) < (int)(0.8 * (a.ae - a.ab))) {
        a.size = a.capacity = ne - nb;
    }
    a.ab = nb;
    a.ae = ne;
}

__device__ __forceinline__ void alloc_set(QAlloc& a, int i, int rows)
{
    if (i >= a.ab && i < a.ae) return;
    const int nb = max(min(i - 8, a.ab), 0);
    const int ne = min(max(i + 8, a.ae), rows);
    vec_resize(a, ne - nb);
    a.ab = nb;
    a.ae = ne;
}

}  // namespace quiver
}  // namespace pbccs
