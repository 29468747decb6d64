// =============================================================================
//  oracle/quiver_oracle.cpp  --  TEST INFRASTRUCTURE ONLY
// -----------------------------------------------------------------------------
//  CPU restatement of ConsensusCore's *Quiver* family:
//  QvEvaluator move scores, the SSE recursor's banded log-space FP32 fills with
//  its 4-row blocks and serial Extra cascade, LinkAlphaBeta / ExtendAlpha,
//  SimpleRecursor::ExtendBeta, the FillAlphaBeta flip-flop controller, the
//  Quiver MutationScorer / MultiReadMutationScorer and the Cephes logAdd of the
//  sum-product combiner.  Only tests/ may load it; the product never does.
//
//  Parity pin: the reference's own Quiver gtest expectations
//  (ConsensusCore/src/Tests/TestRecursors.cpp, TestMutationScorer.cpp,
//  TestMultiReadMutationScorer.cpp, TestQvEvaluator.cpp with
//  ParameterSettings.cpp's TestingParams), recorded in
//  tests/golden/quiver_kats.json by tests/golden/make_golden.py.
//
//  The SSE code is restated lane by lane: every _mm_*_ps is an IEEE single
//  operation per lane, so a scalar loop in the same operation order is
//  bit-identical (build with -ffp-contract=off).  Reads of cells outside a
//  column's allocation read -FLT_MAX (lvalue<float>, LValue.hpp:46-80).
// =============================================================================
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <list>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "oracle_common.hpp"

namespace qorc {
using orc::DEL;
using orc::FWD;
using orc::INS;
using orc::Mut;
using orc::REV;
using orc::SUB;

static const float NEG_INF = -FLT_MAX;   // QvEvaluator.hpp:64, SseRecursor.cpp:59

struct AlphaBetaMismatch {};

// ---------------------------------------------------------------- Cephes SSE math (sse_mathfun.h)
static inline float as_float(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
static inline uint32_t as_bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
static inline float maxps(float a, float b) { return a > b ? a : b; }   // MAXPS: second operand unless a > b
static inline float minps(float a, float b) { return a < b ? a : b; }   // MINPS: second operand unless a < b

// log_ps (sse_mathfun.h:167-258), one lane
static float log_ps1(float x)
{
    const bool invalid = x <= 0.0f;
    const bool zero = x == 0.0f;
    x = maxps(x, as_float(0x00800000u));                 // cut off denormals (min_norm_pos)
    int32_t emm0 = (int32_t)(as_bits(x) >> 23);          // _mm_srli_epi32
    x = as_float(as_bits(x) & ~0x7f800000u);             // inv_mant_mask
    x = as_float(as_bits(x) | as_bits(0.5f));
    emm0 = emm0 - 0x7f;
    float e = (float)emm0;
    e = e + 1.0f;
    const bool mask = x < (float)0.707106781186547524;   // cephes_SQRTHF
    const float tmp0 = mask ? x : 0.0f;
    x = x - 1.0f;
    e = e - (mask ? 1.0f : 0.0f);
    x = x + tmp0;
    const float z = x * x;
    float y = (float)7.0376836292E-2;
    y = y * x; y = y + (float)-1.1514610310E-1;
    y = y * x; y = y + (float)1.1676998740E-1;
    y = y * x; y = y + (float)-1.2420140846E-1;
    y = y * x; y = y + (float)+1.4249322787E-1;
    y = y * x; y = y + (float)-1.6668057665E-1;
    y = y * x; y = y + (float)+2.0000714765E-1;
    y = y * x; y = y + (float)-2.4999993993E-1;
    y = y * x; y = y + (float)+3.3333331174E-1;
    y = y * x;
    y = y * z;
    float tmp = e * (float)-2.12194440e-4;               // cephes_log_q1
    y = y + tmp;
    tmp = z * 0.5f;
    y = y - tmp;
    tmp = e * (float)0.693359375;                        // cephes_log_q2
    x = x + y;
    x = x + tmp;
    if (invalid) x = as_float(as_bits(x) | 0xffffffffu);
    if (zero) x = -std::numeric_limits<float>::infinity();
    return x;
}

// exp_ps (sse_mathfun.h:275-350, USE_SSE2 path), one lane
static float exp_ps1(float x)
{
    x = minps(x, 88.3762626647949f);
    x = maxps(x, -88.3762626647949f);
    float fx = x * (float)1.44269504088896341;           // cephes_LOG2EF
    fx = fx + 0.5f;
    int32_t emm0 = (int32_t)fx;                          // _mm_cvttps_epi32 (truncation)
    float tmp = (float)emm0;
    const float mask = (tmp > fx) ? 1.0f : 0.0f;
    fx = tmp - mask;
    tmp = fx * (float)0.693359375;                       // cephes_exp_C1
    float z = fx * (float)-2.12194440e-4;                // cephes_exp_C2
    x = x - tmp;
    x = x - z;
    z = x * x;
    float y = (float)1.9875691500E-4;
    y = y * x; y = y + (float)1.3981999507E-3;
    y = y * x; y = y + (float)8.3334519073E-3;
    y = y * x; y = y + (float)4.1665795894E-2;
    y = y * x; y = y + (float)1.6666665459E-1;
    y = y * x; y = y + (float)5.0000001201E-1;
    y = y * z;
    y = y + x;
    y = y + 1.0f;
    emm0 = (int32_t)fx;
    emm0 = emm0 + 0x7f;
    emm0 = (int32_t)((uint32_t)emm0 << 23);
    const float pow2n = as_float((uint32_t)emm0);
    y = y * pow2n;
    return y;
}

// logAdd4 / logAdd (detail/SseMath.hpp:66-88), one lane
static float logAdd(float a, float b)
{
    const float mx = maxps(a, b);
    const float mn = minps(a, b);
    const float diff = mn - mx;
    return mx + log_ps1(1.0f + exp_ps1(diff));
}

// detail/Combiner.hpp:53-81.  Scalar Combine = std::max / logAdd; Combine4 = _mm_max_ps / logAdd4.
struct Combiner {
    bool sumProduct = false;
    float C(float x, float y) const { return sumProduct ? logAdd(x, y) : std::max(x, y); }
    float C4(float x, float y) const { return sumProduct ? logAdd(x, y) : maxps(x, y); }
};

// ---------------------------------------------------------------- configuration (QuiverConfig.hpp:50-249)
enum { INCORPORATE = 1, EXTRA = 2, DELETE = 4, MERGE = 8, ALL_MOVES = 15 };

struct QvModelParams {
    std::string chemistry = "*", model = "test";
    float Match = 0, Mismatch = 0, MismatchS = 0, Branch = 0, BranchS = 0, DeletionN = 0, DeletionWithTag = 0,
          DeletionWithTagS = 0, Nce = 0, NceS = 0;
    float Merge[4] = {0, 0, 0, 0}, MergeS[4] = {0, 0, 0, 0};
};

struct QuiverConfig {
    QvModelParams qv;
    int moves = ALL_MOVES;
    float scoreDiff = 12.5f;   // BandingOptions(diagCross, scoreDiff): diagCross is ignored
    float fastScoreThreshold = -12.5f;
    float addThreshold = 1.0f;
    bool sumProduct = false;   // SparseSseQvRecursor (Viterbi) or SparseSseQvSumProductRecursor
    bool simple = false;       // SimpleRecursor family (SimpleQvRecursor, SparseSimpleQvRecursor)
    bool dense = false;        // DenseMatrixF storage (SimpleQvRecursor, SseQvRecursor)
};

// ---------------------------------------------------------------- read features (Features.hpp:52-114)
struct QvRead {
    std::string seq;
    std::vector<float> ins, subs, del, delTag, merge;   // delTag holds the tag base as float(char)
    std::string chemistry = "*";
};

// ---------------------------------------------------------------- evaluator (QvEvaluator.hpp:90-317)
static int EncodeTplBase(char b)   // QvEvaluator.hpp:72-83 (M/N are test-only codes; not indexed here)
{
    switch (b) {
        case 'A': return 0; case 'C': return 1; case 'G': return 2; case 'T': return 3;
    }
    throw std::invalid_argument("template base");
}

struct Evaluator {   // holds its read and params by value, as QvEvaluator does (read_, params_)
    QvRead rd;
    QvModelParams pm;
    const QvRead* r = &rd;
    const QvModelParams* p = &pm;
    Evaluator() {}
    Evaluator(const Evaluator& o) : rd(o.rd), pm(o.pm), tpl(o.tpl), pinStart(o.pinStart), pinEnd(o.pinEnd) {}
    Evaluator& operator=(const Evaluator& o)
    {
        rd = o.rd;
        pm = o.pm;
        tpl = o.tpl;
        pinStart = o.pinStart;
        pinEnd = o.pinEnd;
        return *this;
    }
    std::string tpl;
    bool pinStart = true, pinEnd = true;
    int I() const { return (int)r->seq.size(); }
    int J() const { return (int)tpl.size(); }
    char T(int j) const { return j < J() ? tpl[j] : '\0'; }   // std::string's terminator at j == J
    bool IsMatch(int i, int j) const { return r->seq[i] == tpl[j]; }
    float Inc(int i, int j) const { return IsMatch(i, j) ? p->Match : p->Mismatch + p->MismatchS * r->subs[i]; }
    float Del(int i, int j) const
    {
        if ((!pinStart && i == 0) || (!pinEnd && i == I())) return 0.0f;
        const float tplBase = (float)tpl[j];
        return (i < I() && tplBase == r->delTag[i]) ? p->DeletionWithTag + p->DeletionWithTagS * r->del[i]
                                                     : p->DeletionN;
    }
    float Extra(int i, int j) const
    {
        return (j < J() && IsMatch(i, j)) ? p->Branch + p->BranchS * r->ins[i] : p->Nce + p->NceS * r->ins[i];
    }
    float Merge(int i, int j) const
    {
        if (!(r->seq[i] == tpl[j] && r->seq[i] == tpl[j + 1])) return -FLT_MAX;
        const int b = EncodeTplBase(tpl[j]);
        return p->Merge[b] + p->MergeS[b] * r->merge[i];
    }
    // The SSE forms (Inc4/Del4/Extra4/Merge4, :213-302) equal the scalar forms lane by lane: the same
    // float compare of read base and template base and the same AFFINE4 = offset + slope * qv.
};

// ---------------------------------------------------------------- band matrix (SparseMatrix + SparseVector<float>)
struct Column {
    bool exists = false;
    int ab = 0, ae = 0;               // allocated rows [ab, ae)
    std::vector<float> store;         // storage_ (its capacity is AllocatedEntries, SparseVector-inl.hpp:250)
};

struct QMatrix {
    int rows = 0, cols = 0;
    std::vector<Column> c;
    std::vector<int> ub, ue;          // used row ranges (FinishEditingColumn)
    QMatrix() {}
    QMatrix(int r, int k) : rows(r), cols(k), c(k), ub(k, 0), ue(k, 0) {}
    bool IsNull() const { return rows == 0 && cols == 0; }
    bool Empty(int j) const { return ub[j] >= ue[j]; }
    float Get(int i, int j) const
    {
        const Column& col = c[j];
        if (!col.exists || i < col.ab || i >= col.ae) return NEG_INF;
        return col.store[i - col.ab];
    }
    void Start(int j, int hb, int he)   // StartEditingColumn / ResetForRange (SparseVector-inl.hpp:74-106)
    {
        Column& col = c[j];
        const int nb = std::max(hb - 8, 0), ne = std::min(he + 8, rows);
        if (!col.exists) {
            col.exists = true;
            col.store.assign(ne - nb, NEG_INF);
        } else if ((ne - nb) > (col.ae - col.ab)) {
            col.store.resize(ne - nb);
            std::fill(col.store.begin(), col.store.end(), NEG_INF);
        } else if ((ne - nb) < static_cast<int>(0.8 * (col.ae - col.ab))) {
            std::vector<float>(ne - nb, NEG_INF).swap(col.store);
        } else {
            std::fill(col.store.begin(), col.store.end(), NEG_INF);
        }
        col.ab = nb;
        col.ae = ne;
    }
    void Set(int i, int j, float v)   // SparseVector::Set + ExpandAllocated (:118-141, :171-186)
    {
        Column& col = c[j];
        if (i < col.ab || i >= col.ae) {
            const int nb = std::max(std::min(i - 8, col.ab), 0);
            const int ne = std::min(std::max(i + 8, col.ae), rows);
            col.store.resize(ne - nb);
            std::memmove(&col.store[col.ab - nb], &col.store[0], (col.ae - col.ab) * sizeof(float));
            std::fill(col.store.begin(), col.store.begin() + (col.ab - nb), NEG_INF);
            std::fill(col.store.begin() + (col.ae - nb), col.store.end(), NEG_INF);
            col.ab = nb;
            col.ae = ne;
        }
        col.store[i - col.ab] = v;
    }
    void Finish(int j, int b, int e) { ub[j] = b; ue[j] = e; }
    long long UsedEntries() const
    {
        long long s = 0;
        for (int j = 0; j < cols; ++j) s += ue[j] - ub[j];
        return s;
    }
    bool dense = false;   // DenseMatrixF: the same values (ClearColumn resets the previous used range to
                          // lfloat(), DenseMatrix-inl.hpp:158-172), every cell allocated
    long long AllocatedEntries() const
    {
        if (dense) return (long long)rows * cols;   // DenseMatrix-inl.hpp:242-246
        long long s = 0;
        for (const Column& col : c) s += col.exists ? (long long)col.store.capacity() : 0;
        return s;
    }
};

static const QMatrix& Null()
{
    static const QMatrix n;
    return n;
}

// ---------------------------------------------------------------- recursor
struct Recursor {
    int moves = ALL_MOVES;
    float scoreDiff = 12.5f;
    Combiner Cb;
    bool simple = false;   // SimpleRecursor (Quiver/SimpleRecursor.cpp) instead of SseRecursor
    bool dense = false;    // DenseMatrixF storage (SimpleQvRecursor / SseQvRecursor)

    // ---- SimpleRecursor (Quiver/SimpleRecursor.cpp:60-405): row by row, moves combined in the order
    // Incorporate, Extra, Delete, Merge, the band end tested after every row
    void FillAlphaSimple(const Evaluator& e, const QMatrix& guide, QMatrix& a) const   // :60-135
    {
        const int I = e.I(), J = e.J();
        int hb = 0, he = 0;
        for (int j = 0; j <= J; ++j) {
            Guide(j, guide, a, &hb, &he);
            const int reqEnd = std::min(I + 1, he);
            float score = NEG_INF, thr = NEG_INF, mx = NEG_INF;
            a.Start(j, hb, he);
            const int beginRow = hb;
            int i;
            for (i = beginRow; i < I + 1 && (score >= thr || i < reqEnd); ++i) {
                score = NEG_INF;
                if (i == 0 && j == 0) score = 0.0f;
                if (i > 0 && j > 0) score = Cb.C(score, a.Get(i - 1, j - 1) + e.Inc(i - 1, j - 1));
                if (i > 0) score = Cb.C(score, a.Get(i - 1, j) + e.Extra(i - 1, j));
                if (j > 0) score = Cb.C(score, a.Get(i, j - 1) + e.Del(i, j - 1));
                if ((moves & MERGE) && j > 1 && i > 0) score = Cb.C(score, a.Get(i - 1, j - 2) + e.Merge(i - 1, j - 2));
                a.Set(i, j, score);
                if (score > mx) { mx = score; thr = mx - scoreDiff; }
            }
            const int endRow = i;
            a.Finish(j, beginRow, endRow);
            he = endRow;
            for (i = beginRow; i < endRow && a.Get(i, j) < thr; ++i) {}
            hb = i;
        }
    }

    void FillBetaSimple(const Evaluator& e, const QMatrix& guide, QMatrix& b) const   // :138-222
    {
        const int I = e.I(), J = e.J();
        int hb = I + 1, he = I + 1;
        for (int j = J; j >= 0; --j) {
            Guide(j, guide, b, &hb, &he);
            const int reqBegin = std::max(0, hb);
            b.Start(j, hb, he);
            float score = NEG_INF, thr = NEG_INF, mx = NEG_INF;
            const int endRow = he;
            int i;
            for (i = endRow - 1; i >= 0 && (score >= thr || i >= reqBegin); --i) {
                score = NEG_INF;
                if (i == I && j == J) score = 0.0f;
                if (i < I && j < J) score = Cb.C(score, b.Get(i + 1, j + 1) + e.Inc(i, j));
                if (i < I) score = Cb.C(score, b.Get(i + 1, j) + e.Extra(i, j));
                if (j < J) score = Cb.C(score, b.Get(i, j + 1) + e.Del(i, j));
                if ((moves & MERGE) && j < J - 1 && i < I) score = Cb.C(score, b.Get(i + 1, j + 2) + e.Merge(i, j));
                b.Set(i, j, score);
                if (score > mx) { mx = score; thr = mx - scoreDiff; }
            }
            const int beginRow = i + 1;
            b.Finish(j, beginRow, endRow);
            hb = beginRow;
            for (i = endRow; i > beginRow && b.Get(i - 1, j) < thr; --i) {}
            he = i;
        }
    }

    // :232-295 -- the merge terms are added whatever movesAvailable_ says (no MERGE test in the reference)
    float LinkSimple(const Evaluator& e, const QMatrix& a, int ac, const QMatrix& b, int bc, int absc) const
    {
        const int I = e.I();
        const int ub = RangeUnion4b(a, ac, b, bc), ue = RangeUnion4e(a, ac, b, bc);
        float v = NEG_INF;
        for (int i = ub; i < ue; i++) {
            if (i < I) {
                v = Cb.C(v, a.Get(i, ac - 1) + e.Inc(i, absc - 1) + b.Get(i + 1, bc));
                v = Cb.C(v, a.Get(i, ac - 2) + e.Merge(i, absc - 2) + b.Get(i + 1, bc));
                v = Cb.C(v, a.Get(i, ac - 1) + e.Merge(i, absc - 1) + b.Get(i + 1, bc + 1));
            }
            v = Cb.C(v, a.Get(i, ac - 1) + e.Del(i, absc - 1) + b.Get(i, bc));
        }
        return v;
    }

    // :303-388 (the merge term reads alpha(i - 1, j - 2) for every extension column, as the reference does)
    void ExtendAlphaSimple(const Evaluator& e, const QMatrix& a, int beginColumn, QMatrix& ext, int numExt) const
    {
        for (int extCol = 0; extCol < numExt; extCol++) {
            const int j = beginColumn + extCol;
            int beginRow, endRow;
            if (j < a.cols) { beginRow = a.ub[j]; endRow = a.ue[j]; }
            else { beginRow = a.ub[a.cols - 1]; endRow = a.rows; }
            ext.Start(extCol, beginRow, endRow);
            for (int i = beginRow; i < endRow; i++) {
                float score = NEG_INF;
                if (i > 0 && j > 0) {
                    const float prev = extCol == 0 ? a.Get(i - 1, j - 1) : ext.Get(i - 1, extCol - 1);
                    score = Cb.C(score, prev + e.Inc(i - 1, j - 1));
                }
                if (i > 0) score = Cb.C(score, ext.Get(i - 1, extCol) + e.Extra(i - 1, j));
                if (j > 0) {
                    const float prev = extCol == 0 ? a.Get(i, j - 1) : ext.Get(i, extCol - 1);
                    score = Cb.C(score, prev + e.Del(i, j - 1));
                }
                if ((moves & MERGE) && j > 1 && i > 0) score = Cb.C(score, a.Get(i - 1, j - 2) + e.Merge(i - 1, j - 2));
                ext.Set(i, extCol, score);
            }
            ext.Finish(extCol, beginRow, endRow);
        }
    }

    // RowRange (RecursorBase-inl.hpp:49-82): trims the used range to the rows within scoreDiff of its max
    void RowRange(int j, const QMatrix& m, int* ob, int* oe) const
    {
        int b = m.ub[j], e = m.ue[j];
        int maxRow = b;
        float maxScore = m.Get(maxRow, j);
        for (int i = b + 1; i < e; ++i) {
            const float s = m.Get(i, j);
            if (s > maxScore) { maxRow = i; maxScore = s; }
        }
        const float thr = maxScore - scoreDiff;
        int i;
        for (i = b; i < maxRow && m.Get(i, j) < thr; ++i) {}
        b = i;
        for (i = e - 1; i >= maxRow && m.Get(i, j) < thr; --i) {}
        e = i + 1;
        *ob = b;
        *oe = e;
    }
    // RangeGuide (RecursorBase-inl.hpp:84-114)
    void Guide(int j, const QMatrix& guide, const QMatrix& self, int* hb, int* he) const
    {
        const bool useGuide = !(guide.IsNull() || guide.Empty(j));
        const bool useSelf = !(self.IsNull() || self.Empty(j));
        if (!useGuide && !useSelf) return;
        int b = *hb, e = *he, rb, re;
        if (useGuide) { RowRange(j, guide, &rb, &re); b = std::min(rb, b); e = std::max(re, e); }
        if (useSelf) { RowRange(j, self, &rb, &re); b = std::min(rb, b); e = std::max(re, e); }
        *hb = b;
        *he = e;
    }

    // SseRecursor::FillAlpha (SseRecursor.cpp:73-213)
    void FillAlpha(const Evaluator& e, const QMatrix& guide, QMatrix& a) const
    {
        if (simple) return FillAlphaSimple(e, guide, a);
        const int I = e.I(), J = e.J();
        int hb = 0, he = 0;
        for (int j = 0; j <= J; ++j) {
            Guide(j, guide, a, &hb, &he);
            const int reqEnd = std::min(I + 1, he);
            float score = NEG_INF, thr = NEG_INF, mx = NEG_INF;
            a.Start(j, hb, he);
            int i;
            const int beginRow = hb;
            for (i = beginRow; (i == 0 || (I - i + 1) % 4 != 0) && i <= I; i++) {   // scalar prologue
                score = NEG_INF;
                if (i == 0 && j == 0) score = 0.0f;
                if (i > 0 && j > 0) score = Cb.C(score, a.Get(i - 1, j - 1) + e.Inc(i - 1, j - 1));
                if ((moves & MERGE) && (i > 0 && j > 1)) score = Cb.C(score, a.Get(i - 1, j - 2) + e.Merge(i - 1, j - 2));
                if (j > 0) score = Cb.C(score, a.Get(i, j - 1) + e.Del(i, j - 1));
                if (i > 0) score = Cb.C(score, a.Get(i - 1, j) + e.Extra(i - 1, j));
                a.Set(i, j, score);
                if (score > mx) { mx = score; thr = mx - scoreDiff; }
            }
            for (; i <= I && (score >= thr || i < reqEnd); i += 4) {   // 4-row blocks
                float s4[4], ins[4], s5[5];
                for (int k = 0; k < 4; ++k) {
                    const int r = i + k;
                    float v = NEG_INF;
                    if (j > 0) v = Cb.C4(v, a.Get(r - 1, j - 1) + e.Inc(r - 1, j - 1));
                    if ((moves & MERGE) && j >= 2) v = Cb.C4(v, a.Get(r - 1, j - 2) + e.Merge(r - 1, j - 2));
                    if (j > 0) v = Cb.C4(v, a.Get(r, j - 1) + e.Del(r, j - 1));
                    s4[k] = v;
                    ins[k] = e.Extra(r - 1, j);
                }
                s5[0] = a.Get(i - 1, j);
                for (int k = 0; k < 4; ++k) s5[k + 1] = s4[k];
                for (int ii = 1; ii < 5; ++ii) s5[ii] = Cb.C(s5[ii], s5[ii - 1] + ins[ii - 1]);   // Extra cascade
                for (int k = 0; k < 4; ++k) a.Set(i + k, j, s5[k + 1]);
                const float pmax = *std::max_element(s5 + 1, s5 + 5);
                score = *std::min_element(s5 + 1, s5 + 5);
                if (pmax > mx) { mx = pmax; thr = mx - scoreDiff; }
            }
            const int endRow = i;
            a.Finish(j, beginRow, endRow);
            he = endRow;
            for (i = beginRow; i < endRow && a.Get(i, j) < thr; ++i) {}
            hb = i;
        }
    }

    // SseRecursor::FillBeta (SseRecursor.cpp:216-353)
    void FillBeta(const Evaluator& e, const QMatrix& guide, QMatrix& b) const
    {
        if (simple) return FillBetaSimple(e, guide, b);
        const int I = e.I(), J = e.J();
        int hb = I + 1, he = I + 1;
        for (int j = J; j >= 0; --j) {
            Guide(j, guide, b, &hb, &he);
            const int reqBegin = std::max(0, hb);
            float score = NEG_INF, thr = NEG_INF, mx = NEG_INF;
            b.Start(j, hb, he);
            const int endRow = he;
            int i;
            for (i = endRow - 1; (i == I || (i + 1) % 4 != 0) && i >= 0; i--) {
                score = NEG_INF;
                if (i == I && j == J) score = 0.0f;
                if (i < I && j < J) score = Cb.C(score, b.Get(i + 1, j + 1) + e.Inc(i, j));
                if ((moves & MERGE) && j < J - 1 && i < I) score = Cb.C(score, b.Get(i + 1, j + 2) + e.Merge(i, j));
                if (j < J) score = Cb.C(score, b.Get(i, j + 1) + e.Del(i, j));
                if (i < I) score = Cb.C(score, b.Get(i + 1, j) + e.Extra(i, j));
                b.Set(i, j, score);
                if (score > mx) { mx = score; thr = mx - scoreDiff; }
            }
            i = i - 3;
            for (; i >= 0 && (score >= thr || i >= reqBegin); i -= 4) {
                float s4[4], ins[4], s5[5];
                for (int k = 0; k < 4; ++k) {
                    const int r = i + k;
                    float v = NEG_INF;
                    if (r < I && j < J) v = Cb.C4(v, b.Get(r + 1, j + 1) + e.Inc(r, j));
                    if ((moves & MERGE) && j < J - 1 && r < I) v = Cb.C4(v, b.Get(r + 1, j + 2) + e.Merge(r, j));
                    if (j < J) v = Cb.C4(v, b.Get(r, j + 1) + e.Del(r, j));
                    s4[k] = v;
                    ins[k] = e.Extra(r, j);
                }
                s5[4] = b.Get(i + 4, j);
                for (int k = 0; k < 4; ++k) s5[k] = s4[k];
                for (int ii = 3; ii >= 0; ii--) s5[ii] = Cb.C(s5[ii], s5[ii + 1] + ins[ii]);
                for (int k = 0; k < 4; ++k) b.Set(i + k, j, s5[k]);
                const float pmax = *std::max_element(s5, s5 + 4);
                score = *std::min_element(s5, s5 + 4);
                if (pmax > mx) { mx = pmax; thr = mx - scoreDiff; }
            }
            const int beginRow = i + 4;
            b.Finish(j, beginRow, endRow);
            hb = beginRow;
            for (i = endRow; i > beginRow && b.Get(i - 1, j) < thr; i--) {}
            he = i;
        }
    }
    // NB (FillBeta's 4-row blocks, SseRecursor.cpp:290-338): in the reference, the rows i..i+3 of the
    // r < I guards are evaluated per block (the whole block i < I); the block rows are all < I there.

    // SseRecursor::LinkAlphaBeta (SseRecursor.cpp:355-431)
    float Link(const Evaluator& e, const QMatrix& a, int ac, const QMatrix& b, int bc, int absc) const
    {
        if (simple) return LinkSimple(e, a, ac, b, bc, absc);
        const int I = e.I();
        // RangeUnion of the four used ranges (Interval.hpp:80-99: min of begins, max of ends)
        const int ub = RangeUnion4b(a, ac, b, bc);
        const int ue = RangeUnion4e(a, ac, b, bc);
        float v = NEG_INF;
        float v4[4] = {NEG_INF, NEG_INF, NEG_INF, NEG_INF};
        int i;
        for (i = ub; i < ue - 4; i += 4) {
            for (int k = 0; k < 4; ++k) {
                const int r = i + k;
                v4[k] = Cb.C4(v4[k], a.Get(r, ac - 1) + e.Inc(r, absc - 1) + b.Get(r + 1, bc));
                if (moves & MERGE) {
                    v4[k] = Cb.C4(v4[k], a.Get(r, ac - 2) + e.Merge(r, absc - 2) + b.Get(r + 1, bc));
                    v4[k] = Cb.C4(v4[k], a.Get(r, ac - 1) + e.Merge(r, absc - 1) + b.Get(r + 1, bc + 1));
                }
                v4[k] = Cb.C4(v4[k], a.Get(r, ac - 1) + e.Del(r, absc - 1) + b.Get(r, bc));
            }
        }
        for (; i < ue; i++) {
            if (i < I) {
                v = Cb.C(v, a.Get(i, ac - 1) + e.Inc(i, absc - 1) + b.Get(i + 1, bc));
                if (moves & MERGE) {
                    v = Cb.C(v, a.Get(i, ac - 2) + e.Merge(i, absc - 2) + b.Get(i + 1, bc));
                    v = Cb.C(v, a.Get(i, ac - 1) + e.Merge(i, absc - 1) + b.Get(i + 1, bc + 1));
                }
            }
            v = Cb.C(v, a.Get(i, ac - 1) + e.Del(i, absc - 1) + b.Get(i, bc));
        }
        float acc = NEG_INF;   // std::accumulate(v_array, v_array + 5, NEG_INF, C::Combine)
        for (int k = 0; k < 4; ++k) acc = Cb.C(acc, v4[k]);
        acc = Cb.C(acc, v);
        return acc;
    }
    static int RangeUnion4b(const QMatrix& a, int ac, const QMatrix& b, int bc)
    {
        return std::min(std::min(a.ub[ac - 2], a.ub[ac - 1]), std::min(b.ub[bc], b.ub[bc + 1]));
    }
    static int RangeUnion4e(const QMatrix& a, int ac, const QMatrix& b, int bc)
    {
        return std::max(std::max(a.ue[ac - 2], a.ue[ac - 1]), std::max(b.ue[bc], b.ue[bc + 1]));
    }

    // SseRecursor::ExtendAlpha (SseRecursor.cpp:433-551)
    void ExtendAlpha(const Evaluator& e, const QMatrix& a, int beginColumn, QMatrix& ext, int numExt) const
    {
        if (simple) return ExtendAlphaSimple(e, a, beginColumn, ext, numExt);
        for (int extCol = 0; extCol < numExt; extCol++) {
            const int j = beginColumn + extCol;
            int beginRow, endRow;
            if (j < a.cols) { beginRow = a.ub[j]; endRow = a.ue[j]; }
            else { beginRow = a.ub[a.cols - 1]; endRow = a.rows; }
            ext.Start(extCol, beginRow, endRow);
            int i;
            for (i = beginRow; (i == 0 || (endRow - i) % 4 != 0) && i < endRow; i++) {
                float prev, score = NEG_INF;
                if (i > 0) {
                    prev = (extCol == 0) ? a.Get(i - 1, j - 1) : ext.Get(i - 1, extCol - 1);
                    score = Cb.C(score, prev + e.Inc(i - 1, j - 1));
                    prev = ext.Get(i - 1, extCol);
                    score = Cb.C(score, prev + e.Extra(i - 1, j));
                    if (moves & MERGE) {
                        prev = a.Get(i - 1, j - 2);
                        score = Cb.C(score, prev + e.Merge(i - 1, j - 2));
                    }
                }
                prev = (extCol == 0) ? a.Get(i, j - 1) : ext.Get(i, extCol - 1);
                score = Cb.C(score, prev + e.Del(i, j - 1));
                ext.Set(i, extCol, score);
            }
            for (; i < endRow - 3; i += 4) {
                float s4[4], ins[4], s5[5];
                for (int k = 0; k < 4; ++k) {
                    const int r = i + k;
                    float v = NEG_INF;
                    float prev = (extCol == 0) ? a.Get(r - 1, j - 1) : ext.Get(r - 1, extCol - 1);
                    v = Cb.C4(v, prev + e.Inc(r - 1, j - 1));
                    if ((moves & MERGE) && j >= 2) v = Cb.C4(v, a.Get(r - 1, j - 2) + e.Merge(r - 1, j - 2));
                    prev = (extCol == 0) ? a.Get(r, j - 1) : ext.Get(r, extCol - 1);
                    v = Cb.C4(v, prev + e.Del(r, j - 1));
                    s4[k] = v;
                    ins[k] = e.Extra(r - 1, j);
                }
                s5[0] = ext.Get(i - 1, extCol);
                for (int k = 0; k < 4; ++k) s5[k + 1] = s4[k];
                for (int ii = 1; ii < 5; ii++) s5[ii] = Cb.C(s5[ii], s5[ii - 1] + ins[ii - 1]);
                for (int k = 0; k < 4; ++k) ext.Set(i + k, extCol, s5[k + 1]);
            }
            ext.Finish(extCol, beginRow, endRow);
        }
    }

    // SimpleRecursor::ExtendBeta (Quiver/SimpleRecursor.cpp:407-495)
    void ExtendBeta(const Evaluator& e, const QMatrix& b, int lastColumn, QMatrix& ext, int numExt, int lengthDiff) const
    {
        const int I = b.rows - 1, J = b.cols - 1;
        const int lastExt = numExt - 1;
        for (int j = lastColumn; j > lastColumn - numExt; j--) {
            const int jp = j + lengthDiff;
            const int extCol = lastExt - (lastColumn - j);
            int beginRow, endRow;
            if (j < 0) { beginRow = 0; endRow = b.ue[0]; }
            else { beginRow = b.ub[j]; endRow = b.ue[j]; }
            ext.Start(extCol, beginRow, endRow);
            for (int i = endRow - 1; i >= beginRow; i--) {
                float score = NEG_INF, mv;
                if (i < I && j < J) {
                    const float prev = (extCol == lastExt) ? b.Get(i + 1, j + 1) : ext.Get(i + 1, extCol + 1);
                    mv = prev + e.Inc(i, jp);
                    score = Cb.C(score, mv);
                }
                if (i < I) {
                    mv = ext.Get(i + 1, extCol) + e.Extra(i, jp);
                    score = Cb.C(score, mv);
                }
                if (j < J) {
                    const float prev = (extCol == lastExt) ? b.Get(i, j + 1) : ext.Get(i, extCol + 1);
                    mv = prev + e.Del(i, jp);
                    score = Cb.C(score, mv);
                }
                if ((moves & MERGE) && j < J - 1 && i < I) {
                    mv = b.Get(i + 1, j + 2) + e.Merge(i, jp);
                    score = Cb.C(score, mv);
                }
                ext.Set(i, extCol, score);
            }
            ext.Finish(extCol, beginRow, endRow);
        }
    }

    // RecursorBase::FillAlphaBeta (detail/RecursorBase.cpp:70-116)
    int FillAlphaBeta(const Evaluator& e, QMatrix& a, QMatrix& b) const
    {
        FillAlpha(e, Null(), a);
        FillBeta(e, a, b);
        const int I = e.I(), J = e.J();
        int flips = 0;
        const int maxSize = static_cast<int>(0.5 + 0.04 * (I + 1) * (J + 1));
        if (a.UsedEntries() >= maxSize || b.UsedEntries() >= maxSize) {
            FillAlpha(e, b, a);
            FillBeta(e, a, b);
            FillAlpha(e, b, a);
            flips += 3;
        }
        while (std::fabs(a.Get(I, J) - b.Get(0, 0)) > 0.2 && flips <= 5) {
            if (flips % 2 == 0) FillAlpha(e, b, a);
            else FillBeta(e, a, b);
            flips++;
        }
        if (std::fabs(a.Get(I, J) - b.Get(0, 0)) > 0.2) throw AlphaBetaMismatch();
        return flips;
    }
};

// ---------------------------------------------------------------- mutation scorer (Quiver/MutationScorer.cpp:53-240)
struct MutationScorer {
    Evaluator ev;
    Recursor rec;
    QMatrix alpha, beta, ext;
    int flips = 0;
    MutationScorer(const Evaluator& e, const Recursor& r) : ev(e), rec(r)
    {
        alpha = QMatrix(ev.I() + 1, ev.J() + 1);
        beta = QMatrix(ev.I() + 1, ev.J() + 1);
        ext = QMatrix(ev.I() + 1, 8);   // EXTEND_BUFFER_COLUMNS
        alpha.dense = beta.dense = rec.dense;
        flips = rec.FillAlphaBeta(ev, alpha, beta);
    }
    float Score() const { return beta.Get(0, 0); }
    void Template(const std::string& tpl)   // :74-84 (flip-flop count is not updated)
    {
        ev.tpl = tpl;
        alpha = QMatrix(ev.I() + 1, ev.J() + 1);
        beta = QMatrix(ev.I() + 1, ev.J() + 1);
        alpha.dense = beta.dense = rec.dense;
        rec.FillAlphaBeta(ev, alpha, beta);
    }
    float ScoreMutation(const Mut& m)   // :113-226 (absolute score of the mutated template)
    {
        const int betaLinkCol = 1 + m.end;
        const int absLinkCol = 1 + m.end + m.LengthDiff();
        const std::string oldTpl = ev.tpl;
        const std::string newTpl = orc::ApplyMuts({m}, oldTpl);
        float score;
        const bool atBegin = m.start < 3;
        const bool atEnd = m.end > (int)oldTpl.size() - 2;
        if (!atBegin && !atEnd) {
            ev.tpl = newTpl;
            int extStart, extLen;
            if (m.type == DEL) { extStart = m.start - 1; extLen = 2; }
            else { extStart = m.start; extLen = 1 + (int)m.bases.size(); }
            rec.ExtendAlpha(ev, alpha, extStart, ext, extLen);
            score = rec.Link(ev, ext, extLen, beta, betaLinkCol, absLinkCol);
        } else if (!atBegin && atEnd) {
            ev.tpl = newTpl;
            const int extStart = m.start - 1;
            const int extLen = (int)newTpl.size() - extStart + 1;
            rec.ExtendAlpha(ev, alpha, extStart, ext, extLen);
            score = ext.Get(ev.I(), extLen - 1);
        } else if (atBegin && !atEnd) {
            ev.tpl = newTpl;
            const int extLast = m.end;
            const int extLen = m.end + m.LengthDiff() + 1;
            rec.ExtendBeta(ev, beta, extLast, ext, extLen, m.LengthDiff());
            score = ext.Get(0, 0);
        } else {
            QMatrix ap(ev.I() + 1, (int)newTpl.size() + 1);
            ev.tpl = newTpl;
            rec.FillAlpha(ev, Null(), ap);
            score = ap.Get(ev.I(), (int)newTpl.size());
        }
        ev.tpl = oldTpl;
        return score;
    }
};

// ---------------------------------------------------------------- traceback (detail/RecursorBase.cpp:118-264)
// RecursorBase::Alignment: the Viterbi path through a filled alpha matrix, moves tried in the order
// Incorporate, Delete, Extra, Merge with strict '>' against lfloat(); then replayed into the gapped
// target / query strings of the PairwiseAlignment.  Viterbi combiner only (ShouldNotReachHere otherwise).
static bool Alignment(const Evaluator& e, const QMatrix& a, int moves, std::string* target, std::string* query)
{
    struct Spec { int type, dr, dt; };
    const Spec inc{INCORPORATE, 1, 1}, del{DELETE, 0, 1}, extra{EXTRA, 1, 0}, merge{MERGE, 1, 2};
    const int I = e.I(), J = e.J();
    int i = I, j = J;
    std::vector<Spec> path;
    while (i > 0 || j > 0) {
        Spec best{0, 0, 0};
        float bestScore = -FLT_MAX;
        if (i > 0 && j > 0) {
            const float t = a.Get(i - 1, j - 1) + e.Inc(i - 1, j - 1);
            if (t > bestScore) { best = inc; bestScore = t; }
        }
        if (j > 0) {
            const bool freeDelete = (!e.pinEnd && i == I) || (!e.pinStart && i == 0);
            const float t = a.Get(i, j - 1) + (freeDelete ? 0.0f : e.Del(i, j - 1));
            if (t > bestScore) { best = del; bestScore = t; }
        }
        if (i > 0) {
            const float t = a.Get(i - 1, j) + e.Extra(i - 1, j);
            if (t > bestScore) { best = extra; bestScore = t; }
        }
        if ((moves & MERGE) && i > 0 && j > 1) {
            const float t = a.Get(i - 1, j - 2) + e.Merge(i - 1, j - 2);
            if (t > bestScore) { best = merge; bestScore = t; }
        }
        if (best.type == 0) return false;   // assert(bestMove.MoveType != INVALID_MOVE)
        path.push_back(best);
        i -= best.dr;
        j -= best.dt;
    }
    std::reverse(path.begin(), path.end());
    target->clear();
    query->clear();
    i = j = 0;
    for (const Spec& m : path) {
        if (m.type == INCORPORATE) { *target += e.tpl[j]; *query += e.r->seq[i]; }
        else if (m.type == EXTRA) { *target += '-'; *query += e.r->seq[i]; }
        else if (m.type == DELETE) { *target += e.tpl[j]; *query += '-'; }
        else { *target += e.tpl[j]; *target += e.tpl[j + 1]; *query += '-'; *query += e.r->seq[i]; }
        i += m.dr;
        j += m.dt;
    }
    return true;
}

// ---------------------------------------------------------------- multi-read scorer (Quiver/MultiReadMutationScorer.cpp)
struct MappedRead {
    QvRead read;
    int strand = FWD;
    int ts = 0, te = 0;
};

static bool ReadScoresMutation(const MappedRead& r, const Mut& m)   // :60-71
{
    if (m.type == INS) return r.ts < m.start && m.end <= r.te;
    return r.ts < m.end && m.start < r.te;
}

static Mut OrientedMutation(const MappedRead& r, const Mut& mut)   // :79-120
{
    Mut c(INS, 0, 0, "N");
    if (mut.end - mut.start > 1) {
        const int cs = std::max(mut.start, r.ts), ce = std::min(mut.end, r.te);
        if (mut.type == SUB) c = Mut(mut.type, cs, ce, mut.bases.substr(cs - mut.start, ce - cs));
        else c = Mut(mut.type, cs, ce, mut.bases);
    } else {
        c = mut;
    }
    if (r.strand == FWD) return Mut(c.type, c.start - r.ts, c.end - r.ts, c.bases);
    return Mut(c.type, r.te - c.end, r.te - c.start, orc::RevComp(c.bases));
}

struct ConfigTable {   // QuiverConfigTable (QuiverConfig.cpp:67-138): front-inserted list, "*" fallback
    std::list<std::pair<std::string, QuiverConfig>> table;
    bool InsertAs(const std::string& name, const QuiverConfig& c)
    {
        for (auto& kv : table)
            if (kv.first == name) return false;
        table.emplace_front(name, c);
        return true;
    }
    const QuiverConfig& At(const std::string& name) const
    {
        for (auto& kv : table)
            if (kv.first == name) return kv.second;
        for (auto& kv : table)
            if (kv.first == "*") return kv.second;
        throw std::invalid_argument("Chemistry not found in QuiverConfigTable");
    }
};

struct ReadState {
    MappedRead mr;
    MutationScorer* sc = nullptr;
    bool active = false;
};

struct MultiReadScorer {
    ConfigTable configs;
    float fastThreshold = 0.0f;
    std::string fwd, rev;
    std::vector<ReadState> reads;
    ~MultiReadScorer()
    {
        for (ReadState& r : reads) delete r.sc;
    }
    void Init(const std::string& tpl)   // :123-136
    {
        fwd = tpl;
        rev = orc::RevComp(tpl);
        fastThreshold = 0.0f;
        for (auto& kv : configs.table) fastThreshold = std::min(fastThreshold, kv.second.fastScoreThreshold);
    }
    std::string Window(int strand, int ts, int te) const
    {
        const int len = te - ts;
        return strand == FWD ? fwd.substr(ts, len) : rev.substr((int)fwd.size() - te, len);
    }
    bool AddRead(const MappedRead& mr, float threshold)   // :246-283
    {
        const QuiverConfig& c = configs.At(mr.read.chemistry);
        ReadState rs;
        rs.mr = mr;
        Evaluator ev;
        ev.rd = mr.read;
        ev.pm = c.qv;
        ev.tpl = Window(mr.strand, mr.ts, mr.te);
        Recursor rec;
        rec.moves = c.moves;
        rec.scoreDiff = c.scoreDiff;
        rec.Cb.sumProduct = c.sumProduct;
        rec.simple = c.simple;
        rec.dense = c.dense;
        reads.push_back(rs);
        ReadState& st = reads.back();
        MutationScorer* s = nullptr;
        try {
            s = new MutationScorer(ev, rec);
        } catch (AlphaBetaMismatch&) {
            s = nullptr;
        }
        if (s && threshold < 1.0f) {
            const int I = ev.I(), J = ev.J();
            const int maxSize = static_cast<int>(0.5 + threshold * (I + 1) * (J + 1));
            if (s->alpha.AllocatedEntries() >= maxSize || s->beta.AllocatedEntries() >= maxSize) {
                delete s;
                s = nullptr;
            }
        }
        st.sc = s;
        st.active = s != nullptr;
        return st.active;
    }
    float Delta(ReadState& rs, const Mut& m) { return rs.sc->ScoreMutation(OrientedMutation(rs.mr, m)) - rs.sc->Score(); }
    float Score(const Mut& m)   // :312-326
    {
        float sum = 0;
        for (ReadState& rs : reads)
            if (rs.active && ReadScoresMutation(rs.mr, m)) sum += Delta(rs, m);
        return sum;
    }
    float FastScore(const Mut& m)   // :336-353
    {
        float sum = 0;
        for (ReadState& rs : reads)
            if (rs.active && ReadScoresMutation(rs.mr, m)) {
                sum += Delta(rs, m);
                if (sum < fastThreshold) return sum;
            }
        return sum;
    }
    bool FastIsFavorable(const Mut& m)   // :392-409
    {
        float sum = 0;
        for (ReadState& rs : reads)
            if (rs.active && ReadScoresMutation(rs.mr, m)) {
                sum += Delta(rs, m);
                if (sum < fastThreshold) return false;
            }
        return (double)sum > 0.04;   // MIN_FAVORABLE_SCOREDIFF is a double literal (:52)
    }
    std::vector<float> Scores(const Mut& m, float unscored)
    {
        std::vector<float> out;
        for (ReadState& rs : reads)
            out.push_back((rs.active && ReadScoresMutation(rs.mr, m)) ? Delta(rs, m) : unscored);
        return out;
    }
    float Baseline() const
    {
        float sum = 0;
        for (const ReadState& rs : reads)
            if (rs.active) sum += rs.sc->Score();
        return sum;
    }
    void ApplyMutations(const std::vector<Mut>& muts)   // :205-239
    {
        const std::vector<int> mtp = orc::TargetToQuery(muts, fwd);
        fwd = orc::ApplyMuts(muts, fwd);
        rev = orc::RevComp(fwd);
        for (ReadState& rs : reads) {
            rs.mr.ts = mtp[rs.mr.ts];
            rs.mr.te = mtp[rs.mr.te];
            if (rs.active) {
                try {
                    rs.sc->Template(Window(rs.mr.strand, rs.mr.ts, rs.mr.te));
                } catch (AlphaBetaMismatch&) {
                    rs.active = false;
                }
            }
        }
    }
};

// AbstractRefineConsensus (Consensus-inl.hpp:159-251) over the Quiver scorer (scores are float already)
static bool Refine(MultiReadScorer& mms, int maxIter, int sep, int nbhd, long* nTested, long* nApplied)
{
    bool converged = false;
    std::set<std::string> history;
    std::vector<orc::Scored> favorable;
    for (int iter = 0; iter < maxIter; ++iter) {
        std::vector<Mut> toTry;
        if (iter == 0) {
            toTry = orc::UniqueMutations(mms.fwd, 0, (int)mms.fwd.size());
        } else {
            std::vector<Mut> centers;
            for (const orc::Scored& s : favorable) centers.push_back(s.m);
            toTry = orc::NearbyMutations(mms.fwd, centers, nbhd);
        }
        *nTested += (long)toTry.size();
        favorable.clear();
        for (const Mut& m : toTry)
            if (mms.FastIsFavorable(m)) favorable.push_back({m, mms.Score(m)});
        if (favorable.empty()) { converged = true; break; }
        std::vector<orc::Scored> best = orc::BestSubset(favorable, sep);
        if (best.size() > 1) {
            std::vector<Mut> bm;
            for (const orc::Scored& s : best) bm.push_back(s.m);
            if (history.count(orc::ApplyMuts(bm, mms.fwd))) best.resize(1);
        }
        *nApplied += (long)best.size();
        history.insert(mms.fwd);
        std::vector<Mut> bm;
        for (const orc::Scored& s : best) bm.push_back(s.m);
        mms.ApplyMutations(bm);
    }
    return converged;
}

// ConsensusQVs (Consensus-inl.hpp:274-295)
static std::vector<int> ConsensusQVs(MultiReadScorer& mms)
{
    std::vector<int> qvs;
    const std::string tpl = mms.fwd;
    for (size_t p = 0; p < tpl.size(); ++p) {
        double sum = 0.0;
        for (const Mut& m : orc::UniqueMutations(tpl, (int)p, (int)p + 1)) {
            const double s = mms.Score(m);
            if (s < 0.0) sum += std::exp(s);
        }
        double prob = 1.0 - 1.0 / (1.0 + sum);
        if (prob == 0.0) prob = std::numeric_limits<double>::min();
        qvs.push_back(static_cast<int>(std::round(-10.0 * std::log10(prob))));
    }
    return qvs;
}

}  // namespace qorc

// ============================================================== C ABI for the tests (ctypes)
using namespace qorc;

extern "C" {

float qorc_log_add(float a, float b) { return logAdd(a, b); }

// RecursorBase::Alignment of read r's MutationScorer alpha (Viterbi only): 0 ok, -1 sum-product, -2 no path
int qorc_scorer_alignment(void* h, int r, char* target, char* query, int cap);
float qorc_exp_ps(float x) { return exp_ps1(x); }
float qorc_log_ps(float x) { return log_ps1(x); }

// params: Match, Mismatch, MismatchS, Branch, BranchS, DeletionN, DeletionWithTag, DeletionWithTagS, Nce, NceS,
//         Merge[4], MergeS[4]  (20 floats).  sumProduct bits: 1 sum-product combiner, 2 SimpleRecursor,
//         4 DenseMatrixF (MutationScorer.hpp:93-99's SimpleQvRecursor / SseQvRecursor / Sparse* typedefs)
void* qorc_scorer_new(const char* tpl, const float* params, int moves, float scoreDiff, float fastThr, float addThr,
                      int sumProduct)
{
    MultiReadScorer* s = new MultiReadScorer();
    QuiverConfig c;
    float* f[10] = {&c.qv.Match, &c.qv.Mismatch, &c.qv.MismatchS, &c.qv.Branch, &c.qv.BranchS, &c.qv.DeletionN,
                    &c.qv.DeletionWithTag, &c.qv.DeletionWithTagS, &c.qv.Nce, &c.qv.NceS};
    for (int k = 0; k < 10; ++k) *f[k] = params[k];
    for (int k = 0; k < 4; ++k) {
        c.qv.Merge[k] = params[10 + k];
        c.qv.MergeS[k] = params[14 + k];
    }
    c.moves = moves;
    c.scoreDiff = scoreDiff;
    c.fastScoreThreshold = fastThr;
    c.addThreshold = addThr;
    c.sumProduct = (sumProduct & 1) != 0;
    c.simple = (sumProduct & 2) != 0;   // bit 1: SimpleRecursor, bit 2: DenseMatrixF (see qorc_scorer_new)
    c.dense = (sumProduct & 4) != 0;
    s->configs.InsertAs("*", c);
    s->Init(tpl);
    return s;
}

void qorc_scorer_free(void* h) { delete static_cast<MultiReadScorer*>(h); }

// features: 5 arrays of I floats (ins, subs, del, delTag (as float char codes), merge); NULL = zeros
int qorc_scorer_add_read(void* h, const char* seq, const float* ins, const float* subs, const float* del,
                         const float* delTag, const float* merge, int strand, int ts, int te, float threshold,
                         int useConfigThreshold)
{
    MultiReadScorer* s = static_cast<MultiReadScorer*>(h);
    MappedRead mr;
    mr.read.seq = seq;
    const size_t I = mr.read.seq.size();
    auto fill = [&](std::vector<float>& v, const float* src, float dflt) {
        v.assign(I, dflt);
        if (src)
            for (size_t i = 0; i < I; ++i) v[i] = src[i];
    };
    fill(mr.read.ins, ins, 0.0f);
    fill(mr.read.subs, subs, 0.0f);
    fill(mr.read.del, del, 0.0f);
    fill(mr.read.delTag, delTag, 0.0f);   // QvSequenceFeatures(seq): zero-filled tracks (Features.cpp:75-88)
    fill(mr.read.merge, merge, 0.0f);
    mr.strand = strand;
    mr.ts = ts;
    mr.te = te;
    try {
        const float thr = useConfigThreshold ? s->configs.At("*").addThreshold : threshold;
        return s->AddRead(mr, thr) ? 1 : 0;
    } catch (...) {
        return -1;
    }
}

static Mut MakeMut(int type, int start, int end, const char* bases) { return Mut(type, start, end, bases ? bases : ""); }

float qorc_scorer_score(void* h, int type, int start, int end, const char* bases, int fast)
{
    MultiReadScorer* s = static_cast<MultiReadScorer*>(h);
    const Mut m = MakeMut(type, start, end, bases);
    return fast ? s->FastScore(m) : s->Score(m);
}

int qorc_scorer_scores(void* h, int type, int start, int end, const char* bases, float unscored, float* out)
{
    MultiReadScorer* s = static_cast<MultiReadScorer*>(h);
    const std::vector<float> v = s->Scores(MakeMut(type, start, end, bases), unscored);
    for (size_t k = 0; k < v.size(); ++k) out[k] = v[k];
    return (int)v.size();
}

int qorc_scorer_is_favorable(void* h, int type, int start, int end, const char* bases, int fast)
{
    MultiReadScorer* s = static_cast<MultiReadScorer*>(h);
    const Mut m = MakeMut(type, start, end, bases);
    return fast ? (s->FastIsFavorable(m) ? 1 : 0) : ((double)s->Score(m) > 0.04 ? 1 : 0);
}

// MutationScorer<R>::ScoreMutation on read r's own scorer (read coordinates; absolute score)
float qorc_ms_score(void* h, int r, int type, int start, int end, const char* bases)
{
    MultiReadScorer* s = static_cast<MultiReadScorer*>(h);
    ReadState& rs = s->reads.at(r);
    return rs.sc ? rs.sc->ScoreMutation(MakeMut(type, start, end, bases)) : 0.0f;
}

float qorc_scorer_baseline(void* h) { return static_cast<MultiReadScorer*>(h)->Baseline(); }
int qorc_scorer_num_reads(void* h) { return (int)static_cast<MultiReadScorer*>(h)->reads.size(); }

int qorc_scorer_read_info(void* h, int r, int* active, int* ts, int* te, float* score, int* flips, long long* usedA,
                          long long* usedB, long long* allocA, long long* allocB)
{
    MultiReadScorer* s = static_cast<MultiReadScorer*>(h);
    const ReadState& rs = s->reads.at(r);
    *active = rs.active ? 1 : 0;
    *ts = rs.mr.ts;
    *te = rs.mr.te;
    *score = rs.sc ? rs.sc->Score() : 0.0f;
    *flips = rs.sc ? rs.sc->flips : -1;
    *usedA = rs.sc ? rs.sc->alpha.UsedEntries() : 0;
    *usedB = rs.sc ? rs.sc->beta.UsedEntries() : 0;
    *allocA = rs.sc ? rs.sc->alpha.AllocatedEntries() : 0;
    *allocB = rs.sc ? rs.sc->beta.AllocatedEntries() : 0;
    return 0;
}

// alpha (which = 0) or beta (1) cell of read r; 0 if the read has no scorer
float qorc_scorer_cell(void* h, int r, int which, int i, int j)
{
    MultiReadScorer* s = static_cast<MultiReadScorer*>(h);
    const ReadState& rs = s->reads.at(r);
    if (!rs.sc) return 0.0f;
    return which == 0 ? rs.sc->alpha.Get(i, j) : rs.sc->beta.Get(i, j);
}

int qorc_scorer_template(void* h, char* out, int cap)
{
    MultiReadScorer* s = static_cast<MultiReadScorer*>(h);
    const int n = (int)s->fwd.size();
    if (n + 1 > cap) return -n;
    std::memcpy(out, s->fwd.c_str(), n + 1);
    return n;
}

int qorc_scorer_apply(void* h, int n, const int* types, const int* starts, const int* ends, const char* bases)
{
    MultiReadScorer* s = static_cast<MultiReadScorer*>(h);
    std::vector<Mut> muts;
    for (int k = 0; k < n; ++k)
        muts.push_back(Mut(types[k], starts[k], ends[k], types[k] == DEL ? std::string() : std::string(1, bases[k])));
    try {
        s->ApplyMutations(muts);
    } catch (...) {
        return -1;
    }
    return 0;
}

int qorc_refine(void* h, int maxIter, int sep, int nbhd, long* nTested, long* nApplied)
{
    *nTested = 0;
    *nApplied = 0;
    try {
        return Refine(*static_cast<MultiReadScorer*>(h), maxIter, sep, nbhd, nTested, nApplied) ? 1 : 0;
    } catch (...) {
        return -1;
    }
}

int qorc_qvs(void* h, int* out, int cap)
{
    const std::vector<int> q = ConsensusQVs(*static_cast<MultiReadScorer*>(h));
    if ((int)q.size() > cap) return -(int)q.size();
    for (size_t k = 0; k < q.size(); ++k) out[k] = q[k];
    return (int)q.size();
}

int qorc_scorer_alignment(void* h, int r, char* target, char* query, int cap)
{
    MultiReadScorer* m = static_cast<MultiReadScorer*>(h);
    const ReadState& rs = m->reads.at(r);
    if (!rs.sc) return -2;
    if (rs.sc->rec.Cb.sumProduct) return -1;
    std::string t, q;
    if (!Alignment(rs.sc->ev, rs.sc->alpha, rs.sc->rec.moves, &t, &q)) return -2;
    const int n = (int)std::min<size_t>(t.size(), (size_t)std::max(cap - 1, 0));
    memcpy(target, t.data(), n);
    memcpy(query, q.data(), n);
    target[n] = query[n] = 0;
    return (int)t.size();
}

// QvEvaluator's four moves at listed cells (QvEvaluator.hpp:153-207), NaN outside each move's domain (the
// reference's asserts); out: 4 x n floats, move-major (Inc, Del, Extra, Merge).  Tracks NULL = zeros.
void qorc_eval_moves(const char* seq, const float* ins, const float* subs, const float* del, const float* delTag,
                     const float* merge, const char* tpl, const float* params, int pinStart, int pinEnd,
                     const int* ci, const int* cj, int n, float* out)
{
    Evaluator e;
    e.rd.seq = seq;
    const size_t I = e.rd.seq.size();
    auto fill = [&](std::vector<float>& v, const float* src) {
        v.assign(I, 0.0f);
        if (src)
            for (size_t i = 0; i < I; ++i) v[i] = src[i];
    };
    fill(e.rd.ins, ins);
    fill(e.rd.subs, subs);
    fill(e.rd.del, del);
    fill(e.rd.delTag, delTag);
    fill(e.rd.merge, merge);
    float* f[10] = {&e.pm.Match, &e.pm.Mismatch, &e.pm.MismatchS, &e.pm.Branch, &e.pm.BranchS, &e.pm.DeletionN,
                    &e.pm.DeletionWithTag, &e.pm.DeletionWithTagS, &e.pm.Nce, &e.pm.NceS};
    for (int k = 0; k < 10; ++k) *f[k] = params[k];
    for (int k = 0; k < 4; ++k) {
        e.pm.Merge[k] = params[10 + k];
        e.pm.MergeS[k] = params[14 + k];
    }
    e.tpl = tpl;
    e.pinStart = pinStart != 0;
    e.pinEnd = pinEnd != 0;
    const int Ii = e.I(), J = e.J();
    const float nan = std::numeric_limits<float>::quiet_NaN();
    for (int k = 0; k < n; ++k) {
        const int i = ci[k], j = cj[k];
        out[k] = (i >= 0 && i < Ii && j >= 0 && j < J) ? e.Inc(i, j) : nan;
        out[n + k] = (i >= 0 && i <= Ii && j >= 0 && j < J) ? e.Del(i, j) : nan;
        out[2 * n + k] = (i >= 0 && i < Ii && j >= 0 && j <= J) ? e.Extra(i, j) : nan;
        out[3 * n + k] = (i >= 0 && i < Ii && j >= 0 && j < J - 1) ? e.Merge(i, j) : nan;
    }
}

}  // extern "C"
