// pbccs_amd/csrc/quiver_kernels.hip -- Quiver recursions on gfx950.
//
//   k_qfill    one lane per read: RecursorBase::FillAlphaBeta (detail/RecursorBase.cpp:70-116) over the
//              SSE recursor's fills (SseRecursor.cpp:73-353) into double-buffered band arenas.
//   k_qscore   one lane per (mutation, read): MutationScorer::ScoreMutation (Quiver/MutationScorer.cpp:
//              113-226) -- ExtendAlpha + LinkAlphaBeta in the middle, ExtendAlpha to the end, ExtendBeta
//              (SimpleRecursor.cpp:407-495) at the start, a whole FillAlpha for tiny windows.
// The 4-row SSE blocks are evaluated row by row in the reference's order: the block terms (Inc, Merge,
// Del, each combined from -FLT_MAX), then the serial Extra cascade, then the block's min / max for the
// band test -- every value equals the SSE lane's.
#include "quiver_kernels.hpp"

namespace pbccs {
namespace quiver {
namespace {

// ---- RangeGuide / RowRange (detail/RecursorBase-inl.hpp:49-114) ----------------------------------------
__device__ __forceinline__ void row_range(const QBand& m, int j, float scoreDiff, int* ob, int* oe)
{
    int b = m.range[j].x, e = m.range[j].y;
    int maxRow = b;
    float maxScore = m.Get(maxRow, j);
    // the first maximum, scanning down (strict '>'); loads issued 8 at a time so that one lane's serial scan
    // waits on memory once per 8 rows, not once per row
    int i = b + 1;
    for (; i + 8 <= e; i += 8) {
        float s[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) s[q] = m.Get(i + q, j);
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (s[q] > maxScore) { maxRow = i + q; maxScore = s[q]; }
    }
    for (; i < e; ++i) {
        const float s = m.Get(i, j);
        if (s > maxScore) { maxRow = i; maxScore = s; }
    }
    const float thr = maxScore - scoreDiff;
    for (i = b; i < maxRow && m.Get(i, j) < thr; ++i) {}
    b = i;
    for (i = e - 1; i >= maxRow && m.Get(i, j) < thr; --i) {}
    *ob = b;
    *oe = i + 1;
}

__device__ __forceinline__ void range_guide(int j, const QBand* guide, const QBand* self, float scoreDiff, int* hb, int* he)
{
    const bool useG = guide && !guide->Empty(j);
    const bool useS = self && !self->Empty(j);
    if (!useG && !useS) return;
    int b = *hb, e = *he, rb, re;
    if (useG) { row_range(*guide, j, scoreDiff, &rb, &re); b = min(rb, b); e = max(re, e); }
    if (useS) { row_range(*self, j, scoreDiff, &rb, &re); b = min(rb, b); e = max(re, e); }
    *hb = b;
    *he = e;
}

__device__ __forceinline__ void put(const QBand& m, long long k, float v, bool& ovf)
{
    if (k < m.cap) m.val[k] = v;
    else ovf = true;
}

// Where column j's first used row goes in its arena: packed after the previous columns (SparseMatrixF), or
// at j * (I + 1) + row (DenseMatrixF: every cell has its place, DenseMatrix-inl.hpp:212-221).
__device__ __forceinline__ long long col_base(const QEval& e, int j, int beginRow, long long used)
{
    return e.p->dense ? (long long)j * (e.I() + 1) + beginRow : used;
}
// values an arena must hold for one pass of `used` entries
__device__ __forceinline__ long long values_needed(const QEval& e, long long used)
{
    return e.p->dense ? (long long)(e.J() + 1) * (e.I() + 1) : used;
}

// ---- SseRecursor::FillAlpha (SseRecursor.cpp:73-213) -----------------------------------------------------
// `prev`: this matrix's previous pass (RangeGuide's self hint); `out`: the arena written now.  Rows come
// top-down, so column j's cells are appended at `used` as they are produced.
__device__ __forceinline__ long long fill_alpha(const QEval& e, const QBand* guide, const QBand* prev, const QBand& out,
                                QAlloc* alloc, bool allocExists, bool& ovf)
{
    const int I = e.I(), J = e.J();
    const bool sp = e.p->sumProduct != 0;
    const bool merge = (e.p->moves & kMerge) != 0;
    const float sd = e.p->scoreDiff;
    long long used = 0;
    int hb = 0, he = 0;
    for (int j = 0; j <= J; ++j) {
        range_guide(j, guide, prev, sd, &hb, &he);
        const int reqEnd = min(I + 1, he);
        float score = kNegInf, thr = kNegInf, mx = kNegInf;
        if (alloc) alloc_start(alloc[j], allocExists, hb, he, I + 1);
        const int beginRow = hb;
        const long long base = col_base(e, j, beginRow, used);
        out.off[j] = (int)min(base, (long long)0x7fffffff);
        out.range[j] = make_int2(beginRow, beginRow);   // grows with each row, so reads of it stay exact
        auto set = [&](int r, float v) {
            put(out, base + (r - beginRow), v, ovf);
            out.range[j].y = r + 1;
            if (alloc) alloc_set(alloc[j], r, I + 1);
        };
        int i;
        if (e.p->simple) {   // SimpleRecursor::FillAlpha (Quiver/SimpleRecursor.cpp:60-135): row by row
            for (i = beginRow; i < I + 1 && (score >= thr || i < reqEnd); ++i) {
                score = kNegInf;
                if (i == 0 && j == 0) score = 0.0f;
                if (i > 0 && j > 0) score = comb(sp, score, out.Get(i - 1, j - 1) + e.Inc(i - 1, j - 1));
                if (i > 0) score = comb(sp, score, out.Get(i - 1, j) + e.Extra(i - 1, j));
                if (j > 0) score = comb(sp, score, out.Get(i, j - 1) + e.Del(i, j - 1));
                if (merge && j > 1 && i > 0) score = comb(sp, score, out.Get(i - 1, j - 2) + e.Merge(i - 1, j - 2));
                set(i, score);
                if (score > mx) { mx = score; thr = mx - sd; }
            }
        } else {
        for (i = beginRow; (i == 0 || (I - i + 1) % 4 != 0) && i <= I; i++) {
            score = kNegInf;
            if (i == 0 && j == 0) score = 0.0f;
            if (i > 0 && j > 0) score = comb(sp, score, out.Get(i - 1, j - 1) + e.Inc(i - 1, j - 1));
            if (merge && i > 0 && j > 1) score = comb(sp, score, out.Get(i - 1, j - 2) + e.Merge(i - 1, j - 2));
            if (j > 0) score = comb(sp, score, out.Get(i, j - 1) + e.Del(i, j - 1));
            if (i > 0) score = comb(sp, score, out.Get(i - 1, j) + e.Extra(i - 1, j));
            set(i, score);
            if (score > mx) { mx = score; thr = mx - sd; }
        }
        for (; i <= I && (score >= thr || i < reqEnd); i += 4) {
            float s5[5];
            s5[0] = out.Get(i - 1, j);
            for (int k = 0; k < 4; ++k) {
                const int r = i + k;
                float v = kNegInf;
                if (j > 0) v = comb4(sp, v, out.Get(r - 1, j - 1) + e.Inc(r - 1, j - 1));
                if (merge && j >= 2) v = comb4(sp, v, out.Get(r - 1, j - 2) + e.Merge(r - 1, j - 2));
                if (j > 0) v = comb4(sp, v, out.Get(r, j - 1) + e.Del(r, j - 1));
                s5[k + 1] = v;
            }
            for (int ii = 1; ii < 5; ++ii) {   // Extra cascade (:175-183)
                s5[ii] = comb(sp, s5[ii], s5[ii - 1] + e.Extra(i + ii - 2, j));
                set(i + ii - 1, s5[ii]);
            }
            float pmax = s5[1], pmin = s5[1];   // std::max_element / std::min_element
            for (int ii = 2; ii < 5; ++ii) {
                if (pmax < s5[ii]) pmax = s5[ii];
                if (s5[ii] < pmin) pmin = s5[ii];
            }
            score = pmin;
            if (pmax > mx) { mx = pmax; thr = mx - sd; }
        }
        }
        const int endRow = i;
        out.range[j] = make_int2(beginRow, endRow);
        used += endRow - beginRow;
        he = endRow;
        for (i = beginRow; i < endRow && out.Get(i, j) < thr; ++i) {}
        hb = i;
    }
    return used;   // UsedEntries (the reband test); the arena needs values_needed(e, used)
}

// ---- SseRecursor::FillBeta (SseRecursor.cpp:216-353) -----------------------------------------------------
// Rows come bottom-up and the column's first row is known only at its end: cells go to the read's column
// buffer (indexed by row) and are copied top-down into the arena when the column is finished.
__device__ __forceinline__ long long fill_beta(const QEval& e, const QBand* guide, const QBand* prev, const QBand& out,
                               float* colbuf, QAlloc* alloc, bool allocExists, bool& ovf)
{
    const int I = e.I(), J = e.J();
    const bool sp = e.p->sumProduct != 0;
    const bool merge = (e.p->moves & kMerge) != 0;
    const float sd = e.p->scoreDiff;
    long long used = 0;
    int hb = I + 1, he = I + 1;
    for (int j = J; j >= 0; --j) {
        range_guide(j, guide, prev, sd, &hb, &he);
        const int reqBegin = max(0, hb);
        float score = kNegInf, thr = kNegInf, mx = kNegInf;
        if (alloc) alloc_start(alloc[j], allocExists, hb, he, I + 1);
        const int endRow = he;
        int lo = endRow;   // rows [lo, endRow) of this column are in colbuf
        auto get = [&](int r, int c) -> float {
            if (c == j) return (r >= lo && r < endRow) ? colbuf[r] : kNegInf;
            return out.Get(r, c);
        };
        auto set = [&](int r, float v) {
            colbuf[r] = v;
            lo = r;
            if (alloc) alloc_set(alloc[j], r, I + 1);
        };
        int i;
        if (e.p->simple) {   // SimpleRecursor::FillBeta (Quiver/SimpleRecursor.cpp:138-222): row by row
            for (i = endRow - 1; i >= 0 && (score >= thr || i >= reqBegin); --i) {
                score = kNegInf;
                if (i == I && j == J) score = 0.0f;
                if (i < I && j < J) score = comb(sp, score, get(i + 1, j + 1) + e.Inc(i, j));
                if (i < I) score = comb(sp, score, get(i + 1, j) + e.Extra(i, j));
                if (j < J) score = comb(sp, score, get(i, j + 1) + e.Del(i, j));
                if (merge && j < J - 1 && i < I) score = comb(sp, score, get(i + 1, j + 2) + e.Merge(i, j));
                set(i, score);
                if (score > mx) { mx = score; thr = mx - sd; }
            }
            i = i - 3;   // so that beginRow = i + 4 below is the first row set
        } else {
        for (i = endRow - 1; (i == I || (i + 1) % 4 != 0) && i >= 0; i--) {
            score = kNegInf;
            if (i == I && j == J) score = 0.0f;
            if (i < I && j < J) score = comb(sp, score, get(i + 1, j + 1) + e.Inc(i, j));
            if (merge && j < J - 1 && i < I) score = comb(sp, score, get(i + 1, j + 2) + e.Merge(i, j));
            if (j < J) score = comb(sp, score, get(i, j + 1) + e.Del(i, j));
            if (i < I) score = comb(sp, score, get(i + 1, j) + e.Extra(i, j));
            set(i, score);
            if (score > mx) { mx = score; thr = mx - sd; }
        }
        i = i - 3;
        for (; i >= 0 && (score >= thr || i >= reqBegin); i -= 4) {
            float s5[5];
            for (int k = 0; k < 4; ++k) {
                const int r = i + k;
                float v = kNegInf;
                if (i < I && j < J) v = comb4(sp, v, get(r + 1, j + 1) + e.Inc(r, j));
                if (merge && j < J - 1 && i < I) v = comb4(sp, v, get(r + 1, j + 2) + e.Merge(r, j));
                if (j < J) v = comb4(sp, v, get(r, j + 1) + e.Del(r, j));
                s5[k] = v;
            }
            s5[4] = get(i + 4, j);
            for (int ii = 3; ii >= 0; ii--) {
                s5[ii] = comb(sp, s5[ii], s5[ii + 1] + e.Extra(i + ii, j));
                set(i + ii, s5[ii]);
            }
            float pmax = s5[0], pmin = s5[0];
            for (int ii = 1; ii < 4; ++ii) {
                if (pmax < s5[ii]) pmax = s5[ii];
                if (s5[ii] < pmin) pmin = s5[ii];
            }
            score = pmin;
            if (pmax > mx) { mx = pmax; thr = mx - sd; }
        }
        }
        const int beginRow = i + 4;
        const long long base = col_base(e, j, beginRow, used);
        out.off[j] = (int)min(base, (long long)0x7fffffff);
        for (int r = beginRow; r < endRow; ++r) put(out, base + (r - beginRow), colbuf[r], ovf);
        out.range[j] = make_int2(beginRow, endRow);
        used += endRow - beginRow;
        hb = beginRow;
        for (i = endRow; i > beginRow && out.Get(i - 1, j) < thr; i--) {}
        he = i;
    }
    return used;   // UsedEntries; the arena needs values_needed(e, used)
}

// ---- SseRecursor::ExtendAlpha (SseRecursor.cpp:433-551) --------------------------------------------------
__device__ __forceinline__ void extend_alpha(const QEval& e, const QBand& a, int beginColumn, const QBand& ext, int numExt, bool& ovf)
{
    const bool sp = e.p->sumProduct != 0;
    const bool merge = (e.p->moves & kMerge) != 0;
    long long used = 0;
    for (int c = 0; c < numExt; c++) {
        const int j = beginColumn + c;
        int beginRow, endRow;
        if (j < a.cols) { beginRow = a.range[j].x; endRow = a.range[j].y; }
        else { beginRow = a.range[a.cols - 1].x; endRow = e.I() + 1; }
        ext.off[c] = (int)used;
        ext.range[c] = make_int2(beginRow, beginRow);
        auto set = [&](int r, float v) {
            put(ext, used + (r - beginRow), v, ovf);
            ext.range[c].y = r + 1;
        };
        auto prevCol = [&](int r) { return c == 0 ? a.Get(r, j - 1) : ext.Get(r, c - 1); };
        int i;
        for (i = beginRow; (i == 0 || (endRow - i) % 4 != 0) && i < endRow; i++) {
            float score = kNegInf;
            if (i > 0) {
                score = comb(sp, score, prevCol(i - 1) + e.Inc(i - 1, j - 1));
                score = comb(sp, score, ext.Get(i - 1, c) + e.Extra(i - 1, j));
                if (merge) score = comb(sp, score, a.Get(i - 1, j - 2) + e.Merge(i - 1, j - 2));
            }
            score = comb(sp, score, prevCol(i) + e.Del(i, j - 1));
            set(i, score);
        }
        for (; i < endRow - 3; i += 4) {
            float s5[5];
            s5[0] = ext.Get(i - 1, c);
            for (int k = 0; k < 4; ++k) {
                const int r = i + k;
                float v = kNegInf;
                v = comb4(sp, v, prevCol(r - 1) + e.Inc(r - 1, j - 1));
                if (merge && j >= 2) v = comb4(sp, v, a.Get(r - 1, j - 2) + e.Merge(r - 1, j - 2));
                v = comb4(sp, v, prevCol(r) + e.Del(r, j - 1));
                s5[k + 1] = v;
            }
            for (int ii = 1; ii < 5; ii++) {
                s5[ii] = comb(sp, s5[ii], s5[ii - 1] + e.Extra(i + ii - 2, j));
                set(i + ii - 1, s5[ii]);
            }
        }
        ext.range[c] = make_int2(beginRow, endRow);
        used += endRow - beginRow;
    }
}

// ---- SimpleRecursor::ExtendAlpha (Quiver/SimpleRecursor.cpp:303-388) --------------------------------------
// Row by row; the merge term reads alpha(i - 1, j - 2) for every extension column, as the reference does.
__device__ __forceinline__ void extend_alpha_simple(const QEval& e, const QBand& a, int beginColumn, const QBand& ext,
                                                    int numExt, bool& ovf)
{
    const bool sp = e.p->sumProduct != 0;
    const bool merge = (e.p->moves & kMerge) != 0;
    long long used = 0;
    for (int c = 0; c < numExt; c++) {
        const int j = beginColumn + c;
        int beginRow, endRow;
        if (j < a.cols) { beginRow = a.range[j].x; endRow = a.range[j].y; }
        else { beginRow = a.range[a.cols - 1].x; endRow = e.I() + 1; }
        ext.off[c] = (int)used;
        ext.range[c] = make_int2(beginRow, beginRow);
        for (int i = beginRow; i < endRow; i++) {
            float score = kNegInf;
            if (i > 0 && j > 0) {
                const float prev = c == 0 ? a.Get(i - 1, j - 1) : ext.Get(i - 1, c - 1);
                score = comb(sp, score, prev + e.Inc(i - 1, j - 1));
            }
            if (i > 0) score = comb(sp, score, ext.Get(i - 1, c) + e.Extra(i - 1, j));
            if (j > 0) {
                const float prev = c == 0 ? a.Get(i, j - 1) : ext.Get(i, c - 1);
                score = comb(sp, score, prev + e.Del(i, j - 1));
            }
            if (merge && j > 1 && i > 0) score = comb(sp, score, a.Get(i - 1, j - 2) + e.Merge(i - 1, j - 2));
            put(ext, used + (i - beginRow), score, ovf);
            ext.range[c].y = i + 1;
        }
        ext.range[c] = make_int2(beginRow, endRow);
        used += max(0, endRow - beginRow);
    }
}

// ---- SimpleRecursor::ExtendBeta (Quiver/SimpleRecursor.cpp:407-495) ---------------------------------------
__device__ __forceinline__ void extend_beta(const QEval& e, const QBand& b, int lastColumn, const QBand& ext, int numExt,
                            int lengthDiff, bool& ovf)
{
    const bool sp = e.p->sumProduct != 0;
    const bool merge = (e.p->moves & kMerge) != 0;
    const int I = e.I();
    const int J = b.cols - 1;
    const int lastExt = numExt - 1;
    long long used = 0;
    for (int j = lastColumn; j > lastColumn - numExt; j--) {
        const int jp = j + lengthDiff;
        const int c = lastExt - (lastColumn - j);
        int beginRow, endRow;
        if (j < 0) { beginRow = 0; endRow = b.range[0].y; }
        else { beginRow = b.range[j].x; endRow = b.range[j].y; }
        ext.off[c] = (int)used;
        // rows are produced bottom-up and only rows below the one being computed are still unset; they are
        // never read (the column's reads are ext(i + 1, c)), so the final range is valid from the start
        ext.range[c] = make_int2(beginRow, endRow);
        for (int i = endRow - 1; i >= beginRow; i--) {
            float score = kNegInf;
            if (i < I && j < J) {
                const float prev = (c == lastExt) ? b.Get(i + 1, j + 1) : ext.Get(i + 1, c + 1);
                score = comb(sp, score, prev + e.Inc(i, jp));
            }
            if (i < I) score = comb(sp, score, ext.Get(i + 1, c) + e.Extra(i, jp));
            if (j < J) {
                const float prev = (c == lastExt) ? b.Get(i, j + 1) : ext.Get(i, c + 1);
                score = comb(sp, score, prev + e.Del(i, jp));
            }
            if (merge && j < J - 1 && i < I) score = comb(sp, score, b.Get(i + 1, j + 2) + e.Merge(i, jp));
            put(ext, used + (i - beginRow), score, ovf);
        }
        used += max(0, endRow - beginRow);
    }
}

// ---- SseRecursor::LinkAlphaBeta (SseRecursor.cpp:355-431) ------------------------------------------------
__device__ __forceinline__ float link_alpha_beta(const QEval& e, const QBand& a, int ac, const QBand& b, int bc, int absc)
{
    const bool sp = e.p->sumProduct != 0;
    const bool merge = (e.p->moves & kMerge) != 0;
    const int I = e.I();
    const int ub = min(min(a.range[ac - 2].x, a.range[ac - 1].x), min(b.range[bc].x, b.range[bc + 1].x));
    const int ue = max(max(a.range[ac - 2].y, a.range[ac - 1].y), max(b.range[bc].y, b.range[bc + 1].y));
    if (e.p->simple) {   // SimpleRecursor::LinkAlphaBeta (Quiver/SimpleRecursor.cpp:232-295): merges always added
        float v = kNegInf;
        for (int i = ub; i < ue; i++) {
            if (i < I) {
                v = comb(sp, v, a.Get(i, ac - 1) + e.Inc(i, absc - 1) + b.Get(i + 1, bc));
                v = comb(sp, v, a.Get(i, ac - 2) + e.Merge(i, absc - 2) + b.Get(i + 1, bc));
                v = comb(sp, v, a.Get(i, ac - 1) + e.Merge(i, absc - 1) + b.Get(i + 1, bc + 1));
            }
            v = comb(sp, v, a.Get(i, ac - 1) + e.Del(i, absc - 1) + b.Get(i, bc));
        }
        return v;
    }
    float v = kNegInf;
    float v4[4] = {kNegInf, kNegInf, kNegInf, kNegInf};
    int i;
    for (i = ub; i < ue - 4; i += 4) {
        for (int k = 0; k < 4; ++k) {
            const int r = i + k;
            v4[k] = comb4(sp, v4[k], a.Get(r, ac - 1) + e.Inc(r, absc - 1) + b.Get(r + 1, bc));
            if (merge) {
                v4[k] = comb4(sp, v4[k], a.Get(r, ac - 2) + e.Merge(r, absc - 2) + b.Get(r + 1, bc));
                v4[k] = comb4(sp, v4[k], a.Get(r, ac - 1) + e.Merge(r, absc - 1) + b.Get(r + 1, bc + 1));
            }
            v4[k] = comb4(sp, v4[k], a.Get(r, ac - 1) + e.Del(r, absc - 1) + b.Get(r, bc));
        }
    }
    for (; i < ue; i++) {
        if (i < I) {
            v = comb(sp, v, a.Get(i, ac - 1) + e.Inc(i, absc - 1) + b.Get(i + 1, bc));
            if (merge) {
                v = comb(sp, v, a.Get(i, ac - 2) + e.Merge(i, absc - 2) + b.Get(i + 1, bc));
                v = comb(sp, v, a.Get(i, ac - 1) + e.Merge(i, absc - 1) + b.Get(i + 1, bc + 1));
            }
        }
        v = comb(sp, v, a.Get(i, ac - 1) + e.Del(i, absc - 1) + b.Get(i, bc));
    }
    float acc = kNegInf;   // std::accumulate(v_array, v_array + 5, NEG_INF, C::Combine)
    for (int k = 0; k < 4; ++k) acc = comb(sp, acc, v4[k]);
    return comb(sp, acc, v);
}

// ---- per-read views -----------------------------------------------------------------------------------
// A read's four pass arenas (alpha 0, alpha 1, beta 0, beta 1) are computed on demand from their bases: an
// array of QBand indexed by a run-time arena number would live in scratch.
struct ReadView {
    QEval ev;
    int2* range0;
    int* off0;
    float* val0;
    long long colCap, valCap;
    int cols;
    QAlloc* allocA;
    QAlloc* allocB;
    float* colbuf;
    int4* hint;
};

__device__ __forceinline__ QBand arena(const ReadView& v, int k)
{
    QBand m;
    m.range = v.range0 + (long long)k * v.colCap;
    m.off = v.off0 + (long long)k * v.colCap;
    m.val = v.val0 + (long long)k * v.valCap;
    m.cap = v.valCap;
    m.cols = v.cols;
    return m;
}

__device__ __forceinline__ ReadView read_view(const QBatch& B, int r)
{
    ReadView v;
    const int z = B.rZmw[r];
    const int I = B.rLen[r];
    const long long so = B.rSeq[r];
    v.ev.r.seq = B.seqPool + so;
    const float* f = B.featPool + 5 * so;
    v.ev.r.ins = f;
    v.ev.r.subs = f + I;
    v.ev.r.del = f + 2 * I;
    v.ev.r.tag = f + 3 * I;
    v.ev.r.merge = f + 4 * I;
    v.ev.r.I = I;
    const int ts = B.rTs[r], te = B.rTe[r], L = B.zLen[z];
    v.ev.p = B.params + B.rParam[r];
    v.ev.t.base = B.tplPool + (B.rStrand[r] == 0 ? B.zFwd[z] + ts : B.zRev[z] + (L - te));
    v.ev.t.len = te - ts;
    v.ev.t.editPos = -1;
    const long long cb = B.rColBase[r];
    const int cc = B.rColCap[r];
    v.range0 = B.range + cb;
    v.off0 = B.off + cb;
    v.val0 = B.valPool + B.rValBase[r];
    v.colCap = cc;
    v.valCap = B.rValCap[r];
    v.cols = te - ts + 1;
    v.allocA = B.alloc + cb / 2;   // 2 x colCap alloc slots per read (colBase advances by 4 x colCap)
    v.allocB = v.allocA + cc;
    v.colbuf = B.valPool + B.rColBuf[r];
    v.hint = B.hint + cb / 4;
    return v;
}

__device__ __forceinline__ long long used_entries(const QBand& m)
{
    long long s = 0;
    for (int j = 0; j < m.cols; ++j) s += max(0, m.range[j].y - m.range[j].x);
    return s;
}

__device__ __forceinline__ long long allocated_entries(const QAlloc* a, int cols)
{
    long long s = 0;
    for (int j = 0; j < cols; ++j) s += a[j].capacity;
    return s;
}

// ==== cooperative fill: one wavefront per read ===========================================================
// The SSE recursor's fills with the rows of a column spread over the 64 lanes (SseRecursor.cpp:73-353).
// Per column, every lane evaluates its row's Inc / Merge / Del terms from the two previous columns (held in
// an LDS ring indexed by absolute row), then the Extra cascade -- the one serial dependency, kept in the
// reference's row order -- walks the lanes through v_readlane.  Rows are mapped so that the SSE 4-row blocks
// are lane quads: alpha groups start at rows = I + 1 (mod 4), beta groups at rows = 0 (mod 4).  A chunk of 64
// rows is evaluated speculatively; the band's stopping rule (block min against the running max - ScoreDiff,
// or the guide's reqEnd / reqBegin) is then resolved for all 16 quads at once with a max-scan, and rows past
// the stop are dropped before anything is stored.  Cells and band decisions equal the lane fill's.
constexpr int kQCoopMaxRows = 4096;   // reads of up to 4095 bases (three LDS columns: 48 KB)

__device__ __forceinline__ float rl(float x, int k) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), k)); }
// DPP move of a float (gfx9): lanes without a source, or in rows the row mask leaves out, get `old`
template <int CTRL, int ROWMASK>
__device__ __forceinline__ float dpp_f(float old, float x)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(x), CTRL, ROWMASK, 0xF, false));
}
__device__ __forceinline__ float fmax_ref(float a, float b) { return b > a ? b : a; }   // keeps a on ties

__device__ __forceinline__ float wave_max(float x)
{
    for (int o = 32; o > 0; o >>= 1) x = fmax_ref(x, __shfl_xor(x, o, 64));
    return x;
}

// RowRange (RecursorBase-inl.hpp:49-84) over a previous pass's column, cooperatively
__device__ __forceinline__ void coop_row_range(const QBand& m, int j, float sd, int lane, int* ob, int* oe)
{
    const int2 rg = m.range[j];
    const int b = rg.x, e = rg.y;
    // maxRow: the first row holding the maximum (strict '>' scanning down from b)
    float best = kNegInf;
    int bestRow = 0x7fffffff;
    for (int i = b + lane; i < e; i += 64) {
        const float v = m.Get(i, j);
        if (bestRow == 0x7fffffff || v > best) { best = v; bestRow = i; }   // a lane's rows ascend: first max
    }
    const float mxv = wave_max(best);
    int cand = (bestRow != 0x7fffffff && best == mxv) ? bestRow : 0x7fffffff;
    for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o, 64));
    const int maxRow = cand;
    const float thr = mxv - sd;
    // b' = first row in [b, maxRow) with value >= thr, else maxRow
    int nb = maxRow;
    for (int i0 = b; i0 < maxRow; i0 += 64) {
        const int i = i0 + lane;
        const bool hit = i < maxRow && !(m.Get(i, j) < thr);
        const unsigned long long bal = __ballot(hit);
        if (bal) { nb = i0 + __ffsll((long long)bal) - 1; break; }
    }
    // e' = last row in [maxRow, e) with value >= thr, plus one; else maxRow
    int ne = maxRow;
    for (int i1 = e; i1 > maxRow; i1 -= 64) {
        const int i = i1 - 1 - lane;
        const bool hit = i >= maxRow && !(m.Get(i, j) < thr);
        const unsigned long long bal = __ballot(hit);
        if (bal) { ne = i1 - 1 - (__ffsll((long long)bal) - 1) + 1; break; }
    }
    *ob = nb;
    *oe = ne;
}

__device__ __forceinline__ void coop_range_guide(int j, const QBand* guide, const QBand* self, float sd, int lane,
                                                 int* hb, int* he)
{
    const bool useG = guide && !guide->Empty(j);
    const bool useS = self && !self->Empty(j);
    if (!useG && !useS) return;
    int b = *hb, e = *he, rb, re;
    if (useG) { coop_row_range(*guide, j, sd, lane, &rb, &re); b = min(rb, b); e = max(re, e); }
    if (useS) { coop_row_range(*self, j, sd, lane, &rb, &re); b = min(rb, b); e = max(re, e); }
    *hb = b;
    *he = e;
}

// One column of the LDS ring.  Row i lives at v[i & mask]: either the ring holds the read's full height
// (mask = -1, every row its own slot) or it is a band-height window of a power of two of rows -- a column's
// rows [b, e) are then distinct modulo the ring as long as e - b fits it, which coop_column checks (kQTall
// otherwise).
struct LdsCol {
    float* v;
    int b, e;   // valid rows [b, e)
    int mask;
    __device__ __forceinline__ float at(int i) const { return (i >= b && i < e) ? v[i & mask] : kNegInf; }
};

// The read's QV-feature rows [lo, lo + kQWinRows) staged in LDS, row i at slot i & (kQWinRows - 1): a column's
// chunk reads 65 consecutive rows, and the band moves about a row per column, so the window is reloaded (one
// coalesced pass of the wave) only every few hundred columns instead of six HBM/L2 loads per cell.
constexpr int kQWinRows = 128;
struct QWin {
    float* ins;
    float* subs;
    float* del;
    float* tag;
    float* merge;
    char* seq;
    int lo;
};

// Rows [need0, need1] (clamped to the read's [0, I)) in the window; a reload is wave-uniform.  Alpha chunks
// move down, beta chunks up: the window is placed ahead of them.
template <bool BETA>
__device__ __forceinline__ void win_ensure(QWin& w, const QRead& R, int need0, int need1, int lane)
{
    need0 = max(need0, 0);
    need1 = min(need1, R.I - 1);
    if (need0 > need1 || (need0 >= w.lo && need1 < w.lo + kQWinRows)) return;
    const int lo = BETA ? max(0, need1 + 8 - (kQWinRows - 1)) : max(0, need0 - 8);
    __syncthreads();   // (one wave per block) earlier reads of the slots come first
    for (int q = lane; q < kQWinRows; q += 64) {
        const int i = lo + q;
        if (i < R.I) {
            const int k = i & (kQWinRows - 1);
            w.seq[k] = R.seq[i];
            w.ins[k] = R.ins[i];
            w.subs[k] = R.subs[i];
            w.del[k] = R.del[i];
            w.tag[k] = R.tag[i];
            w.merge[k] = R.merge[i];
        }
    }
    __syncthreads();
    w.lo = lo;
}

// QvEvaluator (QvEvaluator.hpp:150-207) over the window, the same expressions as QEval's
struct QEvalWin {
    const QEval& e;
    const QWin& w;
    __device__ __forceinline__ int K(int i) const { return i & (kQWinRows - 1); }
    __device__ __forceinline__ float Inc(int i, int j) const
    {
        const QParams* p = e.p;
        return (w.seq[K(i)] == e.t.at(j)) ? p->Match : p->Mismatch + p->MismatchS * w.subs[K(i)];
    }
    __device__ __forceinline__ float Del(int i, int j) const
    {
        const QParams* p = e.p;
        const float tb = (float)e.t.at(j);
        return (i < e.r.I && tb == w.tag[K(i)]) ? p->DeletionWithTag + p->DeletionWithTagS * w.del[K(i)] : p->DeletionN;
    }
    __device__ __forceinline__ float Extra(int i, int j) const
    {
        const QParams* p = e.p;
        return (j < e.t.len && w.seq[K(i)] == e.t.at(j)) ? p->Branch + p->BranchS * w.ins[K(i)]
                                                          : p->Nce + p->NceS * w.ins[K(i)];
    }
    __device__ __forceinline__ float Merge(int i, int j) const
    {
        const char a = e.t.at(j), b = e.t.at(j + 1), s = w.seq[K(i)];
        if (!(s == a && s == b)) return kNegInf;
        const int k = tpl_code(a);
        return e.p->Merge[k] + e.p->MergeS[k] * w.merge[K(i)];
    }
};

// One column of one pass.  BETA: rows run downwards (lane l <-> row top - l), the chain from row + 1.
// Returns the column's [begin, end) in *ob / *oe and leaves its cells in cur.v (rows of the range) and in
// the arena at out.off[j].  thrOut: the running threshold after the last evaluated block.
template <bool BETA>
__device__ __forceinline__ void coop_column(const QEval& e0, int j, int lane, int hb, int he, const LdsCol& c1,
                                            const LdsCol& c2, float* cur, const QBand& out, long long base, QAlloc* alloc,
                                            bool& ovf, int* ob, int* oe, float* thrOut, int mask, bool& tall, QWin& win,
                                            int* tbOut)
{
    // tbOut: the next column's threshold row (alpha: the first row of the range at or above the final threshold,
    // else endRow; beta: the last such row + 1, else beginRow) when the column took one chunk -- its cells are then
    // still in registers -- else INT_MIN and the caller scans the LDS column
    const QEval& e = e0;
    const QEvalWin ew{e0, win};
    const int I = e.I(), J = e.J();
    const bool sp = e.p->sumProduct != 0;
    const bool merge = (e.p->moves & kMerge) != 0;
    const float sd = e.p->scoreDiff;
    // first row in processing order, the band guard, and the quad alignment
    const int req = BETA ? max(0, hb) : min(I + 1, he);
    const int first = BETA ? he - 1 : hb;
    int chunk;   // alpha: row of lane 0; beta: row of lane 0 (the top row)
    bool prefix;
    if (!BETA) {
        const int gs = first - ((((first - (I + 1)) % 4) + 4) % 4);
        chunk = gs;
        prefix = first != gs || first == 0;
    } else {
        chunk = first | 3;
        prefix = (first & 3) != 3 || first == I;
    }
    float carry = kNegInf;              // chain value of the previous row in processing order
    float score = kNegInf, mx = kNegInf, thr = kNegInf;
    int stop = BETA ? -1 : I + 1;       // alpha: endRow; beta: beginRow
    const bool empty = BETA ? (first < 0) : (first > I);
    bool done = empty;
    if (empty) stop = BETA ? first + 1 : first;
    int nChunks = 0;
    float lastSv = kNegInf;
    bool lastKeep = false;
    for (int c = 0; !done; ++c) {
        nChunks = c + 1;
        // rows of this chunk past the band-height ring would alias the column's first rows: the read is tall
        if ((unsigned)mask < (unsigned)I && (BETA ? first - (chunk - 64 * c - 63) : chunk + 64 * c + 63 - first) > mask) {
            tall = true;
            *ob = *oe = first;
            *thrOut = thr;
            return;
        }
        // feature rows of this chunk: alpha reads rows row - 1 and row, beta row
        if (BETA) win_ensure<true>(win, e.r, chunk - 64 * c - 63, chunk - 64 * c, lane);
        else win_ensure<false>(win, e.r, chunk + 64 * c - 1, chunk + 64 * c + 63, lane);
        const int row = BETA ? chunk - 64 * c - lane : chunk + 64 * c + lane;
        const bool valid = BETA ? (row <= first && row >= 0) : (row >= first && row <= I);
        const int g = lane >> 2;
        const bool pre = prefix && c == 0 && g == 0;
        float v = kNegInf, x = 0.0f;
        bool has = false;
        if (valid) {
            if (!BETA) {
                if (pre) {
                    if (row == 0 && j == 0) v = 0.0f;
                    if (row > 0 && j > 0) v = comb(sp, v, c1.at(row - 1) + ew.Inc(row - 1, j - 1));
                    if (merge && row > 0 && j > 1) v = comb(sp, v, c2.at(row - 1) + ew.Merge(row - 1, j - 2));
                    if (j > 0) v = comb(sp, v, c1.at(row) + ew.Del(row, j - 1));
                } else {
                    if (j > 0) v = comb4(sp, v, c1.at(row - 1) + ew.Inc(row - 1, j - 1));
                    if (merge && j >= 2) v = comb4(sp, v, c2.at(row - 1) + ew.Merge(row - 1, j - 2));
                    if (j > 0) v = comb4(sp, v, c1.at(row) + ew.Del(row, j - 1));
                }
                has = row > 0;
                if (has) x = ew.Extra(row - 1, j);
            } else {
                if (pre) {
                    if (row == I && j == J) v = 0.0f;
                    if (row < I && j < J) v = comb(sp, v, c1.at(row + 1) + ew.Inc(row, j));
                    if (merge && j < J - 1 && row < I) v = comb(sp, v, c2.at(row + 1) + ew.Merge(row, j));
                    if (j < J) v = comb(sp, v, c1.at(row) + ew.Del(row, j));
                } else {
                    if (j < J) v = comb4(sp, v, c1.at(row + 1) + ew.Inc(row, j));
                    if (merge && j < J - 1) v = comb4(sp, v, c2.at(row + 1) + ew.Merge(row, j));
                    if (j < J) v = comb4(sp, v, c1.at(row) + ew.Del(row, j));
                }
                has = row < I;
                if (has) x = ew.Extra(row, j);
            }
        }
        // the Extra cascade, in processing order through the valid lanes
        float sv = valid ? v : kNegInf;
        const int k0 = BETA ? max(0, chunk - 64 * c - first) : max(0, first - (chunk + 64 * c));
        const int k1 = BETA ? min(63, chunk - 64 * c) : min(63, I - (chunk + 64 * c));
        if (!sp) {
            // Viterbi: the cascade sv_k = max(v_k, sv_{k-1} + x_k) (the lane before k0 reads `carry`) has exactly
            // one solution, computed here by Jacobi sweeps from sv = v: each sweep is one DPP shift, add and max
            // on every lane, and the sweeps only rise towards that solution, so the first sweep that changes no
            // lane has reached it -- the same floats as the serial loop, in 1 + (the longest run of rows the
            // Extra move wins) sweeps instead of one serial step per row.
            // (at most k1 - k0 + 2 sweeps: the serial loop's step count bounds them, NaN inputs included)
            for (int it = k0; it <= k1 + 1; ++it) {
                float prev = dpp_f<0x138, 0xF>(carry, sv);   // wave_shr:1; lane 0 reads carry
                if (lane == k0) prev = carry;
                const float nv = has ? comb(false, v, prev + x) : sv;
                const bool changed = nv != sv;
                sv = nv;
                if (__ballot(changed) == 0) break;
            }
            if (k1 >= k0) carry = rl(sv, k1);
        } else {
            for (int k = k0; k <= k1; ++k) {
                if (lane == k && has) sv = comb(sp, v, carry + x);
                carry = rl(sv, k);
            }
        }
        // band stopping rule per quad: gmin = the quad's block min (the prefix quad: its last row), gmax
        const int qb = lane & ~3;
        // the quad's four values in every lane of the quad (DPP quad_perm broadcasts)
        const float q0 = dpp_f<0x00, 0xF>(kNegInf, sv), q1 = dpp_f<0x55, 0xF>(kNegInf, sv),
                    q2 = dpp_f<0xAA, 0xF>(kNegInf, sv), q3 = dpp_f<0xFF, 0xF>(kNegInf, sv);
        float gmin, gmax;
        if (pre) {
            // rows in processing order within the prefix quad: the valid ones, last = the quad's last valid
            gmax = kNegInf;
            gmin = kNegInf;
            auto visit = [&](int t2, float qv) {
                const int rr = BETA ? chunk - (qb + t2) : chunk + qb + t2;
                const bool vv = BETA ? (rr <= first && rr >= 0) : (rr >= first && rr <= I);
                if (vv) {
                    if (qv > gmax) gmax = qv;
                    gmin = qv;
                }
            };
            visit(0, q0);
            visit(1, q1);
            visit(2, q2);
            visit(3, q3);
        } else {   // std::max_element / std::min_element over the block
            gmax = q0;
            gmin = q0;
            if (gmax < q1) gmax = q1;
            if (q1 < gmin) gmin = q1;
            if (gmax < q2) gmax = q2;
            if (q2 < gmin) gmin = q2;
            if (gmax < q3) gmax = q3;
            if (q3 < gmin) gmin = q3;
        }
        // running max before each quad (exclusive scan over quads, seeded with mx): an inclusive DPP max-scan
        // over the lanes (row_shr 1/2/4/8, then row_bcast 15/31), shifted by one lane.  Only a quad's first lane
        // tests (the ballot below), and gmin / gmax are quad-uniform, so "the quad before" is the lane before.
        float inc = gmax;
        inc = fmax_ref(inc, dpp_f<0x111, 0xF>(kNegInf, inc));
        inc = fmax_ref(inc, dpp_f<0x112, 0xF>(kNegInf, inc));
        inc = fmax_ref(inc, dpp_f<0x114, 0xF>(kNegInf, inc));
        inc = fmax_ref(inc, dpp_f<0x118, 0xF>(kNegInf, inc));
        inc = fmax_ref(inc, dpp_f<0x142, 0xA>(kNegInf, inc));   // row_bcast:15
        inc = fmax_ref(inc, dpp_f<0x143, 0xC>(kNegInf, inc));   // row_bcast:31
        const float mxBefore = fmax_ref(mx, dpp_f<0x138, 0xF>(kNegInf, inc));   // wave_shr:1; lane 0: -FLT_MAX
        const float prevMin = dpp_f<0x138, 0xF>(score, gmin);                  // lane 0: the score so far
        const float scoreBefore = prevMin;
        // the quad's block start (its lowest row) and test; the prefix quad never stops
        const int lowRow = BETA ? chunk - 64 * c - qb - 3 : chunk + 64 * c + qb;
        bool ok;
        if (pre) ok = true;
        else {
            // thr = mx - ScoreDiff once some score raised mx; -FLT_MAX (the literal) before
            const float thrB = mxBefore == kNegInf ? kNegInf : mxBefore - sd;
            ok = BETA ? (lowRow >= 0 && (scoreBefore >= thrB || lowRow >= req))
                      : (lowRow <= I && (scoreBefore >= thrB || lowRow < req));
        }
        const unsigned long long fails = __ballot((lane & 3) == 0 && !ok);
        const int stopQuad = fails ? (__ffsll((long long)fails) - 1) >> 2 : 16;
        // rows of the quads before the stop are the column's
        const bool keep = valid && g < stopQuad;
        if (keep) cur[row & mask] = sv;
        lastSv = sv;
        lastKeep = keep;
        // state after the last kept quad
        if (stopQuad > 0) {
            const int lastLane = 4 * stopQuad - 1;
            score = rl(gmin, lastLane);
            mx = fmax_ref(mx, rl(inc, lastLane));
            thr = mx == kNegInf ? kNegInf : mx - sd;
        }
        if (stopQuad < 16) {
            const int lr = BETA ? chunk - 64 * c - 4 * stopQuad - 3 : chunk + 64 * c + 4 * stopQuad;
            stop = BETA ? lr + 4 : lr;
            done = true;
        } else if (BETA ? (chunk - 64 * c - 63 <= 0) : (chunk + 64 * c + 63 >= I)) {
            stop = BETA ? 0 : I + 1;
            done = true;
        }
    }
    const int beginRow = BETA ? stop : first;
    const int endRow = BETA ? first + 1 : stop;
    if (nChunks == 1) {
        // one chunk: its kept cells are the column's rows [beginRow, endRow), still in registers (lane l holds
        // row chunk + l, beta chunk - l): store them and find the threshold row without re-reading LDS
        const int row = BETA ? chunk - lane : chunk + lane;
        if (lastKeep) {
            const long long k = base + (row - beginRow);
            if (k < out.cap) out.val[k] = lastSv;
            else ovf = true;
        }
        const unsigned long long bal = __ballot(lastKeep && !(lastSv < thr));
        if (!BETA) *tbOut = bal ? chunk + __ffsll((long long)bal) - 1 : endRow;
        else *tbOut = bal ? chunk - (__ffsll((long long)bal) - 1) + 1 : beginRow;
    } else {
        *tbOut = INT_MIN;
        // store the column top-down into the arena
        for (int r = beginRow + lane; r < endRow; r += 64) {
            const long long k = base + (r - beginRow);
            if (k < out.cap) out.val[k] = cur[r & mask];
            else ovf = true;
        }
    }
    *ob = beginRow;
    *oe = endRow;
    *thrOut = thr;
}

template <bool BETA>
__device__ long long coop_fill(const QEval& e, const QBand& guideBand, bool useGuide, const QBand& prevBand, bool usePrev,
                               const QBand& out, QAlloc* alloc,
                               bool allocExists, bool& ovf, float* lds, int ldsRows, int4* hint, int lane, QWin& win)
{
    // returns the pass's used cells, or -1 when a column outgrew the band-height ring (kQTall)
    const int I = e.I(), J = e.J();
    const float sd = e.p->scoreDiff;
    // RowRange of the guide and self matrices for every column, up front and one lane per column: both are
    // finished passes, and only RangeGuide's min / max with the running hints is sequential
    for (int j = lane; j <= J; j += 64) {
        int4 h = make_int4(-1, -1, -1, -1);
        if (useGuide && !guideBand.Empty(j)) row_range(guideBand, j, sd, &h.x, &h.y);
        if (usePrev && !prevBand.Empty(j)) row_range(prevBand, j, sd, &h.z, &h.w);
        hint[j] = h;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    // the LDS ring: cur (column being filled), c1 (previous), c2 (the one before), rotated by value
    // a ring shorter than the read (ldsRows a power of two): rows modulo it; else every row has its slot
    const int mask = ldsRows >= I + 1 ? -1 : ldsRows - 1;
    LdsCol cur{lds, 0, 0, mask}, c1{lds + ldsRows, 0, 0, mask}, c2{lds + 2 * ldsRows, 0, 0, mask};
    long long used = 0;
    bool tall = false;
    int hb = BETA ? I + 1 : 0, he = BETA ? I + 1 : 0;
    int4 hNext = hint[BETA ? J : 0];
    for (int s = 0; s <= J; ++s) {
        const int j = BETA ? J - s : s;
        const int4 h = hNext;
        if (s < J) hNext = hint[BETA ? j - 1 : j + 1];   // one column ahead: its latency hides behind this one
        if (h.x >= 0) { hb = min(h.x, hb); he = max(h.y, he); }   // RangeGuide (RecursorBase-inl.hpp:87-114)
        if (h.z >= 0) { hb = min(h.z, hb); he = max(h.w, he); }
        int b, en, tb;
        float thr;
        coop_column<BETA>(e, j, lane, hb, he, c1, c2, cur.v, out, used, nullptr, ovf, &b, &en, &thr, mask, tall, win,
                          &tb);
        if (tall) return -1;
        cur.b = b;
        cur.e = en;
        if (lane == 0) {
            out.off[j] = (int)min(used, (long long)0x7fffffff);
            out.range[j] = make_int2(b, en);
            hint[j] = make_int4(hb, he, b, en);   // for the allocation bookkeeping below
        }
        used += en - b;
        if (tb != INT_MIN) {
            if (!BETA) { he = en; hb = tb; }
            else { hb = b; he = tb; }
        } else if (!BETA) {
            he = en;
            // hb = first row of the column at or above the threshold (else endRow)
            int nb = en;
            for (int i0 = b; i0 < en; i0 += 64) {
                const int i = i0 + lane;
                const bool hit = i < en && !(cur.v[i & mask] < thr);
                const unsigned long long bal = __ballot(hit);
                if (bal) { nb = i0 + __ffsll((long long)bal) - 1; break; }
            }
            hb = nb;
        } else {
            hb = b;
            int ne = b;
            for (int i1 = en; i1 > b; i1 -= 64) {
                const int i = i1 - 1 - lane;
                const bool hit = i >= b && !(cur.v[i & mask] < thr);
                const unsigned long long bal = __ballot(hit);
                if (bal) { ne = i1 - (__ffsll((long long)bal) - 1); break; }
            }
            he = ne;
        }
        const LdsCol old2 = c2;
        c2 = c1;
        c1 = cur;
        cur = old2;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");   // the pass's stores before later passes read them
    // SparseVector allocation bookkeeping (SparseVector-inl.hpp): per column independent, one lane per column,
    // rows in the order the reference sets them
    if (alloc) {
        for (int j = lane; j <= J; j += 64) {
            const int4 h = hint[j];
            QAlloc a = alloc[j];
            alloc_start(a, allocExists, h.x, h.y, I + 1);
            if (!BETA) {
                for (int r = max(h.z, a.ae); r < h.w; ++r) alloc_set(a, r, I + 1);   // rows inside [ab, ae) are no-ops
            } else {
                for (int r = h.w - 1; r >= h.z; --r) alloc_set(a, r, I + 1);
            }
            alloc[j] = a;
        }
    }
    return used;
}


// ==== grouped cooperative fill: four reads per wavefront, one 16-lane DPP row each =======================
// At the default ScoreDiff a Quiver band column is ~10 rows (AddRead of a 2 kb read uses ~9.8 entries per
// column), so a 64-lane wave per read leaves most lanes idle.  k_qfill_grp runs the same column recursion as
// coop_column with a read per DPP row of 16 lanes: the Jacobi Extra cascade and the block max-scan use
// row-local DPP (row_shr), the stopping rule a 16-bit field of the wave's ballot, and every group walks its
// own read (its own pass schedule, divergent but barrier-free).  Per read it keeps a 64-row band ring, a
// 64-row QV-feature window and a 64-base template window in LDS (2.2 KB); a column taller than the ring
// returns kQTall and the host refills the read with k_qfill_coop.
constexpr int kQG = 16;                                   // lanes per read
constexpr int kQGRing = 64;                               // band ring rows per read
constexpr int kQGWin = 64;                                // QV-feature window rows
constexpr int kQGTWin = 64;                               // template window bases
constexpr int kQGLdsFloats = 3 * kQGRing + 5 * kQGWin + (kQGWin + kQGTWin) / 4;

__device__ __forceinline__ unsigned gballot(bool p, int g) { return (unsigned)((__ballot(p) >> (16 * g)) & 0xFFFFull); }
__device__ __forceinline__ float gread(float x, int g, int k) { return __shfl(x, 16 * g + k, 64); }
__device__ __forceinline__ void wave_lds_order()   // LDS stores of some lanes before later loads of others
{
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

struct QGWin {   // the group's LDS: ring (3 x 64 floats), then the five feature tracks, read bases, template bases
    float* base;
    int lo, tlo;
    __device__ __forceinline__ float* ring() const { return base; }
    __device__ __forceinline__ float* track(int t) const { return base + 3 * kQGRing + t * kQGWin; }
    __device__ __forceinline__ char* seq() const { return reinterpret_cast<char*>(base + 3 * kQGRing + 5 * kQGWin); }
    __device__ __forceinline__ char* tpl() const { return seq() + kQGWin; }
};
struct GRead {   // a read's bases and its five tracks at feat + t * I (ReadView's layout)
    const char* seq;
    const float* feat;
    int I;
};
struct GCol {   // LdsCol with the group ring's fixed mask
    float* v;
    int b, e;
    __device__ __forceinline__ float at(int i) const { return (i >= b && i < e) ? v[i & (kQGRing - 1)] : kNegInf; }
};

template <bool BETA>
__device__ __forceinline__ void gwin_ensure(QGWin& w, const GRead& R, int need0, int need1, int gl)
{
    need0 = max(need0, 0);
    need1 = min(need1, R.I - 1);
    if (need0 > need1 || (need0 >= w.lo && need1 < w.lo + kQGWin)) return;
    const int lo = BETA ? max(0, need1 + 8 - (kQGWin - 1)) : max(0, need0 - 8);
    wave_lds_order();
    for (int q = gl; q < kQGWin; q += kQG) {
        const int i = lo + q;
        if (i < R.I) {
            const int k = i & (kQGWin - 1);
            w.seq()[k] = R.seq[i];
#pragma unroll
            for (int tr = 0; tr < 5; ++tr) w.track(tr)[k] = R.feat[(long long)tr * R.I + i];
        }
    }
    wave_lds_order();
    w.lo = lo;
}

// template bases [need0, need1] (clamped to [0, len)) in the template window
template <bool BETA>
__device__ __forceinline__ void gtwin_ensure(QGWin& w, const char* base, int len, int need0, int need1, int gl)
{
    need0 = max(need0, 0);
    need1 = min(need1, len - 1);
    if (need0 > need1 || (need0 >= w.tlo && need1 < w.tlo + kQGTWin)) return;
    const int lo = BETA ? max(0, need1 + 4 - (kQGTWin - 1)) : max(0, need0 - 4);
    wave_lds_order();
    for (int q = gl; q < kQGTWin; q += kQG) {
        const int j = lo + q;
        if (j < len) w.tpl()[j & (kQGTWin - 1)] = base[j];
    }
    wave_lds_order();
    w.tlo = lo;
}

// QvEvaluator (QvEvaluator.hpp:150-207) over the group's windows, the same expressions as QEval's
struct QEvalG {
    const QParams* p;
    int I, len;
    const QGWin& w;
    __device__ __forceinline__ int K(int i) const { return i & (kQGWin - 1); }
    __device__ __forceinline__ char T(int j) const { return j >= len ? '\0' : w.tpl()[j & (kQGTWin - 1)]; }
    __device__ __forceinline__ char S(int i) const { return w.seq()[K(i)]; }
    __device__ __forceinline__ float F(int t, int i) const { return w.track(t)[K(i)]; }
    __device__ __forceinline__ float Inc(int i, int j) const
    {
        return (S(i) == T(j)) ? p->Match : p->Mismatch + p->MismatchS * F(1, i);
    }
    __device__ __forceinline__ float Del(int i, int j) const
    {
        const float tb = (float)T(j);
        return (i < I && tb == F(3, i)) ? p->DeletionWithTag + p->DeletionWithTagS * F(2, i) : p->DeletionN;
    }
    __device__ __forceinline__ float Extra(int i, int j) const
    {
        return (j < len && S(i) == T(j)) ? p->Branch + p->BranchS * F(0, i) : p->Nce + p->NceS * F(0, i);
    }
    __device__ __forceinline__ float Merge(int i, int j) const
    {
        const char a = T(j), b = T(j + 1), s = S(i);
        if (!(s == a && s == b)) return kNegInf;
        const int k = tpl_code(a);
        return p->Merge[k] + p->MergeS[k] * F(4, i);
    }
};

// coop_column for one read on its 16-lane row (chunks of 16 rows = 4 SSE quads); same outputs
template <bool BETA>
__device__ __forceinline__ void grp_column(const QEvalG& ew, const GRead& R, const char* tbase, int j, int g, int gl,
                                           int hb, int he, const GCol& c1, const GCol& c2, float* cur,
                                           const QBand& out, long long base, bool& ovf, int* ob, int* oe,
                                           float* thrOut, int* tbOut, bool& tall, QGWin& win)
{
    const int I = ew.I, J = ew.len;
    const int mask = kQGRing - 1;
    const bool sp = ew.p->sumProduct != 0;
    const bool merge = (ew.p->moves & kMerge) != 0;
    const float sd = ew.p->scoreDiff;
    const int req = BETA ? max(0, hb) : min(I + 1, he);
    const int first = BETA ? he - 1 : hb;
    int chunk;
    bool prefix;
    if (!BETA) {
        const int gs = first - ((((first - (I + 1)) % 4) + 4) % 4);
        chunk = gs;
        prefix = first != gs || first == 0;
    } else {
        chunk = first | 3;
        prefix = (first & 3) != 3 || first == I;
    }
    float carry = kNegInf;
    float score = kNegInf, mx = kNegInf, thr = kNegInf;
    int stop = BETA ? -1 : I + 1;
    const bool empty = BETA ? (first < 0) : (first > I);
    bool done = empty;
    if (empty) stop = BETA ? first + 1 : first;
    int nChunks = 0;
    float lastSv = kNegInf;
    bool lastKeep = false;
    if (!empty) gtwin_ensure<BETA>(win, tbase, J, BETA ? j : j - 2, BETA ? j + 1 : j, gl);
    for (int c = 0; !done; ++c) {
        nChunks = c + 1;
        if (mask < I && (BETA ? first - (chunk - 16 * c - 15) : chunk + 16 * c + 15 - first) > mask) {
            tall = true;
            *ob = *oe = first;
            *thrOut = thr;
            *tbOut = INT_MIN;
            return;
        }
        if (BETA) gwin_ensure<true>(win, R, chunk - 16 * c - 15, chunk - 16 * c, gl);
        else gwin_ensure<false>(win, R, chunk + 16 * c - 1, chunk + 16 * c + 15, gl);
        const int row = BETA ? chunk - 16 * c - gl : chunk + 16 * c + gl;
        const bool valid = BETA ? (row <= first && row >= 0) : (row >= first && row <= I);
        const int q = gl >> 2;
        const bool pre = prefix && c == 0 && q == 0;
        float v = kNegInf, x = 0.0f;
        bool has = false;
        if (valid) {
            if (!BETA) {
                if (pre) {
                    if (row == 0 && j == 0) v = 0.0f;
                    if (row > 0 && j > 0) v = comb(sp, v, c1.at(row - 1) + ew.Inc(row - 1, j - 1));
                    if (merge && row > 0 && j > 1) v = comb(sp, v, c2.at(row - 1) + ew.Merge(row - 1, j - 2));
                    if (j > 0) v = comb(sp, v, c1.at(row) + ew.Del(row, j - 1));
                } else {
                    if (j > 0) v = comb4(sp, v, c1.at(row - 1) + ew.Inc(row - 1, j - 1));
                    if (merge && j >= 2) v = comb4(sp, v, c2.at(row - 1) + ew.Merge(row - 1, j - 2));
                    if (j > 0) v = comb4(sp, v, c1.at(row) + ew.Del(row, j - 1));
                }
                has = row > 0;
                if (has) x = ew.Extra(row - 1, j);
            } else {
                if (pre) {
                    if (row == I && j == J) v = 0.0f;
                    if (row < I && j < J) v = comb(sp, v, c1.at(row + 1) + ew.Inc(row, j));
                    if (merge && j < J - 1 && row < I) v = comb(sp, v, c2.at(row + 1) + ew.Merge(row, j));
                    if (j < J) v = comb(sp, v, c1.at(row) + ew.Del(row, j));
                } else {
                    if (j < J) v = comb4(sp, v, c1.at(row + 1) + ew.Inc(row, j));
                    if (merge && j < J - 1) v = comb4(sp, v, c2.at(row + 1) + ew.Merge(row, j));
                    if (j < J) v = comb4(sp, v, c1.at(row) + ew.Del(row, j));
                }
                has = row < I;
                if (has) x = ew.Extra(row, j);
            }
        }
        // the Extra cascade through the group's valid lanes, in processing order
        float sv = valid ? v : kNegInf;
        const int k0 = BETA ? max(0, chunk - 16 * c - first) : max(0, first - (chunk + 16 * c));
        const int k1 = BETA ? min(15, chunk - 16 * c) : min(15, I - (chunk + 16 * c));
        if (!sp) {
            // Viterbi: Jacobi sweeps to the cascade's one solution (coop_column), row_shr:1 within the group
            for (int it = k0; it <= k1 + 1; ++it) {
                float prev = dpp_f<0x111, 0xF>(carry, sv);   // row_shr:1; the group's lane 0 reads carry
                if (gl == k0) prev = carry;
                const float nv = has ? comb(false, v, prev + x) : sv;
                const bool changed = nv != sv;
                sv = nv;
                if (gballot(changed, g) == 0) break;
            }
        } else {
            // sum-product: one row per step, the previous row's value one DPP shift away
            for (int k = k0; k <= k1; ++k) {
                float prev = dpp_f<0x111, 0xF>(carry, sv);
                if (gl == k0) prev = carry;
                if (gl == k && has) sv = comb(sp, v, prev + x);
            }
        }
        if (k1 >= k0) carry = gread(sv, g, k1);
        // band stopping rule per quad (coop_column), over the group's four quads
        const int qb = gl & ~3;
        const float q0 = dpp_f<0x00, 0xF>(kNegInf, sv), q1 = dpp_f<0x55, 0xF>(kNegInf, sv),
                    q2 = dpp_f<0xAA, 0xF>(kNegInf, sv), q3 = dpp_f<0xFF, 0xF>(kNegInf, sv);
        float gmin, gmax;
        if (pre) {
            gmax = kNegInf;
            gmin = kNegInf;
            auto visit = [&](int t2, float qv) {
                const int rr = BETA ? chunk - (qb + t2) : chunk + qb + t2;
                const bool vv = BETA ? (rr <= first && rr >= 0) : (rr >= first && rr <= I);
                if (vv) {
                    if (qv > gmax) gmax = qv;
                    gmin = qv;
                }
            };
            visit(0, q0);
            visit(1, q1);
            visit(2, q2);
            visit(3, q3);
        } else {
            gmax = q0;
            gmin = q0;
            if (gmax < q1) gmax = q1;
            if (q1 < gmin) gmin = q1;
            if (gmax < q2) gmax = q2;
            if (q2 < gmin) gmin = q2;
            if (gmax < q3) gmax = q3;
            if (q3 < gmin) gmin = q3;
        }
        // running max before each quad: inclusive row-local DPP max-scan, shifted by one lane
        float inc = gmax;
        inc = fmax_ref(inc, dpp_f<0x111, 0xF>(kNegInf, inc));
        inc = fmax_ref(inc, dpp_f<0x112, 0xF>(kNegInf, inc));
        inc = fmax_ref(inc, dpp_f<0x114, 0xF>(kNegInf, inc));
        inc = fmax_ref(inc, dpp_f<0x118, 0xF>(kNegInf, inc));
        const float mxBefore = fmax_ref(mx, dpp_f<0x111, 0xF>(kNegInf, inc));   // row_shr:1; lane 0: -FLT_MAX
        const float scoreBefore = dpp_f<0x111, 0xF>(score, gmin);               // lane 0: the score so far
        const int lowRow = BETA ? chunk - 16 * c - qb - 3 : chunk + 16 * c + qb;
        bool ok;
        if (pre) ok = true;
        else {
            const float thrB = mxBefore == kNegInf ? kNegInf : mxBefore - sd;
            ok = BETA ? (lowRow >= 0 && (scoreBefore >= thrB || lowRow >= req))
                      : (lowRow <= I && (scoreBefore >= thrB || lowRow < req));
        }
        const unsigned fails = gballot((gl & 3) == 0 && !ok, g);
        const int stopQuad = fails ? (__ffs((int)fails) - 1) >> 2 : 4;
        const bool keep = valid && q < stopQuad;
        if (keep) cur[row & mask] = sv;
        lastSv = sv;
        lastKeep = keep;
        if (stopQuad > 0) {
            const int lastLane = 4 * stopQuad - 1;
            score = gread(gmin, g, lastLane);
            mx = fmax_ref(mx, gread(inc, g, lastLane));
            thr = mx == kNegInf ? kNegInf : mx - sd;
        }
        if (stopQuad < 4) {
            const int lr = BETA ? chunk - 16 * c - 4 * stopQuad - 3 : chunk + 16 * c + 4 * stopQuad;
            stop = BETA ? lr + 4 : lr;
            done = true;
        } else if (BETA ? (chunk - 16 * c - 15 <= 0) : (chunk + 16 * c + 15 >= I)) {
            stop = BETA ? 0 : I + 1;
            done = true;
        }
    }
    const int beginRow = BETA ? stop : first;
    const int endRow = BETA ? first + 1 : stop;
    if (nChunks == 1) {
        const int row = BETA ? chunk - gl : chunk + gl;
        if (lastKeep) {
            const long long k = base + (row - beginRow);
            if (k < out.cap) out.val[k] = lastSv;
            else ovf = true;
        }
        const unsigned bal = gballot(lastKeep && !(lastSv < thr), g);
        if (!BETA) *tbOut = bal ? chunk + __ffs((int)bal) - 1 : endRow;
        else *tbOut = bal ? chunk - (__ffs((int)bal) - 1) + 1 : beginRow;
    } else {
        *tbOut = INT_MIN;
        for (int r = beginRow + gl; r < endRow; r += kQG) {
            const long long k = base + (r - beginRow);
            if (k < out.cap) out.val[k] = cur[r & mask];
            else ovf = true;
        }
    }
    *ob = beginRow;
    *oe = endRow;
    *thrOut = thr;
}

// coop_fill for one read on its 16-lane row
template <bool BETA>
__device__ long long grp_fill(const QEvalG& ew, const GRead& R, const char* tbase, const QBand& guideBand,
                              bool useGuide, const QBand& prevBand, bool usePrev, const QBand& out, QAlloc* alloc,
                              bool allocExists, bool& ovf, float* ring, int4* hint, int g, int gl, QGWin& win)
{
    const int I = ew.I, J = ew.len;
    const float sd = ew.p->scoreDiff;
    const int mask = kQGRing - 1;
    for (int j = gl; j <= J; j += kQG) {
        int4 h = make_int4(-1, -1, -1, -1);
        if (useGuide && !guideBand.Empty(j)) row_range(guideBand, j, sd, &h.x, &h.y);
        if (usePrev && !prevBand.Empty(j)) row_range(prevBand, j, sd, &h.z, &h.w);
        hint[j] = h;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    GCol cur{ring, 0, 0}, c1{ring + kQGRing, 0, 0}, c2{ring + 2 * kQGRing, 0, 0};
    long long used = 0;
    bool tall = false;
    int hb = BETA ? I + 1 : 0, he = BETA ? I + 1 : 0;
    int4 hNext = hint[BETA ? J : 0];
    for (int s = 0; s <= J; ++s) {
        const int j = BETA ? J - s : s;
        const int4 h = hNext;
        if (s < J) hNext = hint[BETA ? j - 1 : j + 1];
        if (h.x >= 0) { hb = min(h.x, hb); he = max(h.y, he); }
        if (h.z >= 0) { hb = min(h.z, hb); he = max(h.w, he); }
        int b, en, tb;
        float thr;
        grp_column<BETA>(ew, R, tbase, j, g, gl, hb, he, c1, c2, cur.v, out, used, ovf, &b, &en, &thr, &tb, tall, win);
        if (tall) return -1;
        cur.b = b;
        cur.e = en;
        if (gl == 0) {
            out.off[j] = (int)min(used, (long long)0x7fffffff);
            out.range[j] = make_int2(b, en);
            hint[j] = make_int4(hb, he, b, en);
        }
        used += en - b;
        if (tb != INT_MIN) {
            if (!BETA) { he = en; hb = tb; }
            else { hb = b; he = tb; }
        } else if (!BETA) {
            he = en;
            int nb = en;
            for (int i0 = b; i0 < en; i0 += kQG) {
                const int i = i0 + gl;
                const unsigned bal = gballot(i < en && !(cur.v[i & mask] < thr), g);
                if (bal) { nb = i0 + __ffs((int)bal) - 1; break; }
            }
            hb = nb;
        } else {
            hb = b;
            int ne = b;
            for (int i1 = en; i1 > b; i1 -= kQG) {
                const int i = i1 - 1 - gl;
                const unsigned bal = gballot(i >= b && !(cur.v[i & mask] < thr), g);
                if (bal) { ne = i1 - (__ffs((int)bal) - 1); break; }
            }
            he = ne;
        }
        const GCol old2 = c2;
        c2 = c1;
        c1 = cur;
        cur = old2;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    if (alloc) {
        for (int j = gl; j <= J; j += kQG) {
            const int4 h = hint[j];
            QAlloc a = alloc[j];
            alloc_start(a, allocExists, h.x, h.y, I + 1);
            if (!BETA) {
                for (int r = max(h.z, a.ae); r < h.w; ++r) alloc_set(a, r, I + 1);
            } else {
                for (int r = h.w - 1; r >= h.z; --r) alloc_set(a, r, I + 1);
            }
            alloc[j] = a;
        }
    }
    return used;
}
}  // namespace

// ---- k_qfill_coop: FillAlphaBeta with one wavefront per read (SparseSse recursors, reads < kQCoopMaxRows) --
// Profiling: the stored cells and algorithmic bytes of a completed fill (every pass's band and column metadata).
__device__ inline void qstat_add(unsigned long long* s, int kind, long long cells, long long cols)
{
    if (!s) return;
    atomicAdd(s + 2 * kind, (unsigned long long)cells);
    atomicAdd(s + 2 * kind + 1, (unsigned long long)(4 * cells + 12 * cols));
}

__global__ void __launch_bounds__(64) k_qfill_coop(QBatch B, const int* __restrict__ reads, int n, int ldsRows,
                                                    int ldsCols)
{
    extern __shared__ float qlds[];
    const int t = blockIdx.x;
    const int lane = threadIdx.x;
    if (t >= n) return;
    const int r = reads[t];
    ReadView v = read_view(B, r);
    const int I = v.ev.I(), J = v.ev.J();
    if (I < 1 || J < 1 || J + 1 > B.rColCap[r] || J + 1 > ldsCols) {
        if (lane == 0) B.rStatus[r] = kQBad;
        return;
    }
    // LDS: the column ring, the QV-feature window, the template window (every column reads its bases)
    float* wf = qlds + 3 * ldsRows;
    QWin win{wf, wf + kQWinRows, wf + 2 * kQWinRows, wf + 3 * kQWinRows, wf + 4 * kQWinRows,
             reinterpret_cast<char*>(wf + 5 * kQWinRows), INT_MIN / 2};
    char* tpl = reinterpret_cast<char*>(wf + 5 * kQWinRows) + kQWinRows;
    for (int j = lane; j < J; j += 64) tpl[j] = v.ev.t.base[j];
    v.ev.t.base = tpl;
    const QEval& e = v.ev;
    for (int k = 0; k < 4; ++k) {
        const QBand m = arena(v, k);
        for (int j = lane; j <= J; j += 64) m.range[j] = make_int2(0, 0);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    bool ovf = false, tall = false;
    long long needA = 0, needB = 0, stCells = 0, stCols = 0;
    int curA = 0, curB = 2;
    bool aPassed = false, bPassed = false;
    auto passA = [&](bool guided) {
        const int nxt = aPassed ? (curA ^ 1) : 0;
        const QBand g = arena(v, curB), self = arena(v, curA), out = arena(v, nxt);
        const long long u = coop_fill<false>(e, g, guided, self, aPassed, out, v.allocA, aPassed, ovf, qlds, ldsRows,
                                             v.hint, lane, win);
        tall = tall || u < 0;
        if (!ovf && u >= 0) { stCells += u; stCols += J + 1; }
        needA = max(needA, u);
        curA = nxt;
        aPassed = true;
        return u;
    };
    auto passB = [&]() {
        const int nxt = bPassed ? (curB ^ 1) : 2;
        const QBand g = arena(v, curA), self = arena(v, curB), out = arena(v, nxt);
        const long long u = coop_fill<true>(e, g, true, self, bPassed, out, v.allocB, bPassed, ovf, qlds, ldsRows,
                                            v.hint, lane, win);
        tall = tall || u < 0;
        if (!ovf && u >= 0) { stCells += u; stCols += J + 1; }
        needB = max(needB, u);
        curB = nxt;
        bPassed = true;
        return u;
    };
    // RecursorBase::FillAlphaBeta (detail/RecursorBase.cpp:70-116) as one loop over the pass schedule, so each
    // pass kind is instantiated once: alpha, beta; the reband triple (alpha, beta, alpha) when either band
    // reached 4% of the matrix; then the flip-flops while alpha and beta disagree.  A tall column ends the
    // fill (kQTall).
    auto a_end = [&]() { return arena(v, curA).Get(I, J); };
    auto b_start = [&]() { return arena(v, curB).Get(0, 0); };
    const int maxSize = (int)(0.5 + 0.04 * (I + 1) * (J + 1));
    long long ua = 0;
    int flips = 0, stage = 0, pending = 0;   // stage 0: first alpha, 1: first beta, 2: reband triple, 3: flip-flops
    for (;;) {
        bool alpha = true, guided = true;
        if (stage == 0) guided = false;
        else if (stage == 1) alpha = false;
        else if (stage == 2) alpha = pending != 2;
        else {
            if (ovf || !((double)fabsf(a_end() - b_start()) > 0.2) || flips > kMaxFlipFlops) break;
            alpha = flips % 2 == 0;
        }
        const long long u = alpha ? passA(guided) : passB();
        if (tall) break;
        if (stage == 0) {
            ua = u;
            stage = 1;
        } else if (stage == 1) {
            ovf = __ballot(ovf) != 0;
            if (!ovf && (ua >= maxSize || u >= maxSize)) {
                stage = 2;
                pending = 3;
                flips += 3;
            } else {
                stage = 3;
            }
        } else if (stage == 2) {
            if (--pending == 0) {
                ovf = __ballot(ovf) != 0;
                stage = 3;
            }
        } else {
            flips++;
            ovf = __ballot(ovf) != 0;
        }
    }
    // AllocatedEntries of both passes: a wave-wide sum over the columns (not a serial walk on lane 0)
    long long capA = 0, capB = 0;
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");   // the last pass's bookkeeping stores come first
    if (!tall && !ovf) {
        for (int j = lane; j <= J; j += 64) {
            capA += v.allocA[j].capacity;
            capB += v.allocB[j].capacity;
        }
        for (int o = 32; o > 0; o >>= 1) {
            capA += __shfl_xor(capA, o, 64);
            capB += __shfl_xor(capB, o, 64);
        }
    }
    if (lane != 0) return;
    if (!tall && !ovf) qstat_add(B.stats, kQStatCoop, stCells, stCols);
    if (tall) {
        B.rStatus[r] = kQTall;
        return;
    }
    B.rUsed[2 * r] = needA;
    B.rUsed[2 * r + 1] = needB;
    if (ovf) {
        B.rStatus[r] = kQOverflow;
        return;
    }
    B.rCurA[r] = curA;
    B.rCurB[r] = curB - 2;
    B.rFlips[r] = flips;
    B.rScore[r] = b_start();
    B.rAlloc[2 * r] = capA;
    B.rAlloc[2 * r + 1] = capB;
    B.rStatus[r] = ((double)fabsf(a_end() - b_start()) > 0.2) ? kQMismatch : kQOk;
}

// ---- k_qfill: MutationScorer ctor / Template() -> FillAlphaBeta ------------------------------------------
// ---- k_qfill_grp: FillAlphaBeta with four reads per wavefront (grp_fill; the pass schedule of k_qfill_coop) --
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3))) k_qfill_grp(QBatch B, const int* __restrict__ reads, int n)
{
    __shared__ float qlds[4 * kQGLdsFloats];
    const int lane = threadIdx.x, g = lane >> 4, gl = lane & 15;
    const int t = blockIdx.x * 4 + g;
    if (t >= n) return;
    const int r = reads[t];
    if (r < 0) return;   // padding: the host lists each QuiverConfig's reads in whole waves
    // the read as offsets from the batch's pools (the pools' bases are kernel arguments, scalar); the wave's
    // reads share one QuiverConfig (the host's list), so its parameters are scalar loads
    const QParams* P = B.params + __builtin_amdgcn_readfirstlane(B.rParam[r]);
    const int z = B.rZmw[r];
    const int I = B.rLen[r];
    const long long so = B.rSeq[r];
    const GRead R{B.seqPool + so, B.featPool + 5 * so, I};
    const int ts = B.rTs[r], te = B.rTe[r], L = B.zLen[z];
    const char* tbase = B.tplPool + (B.rStrand[r] == 0 ? B.zFwd[z] + ts : B.zRev[z] + (L - te));
    const int J = te - ts;
    const long long cb = B.rColBase[r], vb = B.rValBase[r], valCap = B.rValCap[r];
    const int colCap = B.rColCap[r];
    auto arena_k = [&](int k) {
        QBand m;
        m.range = B.range + cb + (long long)k * colCap;
        m.off = B.off + cb + (long long)k * colCap;
        m.val = B.valPool + vb + (long long)k * valCap;
        m.cap = valCap;
        m.cols = J + 1;
        return m;
    };
    QAlloc* allocA = B.alloc + cb / 2;
    QAlloc* allocB = allocA + colCap;
    int4* hint = B.hint + cb / 4;
    if (I < 1 || J < 1 || J + 1 > colCap) {
        if (gl == 0) B.rStatus[r] = kQBad;
        return;
    }
    float* my = qlds + g * kQGLdsFloats;
    QGWin win{my, INT_MIN / 2, INT_MIN / 2};
    const QEvalG ew{P, I, J, win};
    for (int k = 0; k < 4; ++k) {
        const QBand m = arena_k(k);
        for (int j = gl; j <= J; j += kQG) m.range[j] = make_int2(0, 0);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    bool ovf = false, tall = false;
    long long needA = 0, needB = 0, stCells = 0, stCols = 0;
    int curA = 0, curB = 2;
    bool aPassed = false, bPassed = false;
    auto passA = [&](bool guided) {
        const int nxt = aPassed ? (curA ^ 1) : 0;
        const QBand gb = arena_k(curB), self = arena_k(curA), out = arena_k(nxt);
        const long long u = grp_fill<false>(ew, R, tbase, gb, guided, self, aPassed, out, allocA, aPassed, ovf, my,
                                            hint, g, gl, win);
        tall = tall || u < 0;
        if (!ovf && u >= 0) { stCells += u; stCols += J + 1; }
        needA = max(needA, u);
        curA = nxt;
        aPassed = true;
        return u;
    };
    auto passB = [&]() {
        const int nxt = bPassed ? (curB ^ 1) : 2;
        const QBand gb = arena_k(curA), self = arena_k(curB), out = arena_k(nxt);
        const long long u = grp_fill<true>(ew, R, tbase, gb, true, self, bPassed, out, allocB, bPassed, ovf, my,
                                           hint, g, gl, win);
        tall = tall || u < 0;
        if (!ovf && u >= 0) { stCells += u; stCols += J + 1; }
        needB = max(needB, u);
        curB = nxt;
        bPassed = true;
        return u;
    };
    auto a_end = [&]() { return arena_k(curA).Get(I, J); };
    auto b_start = [&]() { return arena_k(curB).Get(0, 0); };
    const int maxSize = (int)(0.5 + 0.04 * (I + 1) * (J + 1));
    long long ua = 0;
    int flips = 0, stage = 0, pending = 0;   // RecursorBase::FillAlphaBeta's schedule, as k_qfill_coop
    for (;;) {
        bool alpha = true, guided = true;
        if (stage == 0) guided = false;
        else if (stage == 1) alpha = false;
        else if (stage == 2) alpha = pending != 2;
        else {
            if (ovf || !((double)fabsf(a_end() - b_start()) > 0.2) || flips > kMaxFlipFlops) break;
            alpha = flips % 2 == 0;
        }
        const long long u = alpha ? passA(guided) : passB();
        if (tall) break;
        if (stage == 0) {
            ua = u;
            stage = 1;
        } else if (stage == 1) {
            ovf = gballot(ovf, g) != 0;
            if (!ovf && (ua >= maxSize || u >= maxSize)) {
                stage = 2;
                pending = 3;
                flips += 3;
            } else {
                stage = 3;
            }
        } else if (stage == 2) {
            if (--pending == 0) {
                ovf = gballot(ovf, g) != 0;
                stage = 3;
            }
        } else {
            flips++;
            ovf = gballot(ovf, g) != 0;
        }
    }
    long long capA = 0, capB = 0;
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    if (!tall && !ovf) {
        for (int j = gl; j <= J; j += kQG) {
            capA += allocA[j].capacity;
            capB += allocB[j].capacity;
        }
        for (int o = 8; o > 0; o >>= 1) {
            capA += __shfl_xor(capA, o, 64);
            capB += __shfl_xor(capB, o, 64);
        }
    }
    if (gl != 0) return;
    if (!tall && !ovf) qstat_add(B.stats, kQStatGrp, stCells, stCols);
    if (tall) {
        B.rStatus[r] = kQTall;
        return;
    }
    B.rUsed[2 * r] = needA;
    B.rUsed[2 * r + 1] = needB;
    if (ovf) {
        B.rStatus[r] = kQOverflow;
        return;
    }
    B.rCurA[r] = curA;
    B.rCurB[r] = curB - 2;
    B.rFlips[r] = flips;
    B.rScore[r] = b_start();
    B.rAlloc[2 * r] = capA;
    B.rAlloc[2 * r + 1] = capB;
    B.rStatus[r] = ((double)fabsf(a_end() - b_start()) > 0.2) ? kQMismatch : kQOk;
}

__global__ void __launch_bounds__(64) k_qfill(QBatch B, const int* __restrict__ reads, int n)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int r = reads[t];
    const ReadView v = read_view(B, r);
    const QEval& e = v.ev;
    const int I = e.I(), J = e.J();
    if (I < 1 || J < 1 || J + 1 > B.rColCap[r]) {
        B.rStatus[r] = kQBad;
        return;
    }
    for (int k = 0; k < 4; ++k) {
        const QBand m = arena(v, k);
        for (int j = 0; j <= J; ++j) m.range[j] = make_int2(0, 0);
    }
    bool ovf = false;
    long long needA = 0, needB = 0, stCells = 0, stCols = 0;
    int curA = 0, curB = 2;   // arena index of the latest alpha / beta pass
    bool aPassed = false, bPassed = false;
    auto passA = [&](bool guided) {
        const int nxt = aPassed ? (curA ^ 1) : 0;
        const QBand g = arena(v, curB), self = arena(v, curA), out = arena(v, nxt);
        // u: UsedEntries (RecursorBase's reband test); a dense arena holds every cell (values_needed)
        const long long u = fill_alpha(e, guided ? &g : nullptr, aPassed ? &self : nullptr, out, v.allocA, aPassed, ovf);
        if (!ovf) { stCells += u; stCols += J + 1; }
        needA = max(needA, values_needed(e, u));
        curA = nxt;
        aPassed = true;
        return u;
    };
    auto passB = [&]() {
        const int nxt = bPassed ? (curB ^ 1) : 2;
        const QBand g = arena(v, curA), self = arena(v, curB), out = arena(v, nxt);
        const long long u = fill_beta(e, &g, bPassed ? &self : nullptr, out, v.colbuf, v.allocB, bPassed, ovf);
        if (!ovf) { stCells += u; stCols += J + 1; }
        needB = max(needB, values_needed(e, u));
        curB = nxt;
        bPassed = true;
        return u;
    };
    // RecursorBase::FillAlphaBeta (detail/RecursorBase.cpp:70-116)
    const long long ua = passA(false);
    const long long ub = passB();
    int flips = 0;
    const int maxSize = (int)(0.5 + 0.04 * (I + 1) * (J + 1));   // REBANDING_THRESHOLD, double arithmetic
    if (!ovf && (ua >= maxSize || ub >= maxSize)) {
        passA(true);
        passB();
        passA(true);
        flips += 3;
    }
    auto a_end = [&]() { return arena(v, curA).Get(I, J); };
    auto b_start = [&]() { return arena(v, curB).Get(0, 0); };
    // fabs(a(I, J) - b(0, 0)) > ALPHA_BETA_MISMATCH_TOLERANCE: a float difference against the double 0.2
    while (!ovf && (double)fabsf(a_end() - b_start()) > 0.2 && flips <= kMaxFlipFlops) {
        if (flips % 2 == 0) passA(true);
        else passB();
        flips++;
    }
    B.rUsed[2 * r] = needA;
    B.rUsed[2 * r + 1] = needB;
    if (ovf) {
        B.rStatus[r] = kQOverflow;
        return;
    }
    qstat_add(B.stats, kQStatLane, stCells, stCols);
    B.rCurA[r] = curA;
    B.rCurB[r] = curB - 2;
    B.rFlips[r] = flips;
    B.rScore[r] = b_start();
    const long long full = (long long)(I + 1) * (J + 1);   // DenseMatrix::AllocatedEntries = Rows * Columns
    B.rAlloc[2 * r] = e.p->dense ? full : allocated_entries(v.allocA, J + 1);
    B.rAlloc[2 * r + 1] = e.p->dense ? full : allocated_entries(v.allocB, J + 1);
    B.rStatus[r] = ((double)fabsf(a_end() - b_start()) > 0.2) ? kQMismatch : kQOk;
}

// ---- k_qscore: MultiReadMutationScorer::Score terms (Quiver/MultiReadMutationScorer.cpp:60-120, 312-326)
__global__ void __launch_bounds__(64) k_qscore(QBatch B, QScoreWork W)
{
    const long long lt = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (lt >= W.nTasks) return;
    const long long t = W.taskList ? W.taskList[lt] : W.taskBase + lt;
    int r, code;
    if (W.nWork > 0) {   // batched round: decode (item, mutation, read) from the task number
        int lo = 0, hi = W.nWork;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (W.wTaskStart[mid] <= t) lo = mid; else hi = mid;
        }
        const long long local = t - W.wTaskStart[lo];
        const int nr = W.wNReads[lo];
        r = W.readList[W.wReadBase[lo] + (int)(local % nr)];
        code = W.codes[W.wMutBase[lo] + local / nr];
        if (!W.rActive[r]) {
            W.delta[t] = __builtin_nanf("");
            return;
        }
    } else {
        r = W.taskRead[t];
        code = W.codes[W.taskMut[t]];
    }
    const int type = (code >> 2) & 3, pos = code >> 4, base = code & 3;
    const int ms = pos, me = (type == 0) ? pos : pos + 1;
    const int ts = B.rTs[r], te = B.rTe[r];
    const bool scores = W.raw || ((type == 0) ? (ts < ms && me <= te) : (ts < me && ms < te));   // ReadScoresMutation
    if (!scores) {
        W.delta[t] = __builtin_nanf("");
        return;
    }
    ReadView v = read_view(B, r);
    QEval& e = v.ev;
    const char* kB = "ACGT";
    // OrientedMutation (:79-120), single-base mutations
    int os, oe;
    char ob;
    if (W.raw) { os = ms; oe = me; ob = kB[base]; }
    else if (B.rStrand[r] == 0) { os = ms - ts; oe = me - ts; ob = kB[base]; }
    else { os = te - me; oe = te - ms; ob = kB[3 - base]; }
    const QBand a = arena(v, B.rCurA[r]);
    const QBand b = arena(v, 2 + B.rCurB[r]);
    const int J = e.J();   // unmutated window length
    const int lengthDiff = (type == 0) ? 1 : (type == 1) ? -1 : 0;
    // MutationScorer::ScoreMutation (Quiver/MutationScorer.cpp:113-226)
    const int betaLinkCol = 1 + oe;
    const int absLinkCol = 1 + oe + lengthDiff;
    const bool atBegin = os < 3;
    const bool atEnd = oe > J - 2;
    e.t.editPos = os;
    e.t.editType = type;
    e.t.editBase = ob;
    e.t.len = J + lengthDiff;
    const int newLen = e.t.len;
    // extend buffer: at most 8 columns (EXTEND_BUFFER_COLUMNS), values bump-allocated from the pool; the
    // per-column ranges and offsets sit in LDS (a per-lane local array would be scratch)
    __shared__ int2 sxr[64][8];
    __shared__ int sxo[64][8];
    int2* xr = sxr[threadIdx.x];
    int* xo = sxo[threadIdx.x];
    QBand ext;
    ext.range = xr;
    ext.off = xo;
    ext.cols = 8;
    const int I = e.I();
    auto alloc = [&](long long n) -> bool {
        const unsigned long long at = atomicAdd(W.scratchTop, (unsigned long long)n);
        if (at + n > W.scratchCap) {
            atomicOr(W.overflow, 1);
            return false;
        }
        ext.val = W.scratch + at;
        ext.cap = n;
        return true;
    };
    bool ovf = false;
    float score;
    if (!atBegin && !atEnd) {
        const int extStart = (type == 1) ? os - 1 : os;
        const int extLen = 2;
        long long need = 0;
        for (int c = 0; c < extLen; ++c) {
            const int j = extStart + c;
            need += (j < a.cols) ? (a.range[j].y - a.range[j].x) : (I + 1 - a.range[a.cols - 1].x);
        }
        if (!alloc(max(need, 1LL))) { W.delta[t] = __builtin_nanf(""); return; }
        if (e.p->simple) extend_alpha_simple(e, a, extStart, ext, extLen, ovf);
        else extend_alpha(e, a, extStart, ext, extLen, ovf);
        score = link_alpha_beta(e, ext, extLen, b, betaLinkCol, absLinkCol);
    } else if (!atBegin && atEnd) {
        const int extStart = os - 1;
        const int extLen = newLen - extStart + 1;
        if (extLen > 8) { atomicOr(W.overflow, 2); W.delta[t] = __builtin_nanf(""); return; }
        if (!alloc((long long)extLen * (I + 1))) { W.delta[t] = __builtin_nanf(""); return; }
        if (e.p->simple) extend_alpha_simple(e, a, extStart, ext, extLen, ovf);
        else extend_alpha(e, a, extStart, ext, extLen, ovf);
        score = ext.Get(I, extLen - 1);
    } else if (atBegin && !atEnd) {
        const int extLast = oe;
        const int extLen = oe + lengthDiff + 1;
        if (extLen > 8) { atomicOr(W.overflow, 2); W.delta[t] = __builtin_nanf(""); return; }
        if (!alloc((long long)extLen * (I + 1))) { W.delta[t] = __builtin_nanf(""); return; }
        extend_beta(e, b, extLast, ext, extLen, lengthDiff, ovf);
        score = ext.Get(0, 0);
    } else {
        // whole fill of the mutated window (tiny windows only)
        if (newLen + 1 > 8) { atomicOr(W.overflow, 2); W.delta[t] = __builtin_nanf(""); return; }
        if (!alloc((long long)(newLen + 1) * (I + 1))) { W.delta[t] = __builtin_nanf(""); return; }
        ext.cols = newLen + 1;
        for (int j = 0; j < ext.cols; ++j) xr[j] = make_int2(0, 0);
        fill_alpha(e, nullptr, nullptr, ext, nullptr, false, ovf);
        score = ext.Get(I, newLen);
    }
    if (ovf) atomicOr(W.overflow, 1);
    W.delta[t] = W.raw ? score : score - B.rScore[r];
}

// ---- k_qreduce: Score / FastIsFavorable of a batched round, one lane per mutation ----------------------
__global__ void __launch_bounds__(256) k_qreduce(QReduceWork W)
{
    const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= W.nMut) return;
    int lo = 0, hi = W.nWork;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (W.wMutStart[mid] <= g) lo = mid; else hi = mid;
    }
    const int nr = W.wNReads[lo];
    const float* d = W.delta + W.wTaskStart[lo] + (g - W.wMutStart[lo]) * nr;
    const float thr = W.wFastThreshold[lo];
    float sum = 0.0f;
    bool fast = true;
    for (int k = 0; k < nr; ++k) {
        const float x = d[k];
        if (x != x) continue;
        sum += x;
        if (sum < thr) fast = false;   // FastIsFavorable returns here; Score keeps summing
    }
    W.score[g] = (double)sum;
    W.fav[g] = (fast && (double)sum > 0.04) ? 1 : 0;   // MIN_FAVORABLE_SCOREDIFF (:52), a double
}

// ---- k_qscore_mid: ScoreMutation's middle case, one wavefront per (item, read, 64-mutation chunk) ----------
// MutationScorer::ScoreMutation (Quiver/MutationScorer.cpp:150-175) away from the window ends is ExtendAlpha
// over two columns (SseRecursor.cpp:433-551 / SimpleRecursor.cpp:303-388) and LinkAlphaBeta of those with
// beta (SseRecursor.cpp:355-431 / SimpleRecursor.cpp:232-295).  Here the three are one top-down walk over the
// link's rows: row i of extension column 0, then of column 1, then row i's link terms.  A row only needs its
// predecessor's values, so the extension columns never leave registers (k_qscore writes them to a bump
// scratch and reads them back).  Every term keeps the reference's order: an extension column's scalar head
// rows combine Inc, Extra, Merge, Del; its 4-row SSE blocks combine Inc, Merge, Del from -FLT_MAX and then the
// Extra cascade; the link's block rows accumulate into 4 SSE lanes, its tail rows into one, and the lanes are
// folded in lane order at the end.  The read's QV-feature rows under the wave's lanes are staged in LDS.
namespace {

struct QMidStage {   // one wave's QV-feature rows [lo, lo + kQMidStageRows)
    float ins[kQMidStageRows], subs[kQMidStageRows], del[kQMidStageRows], tag[kQMidStageRows],
        merge[kQMidStageRows];
    char seq[kQMidStageRows];
};

struct QCol {   // one band column: value at row i is p[i] for i in [x, y), else -FLT_MAX
    const float* p;
    int x, y;
    __device__ __forceinline__ float at(int i) const { return (i >= x && i < y) ? p[i] : kNegInf; }
};

__device__ __forceinline__ QCol qcol(const QBand& m, int j)
{
    QCol c;
    const int2 r = m.range[j];
    c.x = r.x;
    c.y = r.y;
    c.p = m.val + m.off[j] - r.x;
    return c;
}

// QvEvaluator terms (QvEvaluator.hpp:150-207) from a row's features and a template base
struct QMerge {   // Merge(i, j) for the template pair (t(j), t(j + 1)): only reads of a homopolymer base merge
    int base;     // t(j) when t(j) == t(j + 1), else -1 (never matches a read base)
    float c, s;
};
__device__ __forceinline__ QMerge qmerge(const QParams& P, char a, char b)
{
    QMerge m;
    const int k = tpl_code(a);
    m.base = (a == b) ? (int)a : -1;
    m.c = P.Merge[k];
    m.s = P.MergeS[k];
    return m;
}

template <bool SIMPLE, class FEAT>
__device__ __forceinline__ float qmid_walk(const QParams& P, bool sp, bool merge, int I, const FEAT& F, int j0,
                                           const QCol& A1, const QCol& A2, const QCol& B0, const QCol& B1, int b0,
                                           int e0, int b1, int e1, int lb, int le, char t0m1, char t0, char t0p1,
                                           const QMerge& m0, const QMerge& m1, char l1, const QMerge& ml0,
                                           const QMerge& ml1)
{
    auto inc = [&](int s, float subs, char tb) { return (s == tb) ? P.Match : P.Mismatch + P.MismatchS * subs; };
    auto del = [&](int i, float tag, float d, char tb) {
        return (i < I && (float)tb == tag) ? P.DeletionWithTag + P.DeletionWithTagS * d : P.DeletionN;
    };
    auto extra = [&](int s, float ins, char tb) { return (s == tb) ? P.Branch + P.BranchS * ins : P.Nce + P.NceS * ins; };
    auto mrg = [&](int s, float mq, const QMerge& m) { return (s == m.base) ? m.c + m.s * mq : kNegInf; };

    // first SSE-block row of each extension column (the head loop of SseRecursor::ExtendAlpha)
    int p0 = b0, p1 = b1;
    if (!SIMPLE) {
        while (p0 < e0 && (p0 == 0 || (e0 - p0) % 4 != 0)) ++p0;
        while (p1 < e1 && (p1 == 0 || (e1 - p1) % 4 != 0)) ++p1;
    }
    const int blockEnd = SIMPLE ? lb : lb + 4 * max(0, (le - 4 - lb + 3) / 4);   // link rows in 4-row blocks

    // row i - 1 state
    float e0p = kNegInf, e1p = kNegInf;
    float a1p = (lb >= 1) ? A1.at(lb - 1) : kNegInf;
    float a2p = (lb >= 1) ? A2.at(lb - 1) : kNegInf;
    int sP = 0;
    float insP = 0.f, subsP = 0.f, mergeP = 0.f;
    if (lb >= 1) {
        sP = F.seq(lb - 1);
        insP = F.ins(lb - 1);
        subsP = F.subs(lb - 1);
        mergeP = F.merge(lb - 1);
    }
    float bCur = B0.at(lb);
    float v4a = kNegInf, v4b = kNegInf, v4c = kNegInf, v4d = kNegInf, v = kNegInf;
    for (int i = lb; i < le; ++i) {
        int s = 0;
        float ins = 0.f, subs = 0.f, d = 0.f, tag = 0.f, mq = 0.f;
        if (i < I) {
            s = F.seq(i);
            ins = F.ins(i);
            subs = F.subs(i);
            d = F.del(i);
            tag = F.tag(i);
            mq = F.merge(i);
        }
        const float a1c = A1.at(i);
        // extension column 0 (template column j0)
        float e0c = kNegInf;
        if (i >= b0 && i < e0) {
            float x = kNegInf;
            if (SIMPLE) {
                if (i > 0) x = comb(sp, x, a1p + inc(sP, subsP, t0m1));
                if (i > 0) x = comb(sp, x, e0p + extra(sP, insP, t0));
                x = comb(sp, x, a1c + del(i, tag, d, t0m1));
                if (merge && i > 0) x = comb(sp, x, a2p + mrg(sP, mergeP, m0));
            } else if (i < p0) {
                if (i > 0) {
                    x = comb(sp, x, a1p + inc(sP, subsP, t0m1));
                    x = comb(sp, x, e0p + extra(sP, insP, t0));
                    if (merge) x = comb(sp, x, a2p + mrg(sP, mergeP, m0));
                }
                x = comb(sp, x, a1c + del(i, tag, d, t0m1));
            } else {
                x = comb4(sp, x, a1p + inc(sP, subsP, t0m1));
                if (merge && j0 >= 2) x = comb4(sp, x, a2p + mrg(sP, mergeP, m0));
                x = comb4(sp, x, a1c + del(i, tag, d, t0m1));
                x = comb(sp, x, e0p + extra(sP, insP, t0));
            }
            e0c = x;
        }
        // extension column 1 (template column j0 + 1): its merge term reads alpha column j0 - 1, as the
        // reference's ExtendAlpha does for every extension column
        float e1c = kNegInf;
        if (i >= b1 && i < e1) {
            float x = kNegInf;
            if (SIMPLE) {
                if (i > 0) x = comb(sp, x, e0p + inc(sP, subsP, t0));
                if (i > 0) x = comb(sp, x, e1p + extra(sP, insP, t0p1));
                x = comb(sp, x, e0c + del(i, tag, d, t0));
                if (merge && i > 0) x = comb(sp, x, a1p + mrg(sP, mergeP, m1));
            } else if (i < p1) {
                if (i > 0) {
                    x = comb(sp, x, e0p + inc(sP, subsP, t0));
                    x = comb(sp, x, e1p + extra(sP, insP, t0p1));
                    if (merge) x = comb(sp, x, a1p + mrg(sP, mergeP, m1));
                }
                x = comb(sp, x, e0c + del(i, tag, d, t0));
            } else {
                x = comb4(sp, x, e0p + inc(sP, subsP, t0));
                if (merge) x = comb4(sp, x, a1p + mrg(sP, mergeP, m1));
                x = comb4(sp, x, e0c + del(i, tag, d, t0));
                x = comb(sp, x, e1p + extra(sP, insP, t0p1));
            }
            e1c = x;
        }
        // LinkAlphaBeta row i: extension columns (ac - 2, ac - 1) = (0, 1) against beta (bc, bc + 1)
        const float bN0 = B0.at(i + 1), bN1 = B1.at(i + 1);
        if (SIMPLE) {
            if (i < I) {
                v = comb(sp, v, e1c + inc(s, subs, l1) + bN0);
                v = comb(sp, v, e0c + mrg(s, mq, ml0) + bN0);
                v = comb(sp, v, e1c + mrg(s, mq, ml1) + bN1);
            }
            v = comb(sp, v, e1c + del(i, tag, d, l1) + bCur);
        } else if (i < blockEnd) {
            float x = v4a;
            x = comb4(sp, x, e1c + inc(s, subs, l1) + bN0);
            if (merge) {
                x = comb4(sp, x, e0c + mrg(s, mq, ml0) + bN0);
                x = comb4(sp, x, e1c + mrg(s, mq, ml1) + bN1);
            }
            x = comb4(sp, x, e1c + del(i, tag, d, l1) + bCur);
            v4a = v4b;   // rotate: the next row accumulates into the next SSE lane
            v4b = v4c;
            v4c = v4d;
            v4d = x;
        } else {
            if (i < I) {
                v = comb(sp, v, e1c + inc(s, subs, l1) + bN0);
                if (merge) {
                    v = comb(sp, v, e0c + mrg(s, mq, ml0) + bN0);
                    v = comb(sp, v, e1c + mrg(s, mq, ml1) + bN1);
                }
            }
            v = comb(sp, v, e1c + del(i, tag, d, l1) + bCur);
        }
        e0p = e0c;
        e1p = e1c;
        a2p = A2.at(i);
        a1p = a1c;
        sP = s;
        insP = ins;
        subsP = subs;
        mergeP = mq;
        bCur = bN0;
    }
    if (SIMPLE) return v;
    float acc = kNegInf;   // std::accumulate over the 4 SSE lanes, then the tail
    acc = comb(sp, acc, v4a);
    acc = comb(sp, acc, v4b);
    acc = comb(sp, acc, v4c);
    acc = comb(sp, acc, v4d);
    return comb(sp, acc, v);
}

struct QFeatLds {
    const QMidStage* st;
    int lo;
    __device__ __forceinline__ int seq(int i) const { return st->seq[i - lo]; }
    __device__ __forceinline__ float ins(int i) const { return st->ins[i - lo]; }
    __device__ __forceinline__ float subs(int i) const { return st->subs[i - lo]; }
    __device__ __forceinline__ float del(int i) const { return st->del[i - lo]; }
    __device__ __forceinline__ float tag(int i) const { return st->tag[i - lo]; }
    __device__ __forceinline__ float merge(int i) const { return st->merge[i - lo]; }
};

struct QFeatHbm {
    QRead r;
    __device__ __forceinline__ int seq(int i) const { return r.seq[i]; }
    __device__ __forceinline__ float ins(int i) const { return r.ins[i]; }
    __device__ __forceinline__ float subs(int i) const { return r.subs[i]; }
    __device__ __forceinline__ float del(int i) const { return r.del[i]; }
    __device__ __forceinline__ float tag(int i) const { return r.tag[i]; }
    __device__ __forceinline__ float merge(int i) const { return r.merge[i]; }
};

}  // namespace

__global__ void __launch_bounds__(64 * kQMidWaves) k_qscore_mid(QBatch B, QMidWork W)
{
    __shared__ QMidStage stage[kQMidWaves];
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: scalar item search
    const int lane = threadIdx.x & 63;
    const long long wave = (long long)blockIdx.x * kQMidWaves + wid;
    const bool waveLive = wave < W.waveStart[W.nWork];
    int w = 0;
    if (waveLive) {   // binary search of the work item (wave-uniform)
        int lo = 0, hi = W.nWork;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (W.waveStart[mid] <= wave) lo = mid; else hi = mid;
        }
        w = lo;
    }
    w = __builtin_amdgcn_readfirstlane(w);
    const int nr = waveLive ? W.wNReads[w] : 1;
    const long long M = waveLive ? W.wMutCount[w] : 0;
    const int chunks = (int)max(1LL, (M + 63) >> 6);
    const long long local = waveLive ? wave - W.waveStart[w] : 0;
    const int rd = (int)(local / chunks);
    const long long m = (local % chunks) * 64 + lane;
    const bool valid = waveLive && m < M;
    const int r = __builtin_amdgcn_readfirstlane(waveLive ? W.readList[W.wReadBase[w] + rd] : 0);
    const long long t = valid ? W.wTaskStart[w] + m * nr + rd : 0;

    // classify the lane: not scored (NaN), middle case (here), edge case (k_qscore's listed form)
    bool middle = false;
    int os = 0, oe = 0, type = 0, ld = 0;
    char ob = 'A';
    const int ts = B.rTs[r], te = B.rTe[r];
    const int J = te - ts;
    if (valid) {
        const int code = W.codes[W.wMutBase[w] + m];
        type = (code >> 2) & 3;
        const int pos = code >> 4, base = code & 3;
        const int ms = pos, me = (type == 0) ? pos : pos + 1;
        const bool scores = W.rActive[r] && ((type == 0) ? (ts < ms && me <= te) : (ts < me && ms < te));
        if (!scores) {
            W.delta[t] = __builtin_nanf("");
        } else {
            const char* kB = "ACGT";
            if (B.rStrand[r] == 0) { os = ms - ts; oe = me - ts; ob = kB[base]; }
            else { os = te - me; oe = te - ms; ob = kB[3 - base]; }
            ld = (type == 0) ? 1 : (type == 1) ? -1 : 0;
            middle = !(os < 3) && !(oe > J - 2);
            if (!middle) {
                const unsigned long long slot = atomicAdd(W.edgeCount, 1ULL);
                if ((long long)slot < W.edgeCap) W.edgeList[slot] = t;
            }
        }
    }
    ReadView v = read_view(B, r);
    const QParams& P = *v.ev.p;
    const int I = v.ev.I();
    const QBand a = arena(v, B.rCurA[r]);
    const QBand b = arena(v, 2 + B.rCurB[r]);
    const int j0 = (type == 1) ? os - 1 : os;   // ExtendAlpha's first column
    const int bc = 1 + oe;                       // beta link column
    int b0 = 0, e0 = 0, b1 = 0, e1 = 0, lb = 0, le = 0;
    QCol A1{}, A2{}, B0{}, B1{};
    if (middle) {
        A1 = qcol(a, j0 - 1);
        A2 = qcol(a, j0 - 2);
        B0 = qcol(b, bc);
        B1 = qcol(b, bc + 1);
        const int2 r0 = a.range[j0], r1 = a.range[j0 + 1];
        b0 = r0.x; e0 = r0.y; b1 = r1.x; e1 = r1.y;
        lb = min(min(b0, b1), min(B0.x, B1.x));
        le = max(max(e0, e1), max(B0.y, B1.y));
    }
    // the wave's feature rows [lb - 1, le) of its middle lanes, staged in LDS when they fit
    int rLo = middle ? max(0, lb - 1) : INT_MAX, rHi = middle ? min(le, I) : -1;
    for (int o = 32; o > 0; o >>= 1) {
        rLo = min(rLo, __shfl_xor(rLo, o, 64));
        rHi = max(rHi, __shfl_xor(rHi, o, 64));
    }
    const bool staged = rHi >= rLo && rHi - rLo <= kQMidStageRows;
    QMidStage& st = stage[wid];
    if (staged) {
        const QRead& R = v.ev.r;
        for (int q = lane; q < rHi - rLo; q += 64) {
            const int i = rLo + q;
            st.seq[q] = R.seq[i];
            st.ins[q] = R.ins[i];
            st.subs[q] = R.subs[i];
            st.del[q] = R.del[i];
            st.tag[q] = R.tag[i];
            st.merge[q] = R.merge[i];
        }
    }
    __syncthreads();   // every wave of the block reaches this point exactly once
    if (!middle) return;

    // template bases of the mutated window (OrientedMutation applied virtually, as k_qscore's QTpl)
    QTpl T = v.ev.t;
    T.editPos = os;
    T.editType = type;
    T.editBase = ob;
    T.len = J + ld;
    const int absc = 1 + oe + ld;   // absolute link column
    const char t0m2 = T.at(j0 - 2), t0m1 = T.at(j0 - 1), t0 = T.at(j0), t0p1 = T.at(j0 + 1);
    const char la = T.at(absc - 2), l1 = T.at(absc - 1), lc = T.at(absc);
    const QMerge m0 = qmerge(P, t0m2, t0m1), m1 = qmerge(P, t0m1, t0);
    const QMerge ml0 = qmerge(P, la, l1), ml1 = qmerge(P, l1, lc);
    const bool sp = P.sumProduct != 0, mv = (P.moves & kMerge) != 0;
    float score;
    if (staged) {
        const QFeatLds F{&st, rLo};
        score = P.simple ? qmid_walk<true>(P, sp, mv, I, F, j0, A1, A2, B0, B1, b0, e0, b1, e1, lb, le, t0m1, t0, t0p1,
                                           m0, m1, l1, ml0, ml1)
                         : qmid_walk<false>(P, sp, mv, I, F, j0, A1, A2, B0, B1, b0, e0, b1, e1, lb, le, t0m1, t0,
                                            t0p1, m0, m1, l1, ml0, ml1);
    } else {
        const QFeatHbm F{v.ev.r};
        score = P.simple ? qmid_walk<true>(P, sp, mv, I, F, j0, A1, A2, B0, B1, b0, e0, b1, e1, lb, le, t0m1, t0, t0p1,
                                           m0, m1, l1, ml0, ml1)
                         : qmid_walk<false>(P, sp, mv, I, F, j0, A1, A2, B0, B1, b0, e0, b1, e1, lb, le, t0m1, t0,
                                            t0p1, m0, m1, l1, ml0, ml1);
    }
    W.delta[t] = score - B.rScore[r];
}

// ---- k_qqv: ConsensusQVs of a batched round (Consensus-inl.hpp:274-295) ------------------------------------
__global__ void __launch_bounds__(256) k_qqv(QQvWork W, long long nPos)
{
    const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nPos) return;
    int lo = 0, hi = W.nWork;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (W.posStart[mid] <= g) lo = mid; else hi = mid;
    }
    const int p = (int)(g - W.posStart[lo]);
    const int* po = W.posOff + W.posOffBase[lo];
    const double* sc = W.score + W.wMutStart[lo];
    double sum = 0.0;
    for (int m = po[p]; m < po[p + 1]; ++m) {
        const double s = (double)(float)sc[m];   // Score() is a float sum
        if (s < 0.0) sum += exp(s);
    }
    // The scores are the reference's floats bit for bit, but exp / log10 here are OCML's, the reference's
    // glibc's: they may differ by an ulp.  That moves prob by at most err (a few ulps of 1 from the roundings of
    // 1 + sum and its reciprocal, and of sum from its terms), so -10 log10(prob) by at most 4.343 err / prob: a
    // position whose value lies that close to a .5 rounding boundary, or whose 1 + sum sits near the edge of
    // 1.0, is marked -1 and the host recomputes it with the host libm from the same float scores
    // (QuiverBatch::QVsMany), so every QV is the reference's.
    constexpr double eps = 2.220446049250313e-16;
    double prob = 1.0 - 1.0 / (1.0 + sum);
    bool amb = W.hostAll != 0;
    double rel = 0.0;
    if (prob == 0.0) {
        amb = amb || sum > 0.4 * eps;   // 1 + sum rounded to 1.0 here; near 2^-53 the host's sum may not
        prob = 2.2250738585072014e-308;   // std::numeric_limits<double>::min()
    } else {
        rel = (4.0 * eps + 16.0 * eps * sum) / prob;   // (sum: up to ~9 terms, an ulp each and per partial sum)
    }
    const double v = -10.0 * log10(prob);
    const double frac = v - floor(v);
    amb = amb || fabs(frac - 0.5) < 4.35 * rel + 1e-6;
    W.qv[g] = amb ? -1 : (int)round(v);
}

// ---- k_qgather: the mutation scores of the positions k_qqv left to the host, packed for one download ---------
__global__ void __launch_bounds__(256) k_qgather(const double* __restrict__ score, const long long* __restrict__ src,
                                                 const long long* __restrict__ dst, int n, double* __restrict__ out)
{
    const int a = blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= n) return;
    const long long s = src[a], d0 = dst[a], d1 = dst[a + 1];
    for (long long m = d0; m < d1; ++m) out[m] = score[s + (m - d0)];
}

// ---- k_qalign: RecursorBase::Alignment (detail/RecursorBase.cpp:118-264) -------------------------------
// The Viterbi path through a read's final alpha band, one lane per read, walking back from (I, J): moves
// tried in the order Incorporate, Delete, Extra, Merge, strict '>' against -FLT_MAX, the move score added
// to the predecessor cell in float.  The scorer's evaluator pins both ends, so no delete is free.  Writes
// the moves from the end (1 INCORPORATE, 4 DELETE, 2 EXTRA, 8 MERGE); nMoves < 0 when no move is valid
// (the reference asserts).
__global__ void __launch_bounds__(64) k_qalign(QBatch B, const int* __restrict__ reads, int n,
                                               const long long* __restrict__ moveOff, unsigned char* __restrict__ moves,
                                               int* __restrict__ nMoves)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int r = reads[t];
    const ReadView v = read_view(B, r);
    const QEval& e = v.ev;
    const QBand a = arena(v, B.rCurA[r]);
    const bool merge = (e.p->moves & kMerge) != 0;
    unsigned char* out = moves + moveOff[t];
    int i = e.I(), j = e.J(), k = 0;
    while (i > 0 || j > 0) {
        int best = 0;
        float bestScore = kNegInf;
        if (i > 0 && j > 0) {
            const float s = a.Get(i - 1, j - 1) + e.Inc(i - 1, j - 1);
            if (s > bestScore) { best = 1; bestScore = s; }
        }
        if (j > 0) {
            const float s = a.Get(i, j - 1) + e.Del(i, j - 1);
            if (s > bestScore) { best = 4; bestScore = s; }
        }
        if (i > 0) {
            const float s = a.Get(i - 1, j) + e.Extra(i - 1, j);
            if (s > bestScore) { best = 2; bestScore = s; }
        }
        if (merge && i > 0 && j > 1) {
            const float s = a.Get(i - 1, j - 2) + e.Merge(i - 1, j - 2);
            if (s > bestScore) { best = 8; bestScore = s; }
        }
        if (best == 0) { k = -1; break; }
        out[k++] = (unsigned char)best;
        i -= (best == 4) ? 0 : 1;
        j -= (best == 2) ? 0 : (best == 8 ? 2 : 1);
    }
    nMoves[t] = k;
}

// ---- k_qv_moves: QvEvaluator's move scores (Quiver/QvEvaluator.hpp:153-207) at listed cells ----------------
// One lane per (i, j): Inc, Del (with QvEvaluator's pinStart / pinEnd rule, :169-184), Extra and Merge, each NaN
// where the cell is outside the move's domain (the reference's asserts).  out: 4 x n floats (move-major).
__global__ void __launch_bounds__(256) k_qv_moves(QEval e, int pinStart, int pinEnd, const int* __restrict__ ci,
                                                  const int* __restrict__ cj, int n, float* __restrict__ out)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int i = ci[t], j = cj[t], I = e.I(), J = e.J();
    const float nan = __builtin_nanf("");
    float inc = nan, del = nan, extra = nan, merge = nan;
    if (i >= 0 && i < I && j >= 0 && j < J) inc = e.Inc(i, j);
    if (i >= 0 && i <= I && j >= 0 && j < J) del = ((!pinStart && i == 0) || (!pinEnd && i == I)) ? 0.0f : e.Del(i, j);
    if (i >= 0 && i < I && j >= 0 && j <= J) extra = e.Extra(i, j);
    if (i >= 0 && i < I && j >= 0 && j < J - 1) merge = e.Merge(i, j);
    out[t] = inc;
    out[n + t] = del;
    out[2 * n + t] = extra;
    out[3 * n + t] = merge;
}

void launch_qv_moves(const QRead& r, const QParams* p, const char* tpl, int tplLen, int pinStart, int pinEnd,
                     const int* ci, const int* cj, int n, float* out, hipStream_t s)
{
    if (n <= 0) return;
    QEval e;
    e.r = r;
    e.p = p;
    e.t = QTpl{tpl, tplLen};
    hipLaunchKernelGGL(k_qv_moves, dim3((n + 255) / 256), dim3(256), 0, s, e, pinStart, pinEnd, ci, cj, n, out);
}

void launch_qalign(const QBatch& B, const int* reads, int n, const long long* moveOff, unsigned char* moves,
                   int* nMoves, hipStream_t s)
{
    if (n <= 0) return;
    hipLaunchKernelGGL(k_qalign, dim3((n + 63) / 64), dim3(64), 0, s, B, reads, n, moveOff, moves, nMoves);
}

void launch_qfill(const QBatch& B, const int* reads, int n, hipStream_t s)
{
    if (n <= 0) return;
    hipLaunchKernelGGL(k_qfill, dim3((n + 63) / 64), dim3(64), 0, s, B, reads, n);
}

void launch_qfill_coop(const QBatch& B, const int* reads, int n, int maxRows, int maxCols, hipStream_t s)
{
    if (n <= 0) return;
    // the LDS ring: a power of two of rows (a band-height ring, rows modulo its size) or, for reads that fit,
    // their full height
    const int rows = (maxRows & (maxRows - 1)) == 0 ? maxRows : (maxRows + 63) / 64 * 64;
    const int cols = (maxCols + 15) / 16 * 16;
    const size_t lds = (size_t)(3 * rows + 5 * kQWinRows) * sizeof(float) + kQWinRows + cols;
    hipLaunchKernelGGL(k_qfill_coop, dim3(n), dim3(64), lds, s, B, reads, n, rows, cols);
}

void launch_qfill_grp(const QBatch& B, const int* reads, int n, hipStream_t s)
{
    if (n <= 0) return;
    hipLaunchKernelGGL(k_qfill_grp, dim3((n + 3) / 4), dim3(64), 0, s, B, reads, n);
}

void launch_qscore(const QBatch& B, const QScoreWork& W, hipStream_t s)
{
    if (W.nTasks <= 0) return;
    hipLaunchKernelGGL(k_qscore, dim3((unsigned)((W.nTasks + 63) / 64)), dim3(64), 0, s, B, W);
}

void launch_qscore_mid(const QBatch& B, const QMidWork& W, long long nWaves, hipStream_t s)
{
    if (nWaves <= 0) return;
    hipLaunchKernelGGL(k_qscore_mid, dim3((unsigned)((nWaves + kQMidWaves - 1) / kQMidWaves)), dim3(64 * kQMidWaves),
                       0, s, B, W);
}

void launch_qqv(const QQvWork& W, long long nPos, hipStream_t s)
{
    if (nPos <= 0) return;
    hipLaunchKernelGGL(k_qqv, dim3((unsigned)((nPos + 255) / 256)), dim3(256), 0, s, W, nPos);
}

void launch_qgather(const double* score, const long long* src, const long long* dst, int n, double* out, hipStream_t s)
{
    if (n <= 0) return;
    hipLaunchKernelGGL(k_qgather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, score, src, dst, n, out);
}

void launch_qreduce(const QReduceWork& W, hipStream_t s)
{
    if (W.nMut <= 0) return;
    hipLaunchKernelGGL(k_qreduce, dim3((unsigned)((W.nMut + 255) / 256)), dim3(256), 0, s, W);
}

}  // namespace quiver
}  // namespace pbccs
