// =============================================================================
//  oracle/arrow_oracle.cpp  --  TEST INFRASTRUCTURE ONLY
// -----------------------------------------------------------------------------
//  A CPU restatement of the ConsensusCore *Arrow* polishing path that pbccs'
//  `ccs` runs (reference: /root/reference, bnbowman/pbccs).  It exists so that
//  tests/ , __graft_entry__.smoke() and bench.py's `cpu_baseline` leg have an
//  independent checker for the HIP engine in pbccs_amd/.  Nothing in the
//  product (pbccs_amd/, include/) links, loads or calls this file.
//
//  Parity pin: the reference cannot be built here (it needs Boost, which is
//  absent; writing header stand-ins is not allowed), so this restatement is
//  pinned by the reference's own known-answer values
//  (ConsensusCore/src/Demos/MatrixTester.cpp:74-204, 1e-5 relative), the
//  mutation/enumerator gtest expectations (src/Tests/TestMutations.cpp,
//  TestMutationEnumerator.cpp) and the reference polish outputs recorded for
//  the tests/data ZMW 6251 FASTA in SURVEY.md §0 item 4.  See
//  tests/golden/make_golden.py and tests/test_oracle_pins.py.
//
//  Each routine cites the reference file:line it follows ("CC/" =
//  ConsensusCore/).  Written as a plain, scalar, straightforward C++17
//  restatement (same operation order, no FMA contraction: build with
//  -ffp-contract=off), deliberately NOT sharing code with the HIP engine.
// =============================================================================
#include <array>
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <map>
#include <numeric>
#include <set>
#include <stdexcept>
#include <string>
#include <unordered_set>
#include <utility>
#include <vector>

#include "oracle_common.hpp"

namespace orc {

// ---------------------------------------------------------------- constants
static const double kMismatch = 0.00505052456472967;   // CC/include/ConsensusCore/Arrow/ArrowConfig.hpp:54
static const int kExtendColumns = 8;                   // CC/src/C++/Arrow/MutationScorer.cpp:48
static const int kMaxFlipFlops = 5;                    // CC/src/C++/Arrow/SimpleRecursor.cpp:52
static const double kAlphaBetaTol = 0.001;             // SimpleRecursor.cpp:53
static const double kRebandFrac = 0.04;                // SimpleRecursor.cpp:54
static const double kMinFavorable = 0.04;              // CC/src/C++/Arrow/MultiReadMutationScorer.cpp:56

enum { R_SUCCESS = 0, R_ABMISMATCH = 1, R_MEMFAIL = 2, R_POORZ = 3, R_OTHER = 4 };  // Arrow/MultiReadMutationScorer.hpp:60

struct AlphaBetaMismatch {};

// ------------------------------------------------------------ SNR -> params
// Dinucleotide-context transition model, CC/src/C++/Arrow/ContextParameterProvider.cpp:20-110.
// Row order per context: dark(deletion), match, stick; columns: 1, snr, snr^2, snr^3.
struct Trans { double match = 0.0, stick = 0.0, branch = 0.0, del = 0.0; };

static const char* kCtxKey[8] = {"AA", "CC", "GG", "TT", "NA", "NC", "NG", "NT"};
static const double kCtxPoly[8][3][4] = {
    {{3.76122480667588, -0.536010820176981, 0.0275375059387171, -0.000470200724345621},
     {3.57517725358548, -0.0257545295375707, -0.000163673803286944, 5.3256984681724e-06},
     {0.858421613302247, -0.0276654216841666, -8.85549766507732e-05, -4.85355908595337e-05}},
    {{5.66725538674764, -1.10462196933913, 0.0879811093908922, -0.00259393800835979},
     {4.11682756767018, -0.124758322644639, 0.00659795177909886, -0.000361914629195461},
     {3.17103818507405, -0.729020290806687, 0.0749784690396837, -0.00262779517495421}},
    {{3.81920778703052, -0.540309003502589, 0.0389569264893982, -0.000901245733796236},
     {3.31322216145728, 0.123514009118836, -0.00807401406655071, 0.000230843924466035},
     {2.06006877520527, -0.451486652688621, 0.0375212898173045, -0.000937676250926241}},
    {{5.39308368236762, -1.32931568057267, 0.107844580241936, -0.00316462903462847},
     {4.21031404956015, -0.347546363361823, 0.0293839179303896, -0.000893802212450644},
     {2.33143889851302, -0.586068444099136, 0.040044954697795, -0.000957298861394191}},
    {{2.35936060895653, -0.463630601682986, 0.0179206897766131, -0.000230839937063052},
     {3.22847830625841, -0.0886820214931539, 0.00555981712798726, -0.000137686231186054},
     {-0.101031042923432, -0.0138783767832632, -0.00153408019582419, 7.66780338484727e-06}},
    {{5.956054206161, -1.71886470811695, 0.153315470604752, -0.00474488595513198},
     {3.89418464416296, -0.174182841558867, 0.0171719290275442, -0.000653629721359769},
     {2.40532887070852, -0.652606650098156, 0.0688783864119339, -0.00246479494650594}},
    {{3.53508304630569, -0.788027301381263, 0.0469367803413207, -0.00106221924705805},
     {2.85440184222226, 0.166346531056167, -0.0166161828155307, 0.000439492705370092},
     {0.238188180807376, 0.0589443522886522, -0.0123401045958974, 0.000336854126836293}},
    {{5.36199280681367, -1.46099908985536, 0.126755291030074, -0.0039102734460725},
     {3.41597143103046, -0.066984162951578, 0.0138944877787003, -0.000558939998921912},
     {1.37371376794871, -0.246963827944892, 0.0209674231346363, -0.000684856715039738}},
};

static int BaseIndex(char b)
{
    switch (b) { case 'A': return 0; case 'C': return 1; case 'G': return 2; case 'T': return 3; }
    return -1;
}

// ContextParameterProvider::GetTransitionParameters (:66-110).
static Trans ProviderTrans(int ctx, const double snr[4])
{
    const double s = snr[BaseIndex(kCtxKey[ctx][1])];
    const double s2 = s * s;
    const double s3 = s2 * s;
    double xbs[3];
    double total = 1.0;
    for (int k = 0; k < 3; ++k) {
        const double* c = kCtxPoly[ctx][k];
        double xb = c[0] + s * c[1] + s2 * c[2] + s3 * c[3];
        xb = std::exp(xb);
        xbs[k] = xb;
        total += xb;
    }
    const double branch = 1.0 / total;
    for (int k = 0; k < 3; ++k) xbs[k] = xbs[k] / total;
    Trans t;
    t.match = xbs[1];
    t.stick = xbs[2];
    t.branch = branch;
    t.del = xbs[0];
    return t;
}

// ContextParameters (CC/src/C++/Arrow/ContextParameters.cpp:26-47).
struct ContextTable {
    Trans homo[4], het[4];
    explicit ContextTable(const double snr[4])
    {
        for (int b = 0; b < 4; ++b) {
            homo[b] = ProviderTrans(b, snr);
            het[b] = ProviderTrans(4 + b, snr);
        }
    }
    Trans Get(char b1, char b2) const
    {
        const int i2 = BaseIndex(b2);
        if (i2 < 0) throw std::out_of_range("context");
        return (b1 == b2) ? homo[i2] : het[i2];
    }
};

struct ModelParams {   // ArrowConfig.hpp:80-100 (IQV PMFs are all 1.0 and InsQv is 0 in ccs)
    double prMiscall = kMismatch;
    double prNot = 1.0 - kMismatch;
    double prThird = kMismatch / 3.0;
};


// -------------------------------------------------------- strand templates
// TemplateParameterPair (CC/src/C++/Arrow/TemplateParameterPair.cpp, .hpp:29-155).
struct StrandTemplate {
    static const int kNone = -100;
    std::string seq;
    std::vector<Trans> tp;
    int mpos = kNone;
    int moff = 0;
    char mbase[2] = {'0', '0'};
    Trans mtrans[2];

    StrandTemplate() {}
    StrandTemplate(const std::string& s, const ContextTable& ctx) : seq(s), tp(s.size())   // .cpp:43-59
    {
        for (int i = 0; i + 1 < (int)seq.size(); ++i) tp[i] = ctx.Get(seq[i], seq[i + 1]);
        tp[seq.size() - 1] = Trans();
    }
    bool Virtual() const { return mpos != kNone; }
    int Length() const { return (int)seq.size() - moff; }
    int VirtualLength(int start, int len) const   // .hpp:133-147
    {
        if (mpos >= start && mpos < start + len) return len - moff;
        return len;
    }
    std::pair<char, Trans> At(int i) const   // .hpp:88-112
    {
        if (!Virtual()) return {seq[i], tp[i]};
        if (i < mpos - 1) return {seq[i], tp[i]};
        if (i > mpos) return {seq[i + moff], tp[i + moff]};
        const int k = (i == mpos) ? 1 : 0;
        return {mbase[k], mtrans[k]};
    }
    void ClearVirtual()   // .cpp:61-68
    {
        mpos = kNone;
        moff = 0;
        mbase[0] = mbase[1] = '0';
        mtrans[0] = mtrans[1] = Trans();
    }
    void ApplyVirtual(const Mut& m, const ContextTable& ctx)   // .cpp:70-140
    {
        ClearVirtual();
        const int s = m.start;
        mpos = s;
        const int L = (int)seq.size();
        if (m.type == SUB) {
            moff = 0;
            const char nb = m.bases[0];
            mbase[1] = nb;
            if (s > 0) {
                mbase[0] = seq[s - 1];
                mtrans[0] = ctx.Get(seq.at(s - 1), nb);
            }
            if (s + 1 < L) mtrans[1] = ctx.Get(nb, seq.at(s + 1));
        } else if (m.type == DEL) {
            moff = 1;
            const int last = L - 1;
            if (s > 0 && s < last) {
                mbase[0] = seq.at(s - 1);
                mbase[1] = seq.at(s + 1);
                mtrans[0] = ctx.Get(seq.at(s - 1), seq.at(s + 1));
                mtrans[1] = tp[s + 1];
            } else if (s == 0) {
                mbase[1] = seq.at(s + 1);
                mtrans[1] = tp[s + 1];
            } else if (s == last) {
                mbase[0] = seq.at(s - 1);
            }
        } else {
            moff = -1;
            const char nb = m.bases[0];
            mbase[1] = nb;
            if (s > 0) {
                mbase[0] = seq.at(s - 1);
                mtrans[0] = ctx.Get(seq.at(s - 1), nb);
            }
            if (s < L) mtrans[1] = ctx.Get(nb, seq.at(s));
        }
    }
    void ApplyOneReal(const Mut& m, int s, const ContextTable& ctx)   // .cpp:150-210
    {
        if (m.type == SUB) {
            seq.replace(s, m.end - m.start, m.bases);
            if (s + 1 < (int)seq.size()) tp[s] = ctx.Get(seq.at(s), seq.at(s + 1));
            if (s > 0) tp[s - 1] = ctx.Get(seq.at(s - 1), seq.at(s));
        } else if (m.type == DEL) {
            const int last = (int)seq.size() - 1;
            seq.erase(s, m.end - m.start);
            const int n = m.end - m.start;
            if (s > 0 && s < last) {
                tp[s - 1] = ctx.Get(seq.at(s - 1), seq.at(s));
                tp.erase(tp.begin() + s, tp.begin() + s + n);
            } else if (s == 0) {
                tp.erase(tp.begin() + s, tp.begin() + s + n);
            } else if (s == last) {
                tp.erase(tp.begin() + s - 1, tp.begin() + s - 1 + n);
            }
        } else {
            seq.insert(s, m.bases);
            if (s > (int)tp.size()) tp.push_back(Trans());
            else tp.insert(tp.begin() + s, Trans());
            if (s > 0) tp[s - 1] = ctx.Get(seq.at(s - 1), seq.at(s));
            if (s < (int)tp.size()) tp[s] = ctx.Get(seq.at(s), seq.at(s + 1));
        }
    }
    void ApplyReal(std::vector<Mut> muts, const ContextTable& ctx)   // .cpp:212-222
    {
        std::sort(muts.begin(), muts.end());
        int shift = 0;
        for (const Mut& m : muts) {
            ApplyOneReal(m, m.start + shift, ctx);
            shift += m.LengthDiff();
        }
    }
};

// WrappedTemplateParameterPair (.hpp:165-218): a read's window onto a strand template.
struct Window {
    const StrandTemplate* base = nullptr;
    int start = 0, len = 0;
    int Length() const { return base->VirtualLength(start, len); }
    std::pair<char, Trans> At(int i) const { return base->At(i + start); }
};

// --------------------------------------------------------------- band matrix
// ScaledSparseMatrixD = ScaledMatrix<SparseMatrix<double,double>>
// (CC/include/ConsensusCore/Matrix/ScaledMatrix-inl.hpp:14-85, SparseMatrix-inl.hpp:86-271,
//  SparseVector-inl.hpp:42-190).  Cells outside a column's used range read as 0.0: the
// reference zero-fills storage on StartEditingColumn and only sets used rows.
struct BandMatrix {
    int rows = 0, cols = 0;
    std::vector<int> ub, ue;                 // used row range per column
    std::vector<int> ab;                     // first allocated row per column
    std::vector<std::vector<double>> store;  // allocated storage per column
    std::vector<double> logScale;

    BandMatrix() {}
    BandMatrix(int r, int c) : rows(r), cols(c), ub(c, 0), ue(c, 0), ab(c, 0), store(c), logScale(c, 0.0) {}
    bool IsNull() const { return rows == 0 && cols == 0; }
    bool Empty(int j) const { return ub[j] >= ue[j]; }
    double Get(int i, int j) const
    {
        const int k = i - ab[j];
        if (k < 0 || k >= (int)store[j].size()) return 0.0;
        return store[j][k];
    }
    void Start(int j, int hb, int he)
    {
        ab[j] = std::max(hb - 8, 0);
        const int aend = std::min(he + 8, rows);
        store[j].assign(std::max(0, aend - ab[j]), 0.0);
    }
    void Set(int i, int j, double v)
    {
        int k = i - ab[j];
        if (k < 0 || k >= (int)store[j].size()) {   // SparseVector::ExpandAllocated semantics
            const int nb = std::max(std::min(i - 8, ab[j]), 0);
            const int ne = std::min(std::max(i + 8, ab[j] + (int)store[j].size()), rows);
            std::vector<double> grown(ne - nb, 0.0);
            for (size_t t = 0; t < store[j].size(); ++t) grown[ab[j] - nb + t] = store[j][t];
            store[j].swap(grown);
            ab[j] = nb;
            k = i - ab[j];
        }
        store[j][k] = v;
    }
    void Finish(int j, int b, int e)   // ScaledMatrix::FinishEditingColumn (:35-60)
    {
        double c = 0.0;
        for (int i = b; i < e; ++i) c = std::max(c, Get(i, j));
        if (c != 0.0 && c != 1.0) {
            for (int i = b; i < e; ++i) Set(i, j, Get(i, j) / c);
            logScale[j] = std::log(c);
        } else {
            logScale[j] = 0.0;
        }
        ub[j] = b;
        ue[j] = e;
    }
    long UsedEntries() const
    {
        long n = 0;
        for (int j = 0; j < cols; ++j) n += ue[j] - ub[j];
        return n;
    }
    double LogProd(int b, int e) const
    {
        return std::accumulate(logScale.begin() + b, logScale.begin() + e, 0.0);
    }
    double LogProdAll() const { return std::accumulate(logScale.begin(), logScale.end(), 0.0); }
};

static const BandMatrix& NullMatrix()
{
    static BandMatrix n;
    return n;
}

// ------------------------------------------------------------------ recursor
// Arrow::SimpleRecursor<ScaledSparseMatrixD, SumProductCombiner>
// (CC/src/C++/Arrow/SimpleRecursor.cpp).  Combine is `+`; IQV PMFs are 1.0.
struct Recursor {
    std::string read;
    Window tpl;
    ModelParams mp;
    double scoreDiff = 12.5;
    // Diagnostics (orc_scorer_pass_log): per pass of the last FillAlphaBeta -- alpha?, used cells, tallest
    // column, first column taller than 64 rows (-1: none), used cells of the columns before it.
    mutable std::vector<std::array<long long, 5>> passLog;
    void LogPass(bool alpha, const BandMatrix& m) const
    {
        long long used = 0, before = 0, firstTall = -1;
        int mh = 0;
        for (int j = 0; j < m.cols; ++j) {
            const int h = std::max(0, m.ue[j] - m.ub[j]);
            if (h > 64 && firstTall < 0) {
                firstTall = j;
                before = used;
            }
            used += h;
            mh = std::max(mh, h);
        }
        passLog.push_back({alpha ? 1LL : 0LL, used, (long long)mh, firstTall, firstTall < 0 ? used : before});
    }

    // RowRange + RangeGuide (:693-757).  RowRange's threshold (max - scoreDiff) lies below every
    // scaled cell, so it returns the used range unchanged; kept literal here.
    static void Union(int& b, int& e, int ob, int oe) { b = std::min(b, ob); e = std::max(e, oe); }
    void RowRange(int j, const BandMatrix& m, int* ob, int* oe) const
    {
        int b = m.ub[j], e = m.ue[j];
        int maxRow = b;
        double maxScore = m.Get(maxRow, j);
        for (int i = b + 1; i < e; ++i) {
            const double s = m.Get(i, j);
            if (s > maxScore) { maxRow = i; maxScore = s; }
        }
        const double thr = maxScore - scoreDiff;
        int i;
        for (i = b; i < maxRow && m.Get(i, j) < thr; ++i) {}
        b = i;
        for (i = e - 1; i >= maxRow && m.Get(i, j) < thr; --i) {}
        e = i + 1;
        *ob = b;
        *oe = e;
    }
    void Guide(int j, const BandMatrix& guide, const BandMatrix& self, int* hb, int* he) const
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

    // FillAlpha (:60-181)
    void FillAlpha(const BandMatrix& guide, BandMatrix& a) const
    {
        const int I = (int)read.size();
        const int J = tpl.Length();
        a.Start(0, 0, 1);
        a.Set(0, 0, 1.0);
        a.Finish(0, 0, 1);
        int hb = 1, he = 1;
        Trans prevT;
        const double sdn = std::exp(scoreDiff);
        for (int j = 1; j < J; ++j) {
            const std::pair<char, Trans> cur = tpl.At(j - 1);
            Guide(j, guide, a, &hb, &he);
            const int reqEnd = std::min(I, he);
            double thr = 0.0, mx = 0.0, score = 0.0;
            a.Start(j, hb, he);
            const char nextBase = tpl.At(j).first;
            const int b = hb;
            int i;
            for (i = b; i < I && (score >= thr || i < reqEnd); ++i) {
                const char rb = read[i - 1];
                double move = 0.0;
                score = 0.0;
                const double mpe = a.Get(i - 1, j - 1) * (rb == cur.first ? mp.prNot : mp.prThird);
                if (i == 1 && j == 1) move = mpe;
                else if (i != 1 && j != 1) move = mpe * prevT.match;
                score = score + move * 1.0;
                if (i > 1) {
                    const double tep = rb == nextBase ? cur.second.branch : (cur.second.stick / 3.0);
                    move = a.Get(i - 1, j) * tep * 1.0;
                    score = score + move;
                }
                if (j > 1) {
                    move = a.Get(i, j - 1) * prevT.del;
                    score = score + move;
                }
                a.Set(i, j, score);
                if (score > mx) { mx = score; thr = mx / sdn; }
            }
            const int e = i;
            a.Finish(j, b, e);
            prevT = cur.second;
            he = e;
            for (i = b; i < e && a.Get(i, j) < thr; ++i) {}
            hb = i;
        }
        const char lastBase = tpl.At(J - 1).first;
        const double em = read[I - 1] == lastBase ? mp.prNot : mp.prThird;
        const double lik = a.Get(I - 1, J - 1) * em * 1.0;
        a.Start(J, I, I + 1);
        a.Set(I, J, lik);
        a.Finish(J, I, I + 1);
    }

    // FillBeta (:183-296)
    void FillBeta(const BandMatrix& guide, BandMatrix& bm) const
    {
        const int I = (int)read.size();
        const int J = tpl.Length();
        bm.Start(J, I, I + 1);
        bm.Set(I, J, 1.0);
        bm.Finish(J, I, I + 1);
        const double sdn = std::exp(scoreDiff);
        int hb = I, he = I;
        for (int j = J - 1; j > 0; --j) {
            const char nextBase = tpl.At(j).first;
            const Trans curT = tpl.At(j - 1).second;
            Guide(j, guide, bm, &hb, &he);
            const int reqBegin = std::max(0, hb);
            bm.Start(j, hb, he);
            double score = 0.0, thr = 0.0, mx = 0.0;
            const int e = he;
            int i;
            for (i = e - 1; i > 0 && (score >= thr || i >= reqBegin); --i) {
                const char nb = read[i];
                double move;
                score = 0.0;
                const bool same = nb == nextBase;
                const double mpe = bm.Get(i + 1, j + 1) * (same ? mp.prNot : mp.prThird);
                if (i < I - 1) score = score + mpe * curT.match * 1.0;
                else if (i == I - 1 && j == J - 1) score = score + mpe * 1.0;
                if (i < I - 1 && i > 0) {
                    const double tep = same ? curT.branch : (curT.stick / 3.0);
                    move = bm.Get(i + 1, j) * tep * 1.0;
                    score = score + move;
                }
                if (j < J - 1 && j > 0) {
                    move = bm.Get(i, j + 1) * curT.del;
                    score = score + move;
                }
                bm.Set(i, j, score);
                if (score > mx) { mx = score; thr = mx / sdn; }
            }
            const int b = i + 1;
            bm.Finish(j, b, e);
            hb = b;
            for (i = e; i > b && bm.Get(i - 1, j) < thr; --i) {}
            he = i;
        }
        bm.Start(0, 0, 1);
        const double em = (tpl.At(0).first == read[0]) ? mp.prNot : mp.prThird;
        bm.Set(0, 0, em * bm.Get(1, 1) * 1.0);
        bm.Finish(0, 0, 1);
    }

    // LinkAlphaBeta (:306-357)
    double Link(const BandMatrix& a, int ac, const BandMatrix& bm, int bc, int absc) const
    {
        const int I = (int)read.size();
        int ub = a.ub[ac - 2], ue = a.ue[ac - 2];
        // RangeUnion(RangeUnion(r1, r2), RangeUnion(r3, r4)) -- min/max are associative
        Union(ub, ue, a.ub[ac - 1], a.ue[ac - 1]);
        Union(ub, ue, bm.ub[bc], bm.ue[bc]);
        Union(ub, ue, bm.ub[bc + 1], bm.ue[bc + 1]);
        double v = 0.0;
        const char curBase = tpl.At(absc - 1).first;
        const Trans prevT = tpl.At(absc - 2).second;
        for (int i = ub; i < ue; ++i) {
            if (i < I) {
                const char rb = read[i];
                const double mprob = prevT.match * (rb == curBase ? mp.prNot : mp.prThird);
                v = v + a.Get(i, ac - 1) * mprob * bm.Get(i + 1, bc) * 1.0;
            }
            v = v + a.Get(i, ac - 1) * prevT.del * bm.Get(i, bc);
        }
        return std::log(v) + a.LogProd(0, ac) + bm.LogProd(bc, bm.cols);
    }

    // ExtendAlpha (:373-487)
    void ExtendAlpha(const BandMatrix& a, int beginCol, BandMatrix& ext, int nCols) const
    {
        const int maxLeft = tpl.Length();
        const int maxDown = (int)read.size();
        for (int c = 0; c < nCols; ++c) {
            const int j = beginCol + c;
            int b, e;
            if (j < tpl.Length()) {
                b = a.ub[j];
                e = a.ue[j];
                if (j - 1 >= 0) { b = std::min(b, a.ub[j - 1]); e = std::max(e, a.ue[j - 1]); }
                if (j + 1 < tpl.Length()) { b = std::min(b, a.ub[j + 1]); e = std::max(e, a.ue[j + 1]); }
            } else {
                b = a.ub[a.cols - 1];
                e = a.rows;
            }
            ext.Start(c, b, e);
            double score = 0.0;
            const std::pair<char, Trans> cur = tpl.At(j - 1);
            Trans prevT;
            if (j > 1) prevT = tpl.At(j - 2).second;
            char nextBase = 0;
            if (j != maxLeft) nextBase = tpl.At(j).first;
            for (int i = b; i < e; ++i) {
                const char rb = read[i - 1];
                double move = 0.0;
                if (i > 0 && j > 0) {
                    const double prev = c == 0 ? a.Get(i - 1, j - 1) : ext.Get(i - 1, c - 1);
                    const double em = rb == cur.first ? mp.prNot : mp.prThird;
                    if (i == 1 && j == 1) move = em;
                    else if (i < maxDown && j < maxLeft) move = prev * prevT.match * em;
                    else if (i == maxDown && j == maxLeft) move = prev * em;
                    score = move * 1.0;
                }
                if (i > 1 && i < maxDown && j != maxLeft) {
                    const double iep = (nextBase == rb) ? cur.second.branch : (cur.second.stick / 3.0);
                    move = ext.Get(i - 1, c) * iep * 1.0;
                    score = score + move;
                }
                if (j > 1 && j < maxLeft && i != maxDown) {
                    const double prev = c == 0 ? a.Get(i, j - 1) : ext.Get(i, c - 1);
                    move = prev * prevT.del;
                    score = score + move;
                }
                ext.Set(i, c, score);
            }
            ext.Finish(c, b, e);
        }
    }

    // ExtendBeta (:509-628)
    void ExtendBeta(const BandMatrix& bm, int lastCol, BandMatrix& ext, int lengthDiff) const
    {
        const int I = (int)read.size();
        const int J = tpl.Length();
        const int nExt = lengthDiff + lastCol + 1;
        const int firstCol = 0 - lengthDiff;
        const int lastExt = nExt - 1;
        for (int j = lastCol; j > lastCol - nExt; --j) {
            const int jp = j + lengthDiff;
            const int c = lastExt - (lastCol - j);
            int b, e;
            if (j < 0) {
                b = 0;
                e = bm.ue[0];
            } else {
                b = bm.ub[j];
                e = bm.ue[j];
                if (j - 1 >= 0) { b = std::min(b, bm.ub[j - 1]); e = std::max(e, bm.ue[j - 1]); }
                if (j + 1 < tpl.Length()) { b = std::min(b, bm.ub[j + 1]); e = std::max(e, bm.ue[j + 1]); }
            }
            ext.Start(c, b, e);
            const char nextBase = tpl.At(jp).first;
            Trans curT;
            if (jp > 0) curT = tpl.At(jp - 1).second;
            for (int i = e - 1; i >= b; --i) {
                char nb = 'N';
                if (i < I) nb = read[i];
                double move = 0.0;
                double score = 0.0;
                const bool same = nb == nextBase;
                if (i < I && j < J) {
                    const double nxt = (c == lastExt) ? bm.Get(i + 1, j + 1) : ext.Get(i + 1, c + 1);
                    const double em = same ? mp.prNot : mp.prThird;
                    if ((i == I - 1 && jp == J - 1) || (i == 0 && j == firstCol)) move = nxt * em;
                    else if (j > firstCol && i > 0) move = nxt * curT.match * em;
                    score = score + move * 1.0;
                }
                if (i < I - 1 && i > 0 && j > firstCol) {
                    const double iep = same ? curT.branch : (curT.stick / 3.0);
                    move = ext.Get(i + 1, c) * iep * 1.0;
                    score = score + move;
                }
                if (j < J - 1 && j > firstCol && i > 0) {
                    const double nxt = (c == lastExt) ? bm.Get(i, j + 1) : ext.Get(i, c + 1);
                    move = nxt * curT.del;
                    score = score + move;
                }
                ext.Set(i, c, score);
            }
            ext.Finish(c, b, e);
        }
    }

    // FillAlphaBeta (:642-691); returns flip-flop count, throws AlphaBetaMismatch.
    int FillAlphaBeta(BandMatrix& a, BandMatrix& bm) const
    {
        passLog.clear();
        FillAlpha(NullMatrix(), a);
        LogPass(true, a);
        FillBeta(a, bm);
        LogPass(false, bm);
        const int I = (int)read.size();
        const int J = tpl.Length();
        int flips = 0;
        const int maxSize = static_cast<int>(0.5 + kRebandFrac * (I + 1) * (J + 1));
        if (a.UsedEntries() >= maxSize || bm.UsedEntries() >= maxSize) {
            FillAlpha(bm, a);
            LogPass(true, a);
            FillBeta(a, bm);
            LogPass(false, bm);
            FillAlpha(bm, a);
            LogPass(true, a);
            flips += 3;
        }
        double av = std::log(a.Get(I, J)) + a.LogProdAll();
        double bv = std::log(bm.Get(0, 0)) + bm.LogProdAll();
        while (std::fabs(av - bv) > kAlphaBetaTol && flips <= kMaxFlipFlops) {
            if (flips % 2 == 0) {
                FillAlpha(bm, a);
                LogPass(true, a);
            } else {
                FillBeta(a, bm);
                LogPass(false, bm);
            }
            ++flips;
        }
        av = std::log(a.Get(I, J)) + a.LogProdAll();
        bv = std::log(bm.Get(0, 0)) + bm.LogProdAll();
        const double mism = std::fabs(1.0 - av / bv);
        if (mism > kAlphaBetaTol) throw AlphaBetaMismatch();
        return flips;
    }
};

// ---------------------------------------------------------- mutation scorer
// Arrow::MutationScorer (CC/src/C++/Arrow/MutationScorer.cpp:53-272).
struct MutationScorer {
    Recursor rec;
    BandMatrix alpha, beta;
    mutable BandMatrix ext;
    int flips = 0;

    explicit MutationScorer(const Recursor& r) : rec(r)   // :53-75
    {
        const int I = (int)rec.read.size() + 1;
        const int J = rec.tpl.Length() + 1;
        alpha = BandMatrix(I, J);
        beta = BandMatrix(I, J);
        ext = BandMatrix(I, kExtendColumns);
        flips = rec.FillAlphaBeta(alpha, beta);
        if (std::isinf(Score())) throw AlphaBetaMismatch();
    }
    double Score() const { return std::log(beta.Get(0, 0)) + beta.LogProdAll(); }   // :93-98
    void SetTemplate(const Window& w)   // :119-131
    {
        rec.tpl = w;
        const int I = (int)rec.read.size() + 1;
        const int J = rec.tpl.Length() + 1;
        alpha = BandMatrix(I, J);
        beta = BandMatrix(I, J);
        flips = rec.FillAlphaBeta(alpha, beta);
    }
    double ScoreMutation(const Mut& m) const   // :169-272
    {
        if (!rec.tpl.base->Virtual()) throw std::runtime_error("BadExecutionOrder");
        const int betaLinkCol = 1 + m.end;
        const int absLinkCol = 1 + m.end + m.LengthDiff();
        const bool atBegin = m.start < 3;
        const bool atEnd = m.end > beta.cols - 1 - 2;
        double score;
        if (!atBegin && !atEnd) {
            int sc, len;
            if (m.type == DEL) { sc = m.start - 1; len = 2; }
            else { sc = m.start; len = 1 + (int)m.bases.size(); }
            rec.ExtendAlpha(alpha, sc, ext, len);
            score = rec.Link(ext, len, beta, betaLinkCol, absLinkCol);
            score += alpha.LogProd(0, sc);
        } else if (!atBegin && atEnd) {
            const int sc = m.start - 1;
            const int len = rec.tpl.Length() - sc + 1;
            rec.ExtendAlpha(alpha, sc, ext, len);
            score = std::log(ext.Get((int)rec.read.size(), len - 1)) + alpha.LogProd(0, sc) + ext.LogProd(0, len);
        } else if (atBegin && !atEnd) {
            const int last = m.end;
            const int len = m.end + m.LengthDiff() + 1;
            rec.ExtendBeta(beta, last, ext, m.LengthDiff());
            score = std::log(ext.Get(0, 0)) + beta.LogProd(last + 1, beta.cols) + ext.LogProd(0, len);
        } else {
            BandMatrix ap((int)rec.read.size() + 1, rec.tpl.Length() + 1);
            rec.FillAlpha(NullMatrix(), ap);
            score = std::log(ap.Get((int)rec.read.size(), rec.tpl.Length())) + ap.LogProdAll();
        }
        return score;
    }
};

// ------------------------------------------------------ per-base expectation
// ExpectedContextLL / PerBaseMeanAndVariance (CC/include/ConsensusCore/Arrow/Expectations.hpp:12-55).
static std::pair<double, double> ExpectedLL(const Trans& t, double eps)
{
    const double p_m = t.match, l_m = std::log(p_m), l2_m = l_m * l_m;
    const double p_d = t.del, l_d = std::log(p_d), l2_d = l_d * l_d;
    const double p_b = t.branch, l_b = std::log(p_b), l2_b = l_b * l_b;
    const double p_s = t.stick, l_s = std::log(p_s), l2_s = l_s * l_s;
    const double lgThird = -std::log(3.0);
    const double E_M = (1.0 - eps) * 0.0 + eps * lgThird, E2_M = eps * lgThird * lgThird;
    const double E_D = 0.0, E2_D = E_D * E_D;
    const double E_B = 0.0, E2_B = E_B * E_B;
    const double E_S = lgThird, E2_S = E_S * E_S;
    auto enn = [=](double lm, double ld, double lb, double ls, double em, double ed, double eb, double es) {
        const double e_md = (lm + em) * p_m / (p_m + p_d) + (ld + ed) * p_d / (p_m + p_d);
        const double e_i = (lb + eb) * p_b / (p_b + p_s) + (ls + es) * p_s / (p_b + p_s);
        const double e_bs = e_i * (p_s + p_b) / (p_m + p_d);
        return e_md + e_bs;
    };
    const double mean = enn(l_m, l_d, l_b, l_s, E_M, E_D, E_B, E_S);
    const double var = enn(l2_m, l2_d, l2_b, l2_s, E2_M, E2_D, E2_B, E2_S) - mean * mean;
    return {mean, var};
}

static std::vector<std::pair<double, double>> PerBaseMeanVar(const StrandTemplate& t, double eps)
{
    std::vector<std::pair<double, double>> mv;
    for (int i = 0; i < t.Length(); ++i) mv.push_back(ExpectedLL(t.At(i).second, eps));
    return mv;
}

// -------------------------------------------------- multi-read mutation scorer
// Arrow::MultiReadMutationScorer (CC/src/C++/Arrow/MultiReadMutationScorer.cpp:70-504, .hpp:60-284).
struct MappedRead {
    std::string seq;
    int strand = FWD;
    int ts = 0, te = 0;
};

struct ReadState {
    MappedRead read;
    MutationScorer* scorer = nullptr;
    bool active = false;
};

struct MultiReadScorer {
    ContextTable ctx;
    ModelParams mp;
    double scoreDiff = 12.5;
    double fastThreshold = -12.5;
    double addThreshold = std::numeric_limits<double>::quiet_NaN();
    StrandTemplate fwd, rev;
    std::vector<ReadState> reads;

    MultiReadScorer(const std::string& tpl, const double snr[4], double sd, double fastThr, double addThr)
        : ctx(snr), scoreDiff(sd), fastThreshold(fastThr), addThreshold(addThr),
          fwd(tpl, ctx), rev(RevComp(tpl), ctx) {}
    ~MultiReadScorer()
    {
        for (ReadState& rs : reads) delete rs.scorer;
    }
    int TemplateLength() const { return (int)fwd.seq.size(); }
    Window WindowFor(int strand, int ts, int te)   // .cpp:199-213
    {
        Window w;
        const int len = te - ts;
        if (strand == FWD) { w.base = &fwd; w.start = ts; }
        else { w.base = &rev; w.start = TemplateLength() - te; }
        w.len = len;
        return w;
    }
    static bool ReadScores(const MappedRead& r, const Mut& m)   // :70-80
    {
        if (m.type == INS) return r.ts <= m.end && m.start <= r.te;
        return r.ts < m.end && m.start < r.te;
    }
    static Mut Oriented(const MappedRead& r, const Mut& m)   // :93-139
    {
        Mut c = m;
        if (m.end - m.start > 1) {
            const int cs = std::max(m.start, r.ts);
            const int ce = std::min(m.end, r.te);
            if (m.type == SUB) c = Mut(m.type, cs, ce, m.bases.substr(cs - m.start, ce - cs));
            else c = Mut(m.type, cs, ce, m.bases);
        }
        if (r.strand == FWD) return Mut(c.type, c.start - r.ts, c.end - r.ts, c.bases);
        return Mut(c.type, r.te - c.end, r.te - c.start, RevComp(c.bases));
    }
    int AddRead(const MappedRead& mr, double threshold)   // :275-325
    {
        int res = R_SUCCESS;
        Recursor rec;
        rec.read = mr.seq;
        rec.tpl = WindowFor(mr.strand, mr.ts, mr.te);
        rec.mp = mp;
        rec.scoreDiff = scoreDiff;
        MutationScorer* sc = nullptr;
        try {
            sc = new MutationScorer(rec);
        } catch (AlphaBetaMismatch&) {
            sc = nullptr;
            res = R_ABMISMATCH;
        }
        if (sc != nullptr && !std::isnan(threshold)) {
            const double ll = sc->Score();
            double mean = 0.0, var = 0.0;
            const StrandTemplate& t = (mr.strand == FWD) ? fwd : rev;
            const std::vector<std::pair<double, double>> mv = PerBaseMeanVar(t, mp.prMiscall);
            for (int i = mr.ts; i < mr.te - 1; ++i) {
                mean += mv[i].first;
                var += mv[i].second;
            }
            const double z = (ll - mean) / std::sqrt(var);
            if (!std::isfinite(ll) || !std::isfinite(z) || z < threshold) {
                res = R_POORZ;
                delete sc;
                sc = nullptr;
            }
        }
        ReadState rs;
        rs.read = mr;
        rs.scorer = sc;
        rs.active = sc != nullptr;
        // the scorer's window must point at *our* template objects
        reads.push_back(rs);
        return res;
    }
    void ApplyVirtualBoth(const Mut& m)   // :338-348
    {
        fwd.ApplyVirtual(m, ctx);
        const int L = (int)fwd.seq.size();
        Mut rc(m.type, L - m.end, L - m.start, RevComp(m.bases));
        rev.ApplyVirtual(rc, ctx);
    }
    double Score(const Mut& m, double fastThr)   // :338-368
    {
        ApplyVirtualBoth(m);
        double sum = 0.0;
        for (const ReadState& rs : reads) {
            if (rs.active && ReadScores(rs.read, m)) {
                const Mut om = Oriented(rs.read, m);
                sum += (rs.scorer->ScoreMutation(om) - rs.scorer->Score());
            }
            if (sum < fastThr) break;
        }
        fwd.ClearVirtual();
        rev.ClearVirtual();
        return sum;
    }
    double Score(const Mut& m) { return Score(m, -DBL_MAX); }
    double FastScore(const Mut& m) { return Score(m, fastThreshold); }
    std::vector<double> Scores(const Mut& m, double unscored)   // :384-417
    {
        ApplyVirtualBoth(m);
        std::vector<double> out;
        for (const ReadState& rs : reads) {
            if (rs.active && ReadScores(rs.read, m))
                out.push_back(rs.scorer->ScoreMutation(Oriented(rs.read, m)) - rs.scorer->Score());
            else
                out.push_back(unscored);
        }
        fwd.ClearVirtual();
        rev.ClearVirtual();
        return out;
    }
    bool IsFavorable(const Mut& m) { return Score(m) > kMinFavorable; }
    bool FastIsFavorable(const Mut& m) { return FastScore(m) > kMinFavorable; }
    double BaselineScore() const   // :495-504
    {
        double s = 0.0;
        for (const ReadState& rs : reads)
            if (rs.active) s += rs.scorer->Score();
        return s;
    }
    void ApplyMutations(const std::vector<Mut>& muts)   // :235-267
    {
        const std::vector<int> mtp = TargetToQuery(muts, fwd.seq);
        fwd.ApplyReal(muts, ctx);
        rev = StrandTemplate(RevComp(fwd.seq), ctx);
        for (ReadState& rs : reads) {
            try {
                const int nts = mtp[rs.read.ts];
                const int nte = mtp[rs.read.te];
                rs.read.ts = nts;
                rs.read.te = nte;
                if (rs.active) rs.scorer->SetTemplate(WindowFor(rs.read.strand, nts, nte));
            } catch (AlphaBetaMismatch&) {
                rs.active = false;
            }
        }
    }
    // ZScores (.hpp:208-263)
    void ZScores(double* zg, double* za, std::vector<double>* zs) const
    {
        const std::vector<std::pair<double, double>> fm = PerBaseMeanVar(fwd, mp.prMiscall);
        const std::vector<std::pair<double, double>> rm = PerBaseMeanVar(rev, mp.prMiscall);
        zs->clear();
        double gmean = 0.0, gvar = 0.0;
        size_t n = 0;
        for (const ReadState& rs : reads) {
            if (!rs.active) { zs->push_back(std::numeric_limits<double>::quiet_NaN()); continue; }
            n += 1;
            const double ll = rs.scorer->Score();
            double mu = 0.0, var = 0.0;
            const int s = rs.read.ts, e = rs.read.te - 1, len = e - s;
            if (len < 1) { zs->push_back(std::numeric_limits<double>::quiet_NaN()); continue; }
            const std::vector<std::pair<double, double>>& mv = (rs.read.strand == FWD) ? fm : rm;
            for (int i = s; i < e; ++i) { mu += mv[i].first; var += mv[i].second; }
            gmean += mu;
            gvar += var;
            zs->push_back((ll - mu) / std::sqrt(var));
        }
        const double gs = BaselineScore();
        *zg = (gvar == 0.0) ? std::numeric_limits<double>::quiet_NaN() : (gs - gmean) / std::sqrt(gvar);
        *za = (n == 0 || gvar == 0.0) ? std::numeric_limits<double>::quiet_NaN()
                                      : (gs / n - gmean / n) / std::sqrt(gvar / n);
    }
};

// ------------------------------------------------------- refine / QV loop
// AbstractRefineConsensus / BestSubset / ConsensusQVs (CC/include/ConsensusCore/Consensus-inl.hpp:70-295).

static bool Refine(MultiReadScorer& mms, int maxIter, int sep, int nbhd, long* nTested, long* nApplied,
                   std::vector<std::vector<Mut>>* appliedLog)
{
    bool converged = false;
    std::set<std::string> history;   // the reference keeps boost::hash values of the templates
    std::vector<Scored> favorable;
    for (int iter = 0; iter < maxIter; ++iter) {
        std::vector<Mut> toTry;
        if (iter == 0) {
            toTry = UniqueMutations(mms.fwd.seq, 0, (int)mms.fwd.seq.size());
        } else {
            std::vector<Mut> centers;
            for (const Scored& s : favorable) centers.push_back(s.m);
            toTry = NearbyMutations(mms.fwd.seq, centers, nbhd);
        }
        *nTested += (long)toTry.size();
        favorable.clear();
        for (const Mut& m : toTry) {
            if (mms.FastIsFavorable(m)) {
                const float s = (float)mms.Score(m);
                favorable.push_back({m, s});
            }
        }
        if (favorable.empty()) { converged = true; break; }
        std::vector<Scored> best = BestSubset(favorable, sep);
        if (best.size() > 1) {
            std::vector<Mut> bm;
            for (const Scored& s : best) bm.push_back(s.m);
            const std::string next = ApplyMuts(bm, mms.fwd.seq);
            if (history.count(next)) best.resize(1);
        }
        *nApplied += (long)best.size();
        history.insert(mms.fwd.seq);
        std::vector<Mut> bm;
        for (const Scored& s : best) bm.push_back(s.m);
        if (appliedLog) appliedLog->push_back(bm);
        mms.ApplyMutations(bm);
    }
    return converged;
}

static int ProbabilityToQV(double p)   // Consensus-inl.hpp:130-138
{
    if (p < 0.0 || p > 1.0) throw std::invalid_argument("probability");
    if (p == 0.0) p = std::numeric_limits<double>::min();
    return static_cast<int>(std::round(-10.0 * std::log10(p)));
}

static std::vector<int> ConsensusQVs(MultiReadScorer& mms)   // Consensus-inl.hpp:274-295
{
    std::vector<int> qvs;
    const std::string tpl = mms.fwd.seq;
    for (size_t p = 0; p < tpl.size(); ++p) {
        double sum = 0.0;
        for (const Mut& m : UniqueMutations(tpl, (int)p, (int)p + 1)) {
            const double s = mms.Score(m);
            if (s < 0.0) sum += std::exp(s);
        }
        qvs.push_back(ProbabilityToQV(1.0 - 1.0 / (1.0 + sum)));
    }
    return qvs;
}

}  // namespace orc

// =============================================================================
//  extern "C" surface used by tests/ (via oracle/oracle.py) and bench.py's
//  cpu_baseline leg.  Mutations cross as (type, start, end, newBases).
// =============================================================================
using namespace orc;

extern "C" {

void* orc_scorer_new(const char* tpl, const double* snr, double scoreDiff, double fastThr, double addThr)
{
    try {
        return new MultiReadScorer(tpl, snr, scoreDiff, fastThr, addThr);
    } catch (...) {
        return nullptr;
    }
}

void orc_scorer_free(void* h) { delete static_cast<MultiReadScorer*>(h); }

int orc_scorer_add_read(void* h, const char* seq, int strand, int ts, int te, double threshold)
{
    MultiReadScorer* s = static_cast<MultiReadScorer*>(h);
    MappedRead r;
    r.seq = seq;
    r.strand = strand;
    r.ts = ts;
    r.te = te;
    try {
        return s->AddRead(r, threshold);
    } catch (...) {
        return -1;
    }
}

int orc_scorer_num_reads(void* h) { return (int)static_cast<MultiReadScorer*>(h)->reads.size(); }

int orc_scorer_read_info(void* h, int r, int* active, int* ts, int* te, double* ll, int* flips)
{
    MultiReadScorer* s = static_cast<MultiReadScorer*>(h);
    const ReadState& rs = s->reads.at(r);
    *active = rs.active ? 1 : 0;
    *ts = rs.read.ts;
    *te = rs.read.te;
    *ll = rs.scorer ? rs.scorer->Score() : std::numeric_limits<double>::quiet_NaN();
    *flips = rs.scorer ? rs.scorer->flips : -1;
    return 0;
}

static Mut MakeMut(int type, int start, int end, const char* bases)
{
    return Mut(type, start, end, std::string(bases ? bases : ""));
}

double orc_scorer_score(void* h, int type, int start, int end, const char* bases, double fastThr)
{
    return static_cast<MultiReadScorer*>(h)->Score(MakeMut(type, start, end, bases), fastThr);
}

int orc_scorer_scores(void* h, int type, int start, int end, const char* bases, double unscored, double* out)
{
    std::vector<double> v = static_cast<MultiReadScorer*>(h)->Scores(MakeMut(type, start, end, bases), unscored);
    for (size_t i = 0; i < v.size(); ++i) out[i] = v[i];
    return (int)v.size();
}

double orc_scorer_baseline(void* h) { return static_cast<MultiReadScorer*>(h)->BaselineScore(); }

int orc_scorer_template(void* h, int strand, char* out, int cap)
{
    MultiReadScorer* s = static_cast<MultiReadScorer*>(h);
    const std::string& t = strand == FWD ? s->fwd.seq : s->rev.seq;
    if ((int)t.size() + 1 > cap) return -(int)t.size() - 1;
    std::memcpy(out, t.c_str(), t.size() + 1);
    return (int)t.size();
}

int orc_scorer_apply(void* h, int n, const int* types, const int* starts, const int* ends, const char* bases)
{
    // bases: n single characters (single-base mutations); '-' for deletions
    std::vector<Mut> muts;
    for (int i = 0; i < n; ++i) {
        std::string nb = types[i] == DEL ? std::string() : std::string(1, bases[i]);
        muts.push_back(Mut(types[i], starts[i], ends[i], nb));
    }
    try {
        static_cast<MultiReadScorer*>(h)->ApplyMutations(muts);
    } catch (...) {
        return -1;
    }
    return 0;
}

void orc_scorer_zscores(void* h, double* zg, double* za, double* zs)
{
    std::vector<double> v;
    static_cast<MultiReadScorer*>(h)->ZScores(zg, za, &v);
    for (size_t i = 0; i < v.size(); ++i) zs[i] = v[i];
}

// Refine; applied mutations are logged as (iter, type, start, base) rows into `log` (cap rows).
int orc_refine(void* h, int maxIter, int sep, int nbhd, long* nTested, long* nApplied, int* log, int logCap,
               int* nLog)
{
    MultiReadScorer* s = static_cast<MultiReadScorer*>(h);
    std::vector<std::vector<Mut>> applied;
    *nTested = 0;
    *nApplied = 0;
    int conv;
    try {
        conv = Refine(*s, maxIter, sep, nbhd, nTested, nApplied, &applied) ? 1 : 0;
    } catch (...) {
        return -1;
    }
    int k = 0;
    for (size_t it = 0; it < applied.size(); ++it)
        for (const Mut& m : applied[it]) {
            if (k < logCap) {
                log[4 * k + 0] = (int)it;
                log[4 * k + 1] = m.type;
                log[4 * k + 2] = m.start;
                log[4 * k + 3] = m.bases.empty() ? '-' : m.bases[0];
            }
            ++k;
        }
    *nLog = k;
    return conv;
}

int orc_qvs(void* h, int* out, int cap)
{
    std::vector<int> q;
    try {
        q = ConsensusQVs(*static_cast<MultiReadScorer*>(h));
    } catch (...) {
        return -1;
    }
    if ((int)q.size() > cap) return -(int)q.size();
    for (size_t i = 0; i < q.size(); ++i) out[i] = q[i];
    return (int)q.size();
}

// Enumeration helpers (tests pin these against TestMutationEnumerator / TestMutations).
int orc_enum_unique(const char* tpl, int b, int e, int* types, int* starts, char* bases, int cap)
{
    std::vector<Mut> v = UniqueMutations(tpl, b, e);
    for (size_t i = 0; i < v.size() && (int)i < cap; ++i) {
        types[i] = v[i].type;
        starts[i] = v[i].start;
        bases[i] = v[i].bases.empty() ? '-' : v[i].bases[0];
    }
    return (int)v.size();
}

int orc_enum_nearby(const char* tpl, int nc, const int* cstarts, int nbhd, int* types, int* starts, char* bases,
                    int cap)
{
    std::vector<Mut> centers;
    for (int i = 0; i < nc; ++i) centers.push_back(Mut::Single(SUB, cstarts[i], 'A'));
    std::vector<Mut> v = NearbyMutations(tpl, centers, nbhd);
    for (size_t i = 0; i < v.size() && (int)i < cap; ++i) {
        types[i] = v[i].type;
        starts[i] = v[i].start;
        bases[i] = v[i].bases.empty() ? '-' : v[i].bases[0];
    }
    return (int)v.size();
}

int orc_apply_mutations(const char* tpl, int n, const int* types, const int* starts, const int* ends,
                        const char* bases, char* out, int cap, int* mtp, int mtpCap)
{
    std::vector<Mut> muts;
    for (int i = 0; i < n; ++i) {
        std::string nb = types[i] == DEL ? std::string() : std::string(1, bases[i]);
        muts.push_back(Mut(types[i], starts[i], ends[i], nb));
    }
    const std::string r = ApplyMuts(muts, tpl);
    const std::vector<int> t = TargetToQuery(muts, tpl);
    if ((int)r.size() + 1 > cap || (int)t.size() > mtpCap) return -1;
    std::memcpy(out, r.c_str(), r.size() + 1);
    for (size_t i = 0; i < t.size(); ++i) mtp[i] = t[i];
    return (int)r.size();
}

void orc_context_params(const double* snr, double* out /* 8 x 4: match, stick, branch, deletion */)
{
    for (int c = 0; c < 8; ++c) {
        const Trans t = ProviderTrans(c, snr);
        out[4 * c + 0] = t.match;
        out[4 * c + 1] = t.stick;
        out[4 * c + 2] = t.branch;
        out[4 * c + 3] = t.del;
    }
}

}  // extern "C"

// Diagnostics (test infrastructure): histogram of read r's final alpha column heights, bins of 8 rows (the last
// bin counts everything taller).
extern "C" int orc_scorer_height_hist(void* h, int r, long long* hist, int nbins)
{
    MultiReadScorer* s = static_cast<MultiReadScorer*>(h);
    const ReadState& rs = s->reads.at(r);
    if (!rs.scorer) return -1;
    const BandMatrix& m = rs.scorer->alpha;
    for (int b = 0; b < nbins; ++b) hist[b] = 0;
    for (int j = 1; j + 1 < m.cols; ++j) {
        const int hgt = std::max(0, m.ue[j] - m.ub[j]);
        hist[std::min(nbins - 1, hgt / 8)] += 1;
    }
    return 0;
}

// Diagnostics (test infrastructure): read r's last FillAlphaBeta, one row of 5 per pass (see Recursor::passLog).
extern "C" int orc_scorer_pass_log(void* h, int r, long long* out, int cap)
{
    MultiReadScorer* s = static_cast<MultiReadScorer*>(h);
    const ReadState& rs = s->reads.at(r);
    if (!rs.scorer) return -1;
    const auto& log = rs.scorer->rec.passLog;
    const int n = (int)log.size();
    for (int k = 0; k < n && k < cap; ++k)
        for (int q = 0; q < 5; ++q) out[5 * k + q] = log[k][q];
    return n;
}

// Diagnostics (test infrastructure): used-cell count and tallest column of read r's alpha and beta bands.
extern "C" int orc_scorer_band_stats(void* h, int r, long long* aUsed, long long* bUsed, int* aMaxH, int* bMaxH)
{
    MultiReadScorer* s = static_cast<MultiReadScorer*>(h);
    const ReadState& rs = s->reads.at(r);
    if (!rs.scorer) return -1;
    auto stats = [](const BandMatrix& m, long long* used, int* mh) {
        *used = 0;
        *mh = 0;
        for (int j = 0; j < m.cols; ++j) {
            const int hgt = std::max(0, m.ue[j] - m.ub[j]);
            *used += hgt;
            *mh = std::max(*mh, hgt);
        }
    };
    stats(rs.scorer->alpha, aUsed, aMaxH);
    stats(rs.scorer->beta, bUsed, bMaxH);
    return 0;
}

// Diagnostics (test infrastructure): cells of read r's alpha band that are exactly zero, and cells whose
// whole 64-row chunk (rows counted from each column's first used row) is zero.
// Diagnostics (test infrastructure): zero structure of read r's alpha band for chunks of `chunk` rows: out[0] used
// cells, out[1] exact zeros, out[2] cells of all-zero chunks, out[3] zeros before a column's first non-zero
// cell, out[4] zeros after its last non-zero cell.
extern "C" int orc_scorer_band_zero_profile(void* h, int r, int chunk, long long* out)
{
    MultiReadScorer* s = static_cast<MultiReadScorer*>(h);
    const ReadState& rs = s->reads.at(r);
    if (!rs.scorer) return -1;
    const BandMatrix& m = rs.scorer->alpha;
    for (int q = 0; q < 5; ++q) out[q] = 0;
    for (int j = 0; j < m.cols; ++j) {
        int first = -1, last = -1;
        for (int i = m.ub[j]; i < m.ue[j]; ++i)
            if (m.Get(i, j) != 0.0) {
                if (first < 0) first = i;
                last = i;
            }
        out[0] += std::max(0, m.ue[j] - m.ub[j]);
        out[3] += first < 0 ? std::max(0, m.ue[j] - m.ub[j]) : first - m.ub[j];
        out[4] += first < 0 ? 0 : m.ue[j] - 1 - last;
        for (int c0 = m.ub[j]; c0 < m.ue[j]; c0 += chunk) {
            const int c1 = std::min(c0 + chunk, m.ue[j]);
            int z = 0;
            for (int i = c0; i < c1; ++i) z += (m.Get(i, j) == 0.0);
            out[1] += z;
            if (z == c1 - c0) out[2] += z;
        }
    }
    return 0;
}

extern "C" int orc_scorer_band_zeros(void* h, int r, long long* zeros, long long* zeroChunkCells)
{
    MultiReadScorer* s = static_cast<MultiReadScorer*>(h);
    const ReadState& rs = s->reads.at(r);
    if (!rs.scorer) return -1;
    const BandMatrix& m = rs.scorer->alpha;
    *zeros = 0;
    *zeroChunkCells = 0;
    for (int j = 0; j < m.cols; ++j) {
        for (int c0 = m.ub[j]; c0 < m.ue[j]; c0 += 64) {
            const int c1 = std::min(c0 + 64, m.ue[j]);
            int z = 0;
            for (int i = c0; i < c1; ++i) z += (m.Get(i, j) == 0.0);
            *zeros += z;
            if (z == c1 - c0) *zeroChunkCells += z;
        }
    }
    return 0;
}
