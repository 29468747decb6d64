// include/pbccs_amd/Quiver.hpp -- the Quiver half of the ConsensusCore facade (ConsensusCore/include/ConsensusCore/
// Quiver/), header-only over the C ABI in include/pbccs_amd.h, beside the Arrow half in ConsensusCore.hpp.  A caller
// of ConsensusCore's Quiver classes compiles against the MI355X engine by swapping its Quiver includes for this one.
//
// Mirrored surface (reference file:line):
//   Move, BandingOptions, QvModelParams, QuiverConfig, QuiverConfigTable   Quiver/QuiverConfig.hpp:50-249,
//                                                                           QuiverConfig.cpp:67-138
//   QvSequenceFeatures, QvRead, MappedQvRead                               Features.hpp:69-100, Read.hpp:47-97
//   QvEvaluator (Inc / Del / Extra / Merge evaluated on the device)        Quiver/QvEvaluator.hpp:90-317
//   the recursor types (SparseSseQvRecursor, SparseSseQvSumProductRecursor, SseQvRecursor, SimpleQvRecursor,
//   SparseSimpleQvRecursor and their sum-product forms)                   Quiver/MutationScorer.hpp:93-99
//   AbstractMultiReadMutationScorer, MultiReadMutationScorer<R>,
//   SparseSseQv(SumProduct)MultiReadMutationScorer                        Quiver/MultiReadMutationScorer.hpp:55-245
//   RefineConsensus / ConsensusQVs over a Quiver scorer                    Consensus.hpp:63-79
// BandingOptions here is ConsensusCore::BandingOptions (Quiver's); Arrow's is ConsensusCore::Arrow::BandingOptions,
// as in the reference.
#pragma once

#include <cmath>
#include <limits>
#include <list>
#include <string>
#include <utility>
#include <vector>

#include "ConsensusCore.hpp"

namespace ConsensusCore {

// Move bits and BandingOptions (Quiver/QuiverConfig.hpp:50-74)
enum Move {
    INVALID_MOVE = 0x0,
    INCORPORATE = 0x1,
    EXTRA = 0x2,
    DELETE = 0x4,
    MERGE = 0x8,
    BASIC_MOVES = (INCORPORATE | EXTRA | DELETE),
    ALL_MOVES = (BASIC_MOVES | MERGE)
};

struct BandingOptions {
    float ScoreDiff;
    BandingOptions(int /*diagonalCross*/, float scoreDiff) : ScoreDiff(scoreDiff) {}
    BandingOptions(int /*diagonalCross*/, float scoreDiff, float /*dynamicAdjustFactor*/, float /*dynamicAdjustOffset*/)
        : ScoreDiff(scoreDiff)
    {}
};

// QvModelParams (Quiver/QuiverConfig.hpp:77-190)
struct QvModelParams {
    std::string ChemistryName, ModelName;
    float Match, Mismatch, MismatchS, Branch, BranchS, DeletionN, DeletionWithTag, DeletionWithTagS, Nce, NceS;
    float Merge[4], MergeS[4];
    QvModelParams(const std::string& chemistryName, const std::string& modelName, float match, float mismatch,
                  float mismatchS, float branch, float branchS, float deletionN, float deletionWithTag,
                  float deletionWithTagS, float nce, float nceS, float merge, float mergeS)
        : ChemistryName(chemistryName), ModelName(modelName), Match(match), Mismatch(mismatch), MismatchS(mismatchS),
          Branch(branch), BranchS(branchS), DeletionN(deletionN), DeletionWithTag(deletionWithTag),
          DeletionWithTagS(deletionWithTagS), Nce(nce), NceS(nceS)
    {
        for (int b = 0; b < 4; ++b) {
            Merge[b] = merge;
            MergeS[b] = mergeS;
        }
    }
    QvModelParams(const std::string& chemistryName, const std::string& modelName, float match, float mismatch,
                  float mismatchS, float branch, float branchS, float deletionN, float deletionWithTag,
                  float deletionWithTagS, float nce, float nceS, float merge_A, float merge_C, float merge_G,
                  float merge_T, float mergeS_A, float mergeS_C, float mergeS_G, float mergeS_T)
        : ChemistryName(chemistryName), ModelName(modelName), Match(match), Mismatch(mismatch), MismatchS(mismatchS),
          Branch(branch), BranchS(branchS), DeletionN(deletionN), DeletionWithTag(deletionWithTag),
          DeletionWithTagS(deletionWithTagS), Nce(nce), NceS(nceS), Merge{merge_A, merge_C, merge_G, merge_T},
          MergeS{mergeS_A, mergeS_C, mergeS_G, mergeS_T}
    {}
    float Merge_A() const { return Merge[0]; }
    float Merge_C() const { return Merge[1]; }
    float Merge_G() const { return Merge[2]; }
    float Merge_T() const { return Merge[3]; }
    float MergeS_A() const { return MergeS[0]; }
    float MergeS_C() const { return MergeS[1]; }
    float MergeS_G() const { return MergeS[2]; }
    float MergeS_T() const { return MergeS[3]; }
    pbccs_qv_model_params ToC() const
    {
        pbccs_qv_model_params c;
        c.match = Match;
        c.mismatch = Mismatch;
        c.mismatch_s = MismatchS;
        c.branch = Branch;
        c.branch_s = BranchS;
        c.deletion_n = DeletionN;
        c.deletion_with_tag = DeletionWithTag;
        c.deletion_with_tag_s = DeletionWithTagS;
        c.nce = Nce;
        c.nce_s = NceS;
        for (int b = 0; b < 4; ++b) {
            c.merge[b] = Merge[b];
            c.merge_s[b] = MergeS[b];
        }
        return c;
    }
};

// QuiverConfig (Quiver/QuiverConfig.hpp:193-208)
struct QuiverConfig {
    QvModelParams QvParams;
    int MovesAvailable;
    BandingOptions Banding;
    float FastScoreThreshold;
    float AddThreshold;
    QuiverConfig(const QvModelParams& qvParams, int movesAvailable, const BandingOptions& bandingOptions,
                 float fastScoreThreshold, float addThreshold = 1.0f)
        : QvParams(qvParams), MovesAvailable(movesAvailable), Banding(bandingOptions),
          FastScoreThreshold(fastScoreThreshold), AddThreshold(addThreshold)
    {}
};

// QuiverConfigTable (Quiver/QuiverConfig.hpp:212-249, QuiverConfig.cpp:67-138): entries pushed to the front; At()
// finds the chemistry, else the "*" fallback.
class QuiverConfigTable {
public:
    typedef std::pair<const std::string, const QuiverConfig> QuiverConfigTableEntry;
    typedef std::list<QuiverConfigTableEntry>::const_iterator const_iterator;
    bool InsertDefault(const QuiverConfig& config) { return InsertAs_("*", config); }
    bool Insert(const QuiverConfig& config) { return InsertAs(config.QvParams.ChemistryName, config); }
    bool InsertAs(const std::string& name, const QuiverConfig& config)
    {
        if (name == "*") throw InvalidInputError("Cannot Insert(...) a QuiverConfig with chemistry '*'");
        return InsertAs_(name, config);
    }
    int Size() const { return (int)table_.size(); }
    const QuiverConfig& At(const std::string& name) const
    {
        for (const auto& e : table_)
            if (e.first == name) return e.second;
        for (const auto& e : table_)
            if (e.first == "*") return e.second;
        throw InvalidInputError("Chemistry not found in QuiverConfigTable");
    }
    std::vector<std::string> Keys() const
    {
        std::vector<std::string> k;
        for (const auto& e : table_) k.push_back(e.first);
        return k;
    }
    const_iterator begin() const { return table_.begin(); }
    const_iterator end() const { return table_.end(); }

private:
    bool InsertAs_(const std::string& name, const QuiverConfig& config)
    {
        for (const auto& e : table_)
            if (e.first == name) return false;
        table_.push_front(QuiverConfigTableEntry(name, config));
        return true;
    }
    std::list<QuiverConfigTableEntry> table_;
};

// QvSequenceFeatures (Features.hpp:69-100): the bases and five QV tracks (a null track pointer reads as zeros)
struct QvSequenceFeatures {
    std::string Sequence;
    std::vector<float> SequenceAsFloat, InsQv, SubsQv, DelQv, DelTag, MergeQv;
    explicit QvSequenceFeatures(const std::string& seq) : QvSequenceFeatures(seq, (const float*)nullptr, nullptr,
                                                                             nullptr, nullptr, nullptr)
    {}
    QvSequenceFeatures(const std::string& seq, const float* insQv, const float* subsQv, const float* delQv,
                       const float* delTag, const float* mergeQv)
        : Sequence(seq)
    {
        const size_t n = seq.size();
        for (char c : seq) SequenceAsFloat.push_back((float)c);
        auto track = [n](std::vector<float>& v, const float* src) { v.assign(n, 0.0f);
                                                                    if (src) v.assign(src, src + n); };
        track(InsQv, insQv);
        track(SubsQv, subsQv);
        track(DelQv, delQv);
        track(DelTag, delTag);
        track(MergeQv, mergeQv);
    }
    QvSequenceFeatures(const std::string& seq, const unsigned char* insQv, const unsigned char* subsQv,
                       const unsigned char* delQv, const unsigned char* delTag, const unsigned char* mergeQv)
        : QvSequenceFeatures(seq)
    {
        const size_t n = seq.size();
        auto track = [n](std::vector<float>& v, const unsigned char* src) {
            if (src)
                for (size_t i = 0; i < n; ++i) v[i] = (float)src[i];
        };
        track(InsQv, insQv);
        track(SubsQv, subsQv);
        track(DelQv, delQv);
        track(DelTag, delTag);
        track(MergeQv, mergeQv);
    }
    int Length() const { return (int)Sequence.size(); }
    const char& operator[](int i) const { return Sequence[i]; }
    char ElementAt(int i) const { return Sequence[i]; }
};

struct QvRead {
    QvSequenceFeatures Features;
    std::string Name, Chemistry;
    QvRead(const QvSequenceFeatures& f, const std::string& name, const std::string& chem)
        : Features(f), Name(name), Chemistry(chem)
    {}
    int Length() const { return Features.Length(); }
};

struct MappedQvRead : public QvRead {
    StrandEnum Strand;
    int TemplateStart, TemplateEnd;
    bool PinStart, PinEnd;
    MappedQvRead(const QvRead& r, StrandEnum strand, int ts, int te, bool pinStart = true, bool pinEnd = true)
        : QvRead(r), Strand(strand), TemplateStart(ts), TemplateEnd(te), PinStart(pinStart), PinEnd(pinEnd)
    {}
};

// QvEvaluator (Quiver/QvEvaluator.hpp:90-317).  The move scores come from the device's evaluator (the one the
// recursions use): Inc / Del / Extra / Merge evaluate one cell per call, Moves() many cells in one launch.
class QvEvaluator {
public:
    typedef QvSequenceFeatures FeaturesType;
    typedef QvModelParams ParamsType;
    QvEvaluator(const QvRead& read, const std::string& tpl, const QvModelParams& params, bool pinStart = true,
                bool pinEnd = true)
        : read_(read), params_(params), tpl_(tpl), pinStart_(pinStart), pinEnd_(pinEnd)
    {}
    std::string ReadName() const { return read_.Name; }
    std::string Basecalls() const { return read_.Features.Sequence; }
    std::string Template() const { return tpl_; }
    void Template(std::string tpl) { tpl_ = tpl; }
    int ReadLength() const { return read_.Features.Length(); }
    int TemplateLength() const { return (int)tpl_.size(); }
    bool PinEnd() const { return pinEnd_; }
    bool PinStart() const { return pinStart_; }
    bool IsMatch(int i, int j) const { return read_.Features[i] == tpl_[j]; }
    float Inc(int i, int j) const { return One(i, j, 0); }
    float Del(int i, int j) const { return One(i, j, 1); }
    float Extra(int i, int j) const { return One(i, j, 2); }
    float Merge(int i, int j) const { return One(i, j, 3); }
    // the four moves at cells (i[k], j[k]); NaN where a cell is outside a move's domain
    void Moves(const std::vector<int>& i, const std::vector<int>& j, std::vector<float>* inc, std::vector<float>* del,
               std::vector<float>* extra, std::vector<float>* merge) const
    {
        if (i.size() != j.size()) throw InvalidInputError("cell lists differ in length");
        const int n = (int)i.size();
        std::vector<float>* outs[4] = {inc, del, extra, merge};
        for (std::vector<float>* o : outs)
            if (o) o->assign(n, 0.0f);
        const QvSequenceFeatures& f = read_.Features;
        pbccs_qv_features c;
        c.seq = f.Sequence.data();
        c.len = f.Length();
        c.ins_qv = f.InsQv.data();
        c.subs_qv = f.SubsQv.data();
        c.del_qv = f.DelQv.data();
        c.del_tag = f.DelTag.data();
        c.merge_qv = f.MergeQv.data();
        const pbccs_qv_model_params p = params_.ToC();
        detail::Check(pbccs_qv_evaluator_moves(detail::DefaultEngine(), &c, tpl_.data(), (int)tpl_.size(), &p,
                                               pinStart_ ? 1 : 0, pinEnd_ ? 1 : 0, i.data(), j.data(), n,
                                               inc ? inc->data() : nullptr, del ? del->data() : nullptr,
                                               extra ? extra->data() : nullptr, merge ? merge->data() : nullptr));
    }

private:
    float One(int i, int j, int which) const
    {
        std::vector<float> v[4];
        Moves(std::vector<int>(1, i), std::vector<int>(1, j), which == 0 ? &v[0] : nullptr,
              which == 1 ? &v[1] : nullptr, which == 2 ? &v[2] : nullptr, which == 3 ? &v[3] : nullptr);
        return v[which][0];
    }
    QvRead read_;
    QvModelParams params_;
    std::string tpl_;
    bool pinStart_, pinEnd_;
};

// The recursor types ConsensusCore instantiates its Quiver scorers over (Quiver/MutationScorer.hpp:93-99,
// SseRecursor.hpp, SimpleRecursor.hpp): recursor family x matrix storage x combiner.
template <int Kind, bool SumProduct>
struct QvRecursorType {
    static const int Recursor = Kind;             // PBCCS_QV_RECURSOR_*
    static const bool IsSumProduct = SumProduct;  // Viterbi (max) or sum-product (logAdd) combiner
    typedef QvEvaluator EvaluatorType;
};
typedef QvRecursorType<PBCCS_QV_RECURSOR_SPARSE_SSE, false> SparseSseQvRecursor;
typedef QvRecursorType<PBCCS_QV_RECURSOR_SPARSE_SSE, true> SparseSseQvSumProductRecursor;
typedef QvRecursorType<PBCCS_QV_RECURSOR_SPARSE_SIMPLE, false> SparseSimpleQvRecursor;
typedef QvRecursorType<PBCCS_QV_RECURSOR_SPARSE_SIMPLE, true> SparseSimpleQvSumProductRecursor;
typedef QvRecursorType<PBCCS_QV_RECURSOR_DENSE_SSE, false> SseQvRecursor;
typedef QvRecursorType<PBCCS_QV_RECURSOR_DENSE_SSE, true> SseQvSumProductRecursor;
typedef QvRecursorType<PBCCS_QV_RECURSOR_DENSE_SIMPLE, false> SimpleQvRecursor;
typedef QvRecursorType<PBCCS_QV_RECURSOR_DENSE_SIMPLE, true> SimpleQvSumProductRecursor;

// AbstractMultiReadMutationScorer (Quiver/MultiReadMutationScorer.hpp:55-124)
class AbstractMultiReadMutationScorer {
public:
    virtual ~AbstractMultiReadMutationScorer() {}
    virtual int TemplateLength() const = 0;
    virtual int NumReads() const = 0;
    virtual std::string Template(StrandEnum strand = FORWARD_STRAND) const = 0;
    virtual std::string Template(StrandEnum strand, int templateStart, int templateEnd) const = 0;
    virtual void ApplyMutations(const std::vector<Mutation>& mutations) = 0;
    virtual bool AddRead(const MappedQvRead& mappedRead, float threshold) = 0;
    virtual bool AddRead(const MappedQvRead& mappedRead) = 0;
    virtual float Score(const Mutation& m) const = 0;
    virtual float FastScore(const Mutation& m) const = 0;
    virtual std::vector<float> Scores(const Mutation& m, float unscoredValue) const = 0;
    virtual std::vector<float> Scores(const Mutation& m) const = 0;
    virtual bool IsFavorable(const Mutation& m) const = 0;
    virtual bool FastIsFavorable(const Mutation& m) const = 0;
    virtual std::vector<int> AllocatedMatrixEntries() const = 0;
    virtual std::vector<int> NumFlipFlops() const = 0;
    virtual float Score(MutationType mutationType, int position, const std::string& newBases) const = 0;
    virtual std::vector<float> Scores(MutationType mutationType, int position, const std::string& newBases,
                                      float unscoredValue) const = 0;
    virtual float BaselineScore() const = 0;
    virtual std::vector<float> BaselineScores() const = 0;
    // beyond the reference's abstract surface: MutationScorer<R>::ScoreMutation on read i's own scorer
    // (Quiver/MutationScorer.cpp:113-226) and RecursorBase::Alignment of read i (detail/RecursorBase.cpp:124-264)
    virtual float ReadScoreMutation(int i, const Mutation& m) const = 0;
    virtual std::pair<std::string, std::string> Alignment(int i) const = 0;
    virtual pbccs_quiver_scorer* Handle() const = 0;
};

// MultiReadMutationScorer<R> (Quiver/MultiReadMutationScorer.hpp:150-240) over the engine's Quiver scorer
template <typename R>
class MultiReadMutationScorer : public AbstractMultiReadMutationScorer {
public:
    typedef R RecursorType;
    typedef typename R::EvaluatorType EvaluatorType;
    MultiReadMutationScorer(const QuiverConfigTable& paramsByChemistry, std::string tpl) : handle_(nullptr)
    {
        std::vector<pbccs_quiver_config> cfgs;
        std::vector<std::string> names;
        for (const auto& e : paramsByChemistry) {
            const QuiverConfig& q = e.second;
            pbccs_quiver_config c;
            c.params = q.QvParams.ToC();
            c.moves_available = q.MovesAvailable;
            c.score_diff = q.Banding.ScoreDiff;
            c.fast_score_threshold = q.FastScoreThreshold;
            c.add_threshold = q.AddThreshold;
            c.sum_product = R::IsSumProduct ? 1 : 0;
            c.recursor = R::Recursor;
            cfgs.push_back(c);
            names.push_back(e.first);
        }
        std::vector<const char*> np;
        for (const std::string& n : names) np.push_back(n.c_str());
        detail::Check(pbccs_quiver_scorer_create(detail::DefaultEngine(), cfgs.data(), np.data(), (int)cfgs.size(),
                                                 tpl.data(), (int)tpl.size(), &handle_));
    }
    ~MultiReadMutationScorer()
    {
        if (handle_) pbccs_quiver_scorer_destroy(handle_);
    }
    MultiReadMutationScorer(const MultiReadMutationScorer&) = delete;
    MultiReadMutationScorer& operator=(const MultiReadMutationScorer&) = delete;

    int TemplateLength() const override { return (int)Template().size(); }
    int NumReads() const override { return pbccs_quiver_scorer_num_reads(handle_); }
    std::string Template(StrandEnum strand = FORWARD_STRAND) const override
    {
        int len = 0;
        char probe = 0;   // cap 0: the call reports the length (PBCCS_ERANGE)
        (void)pbccs_quiver_scorer_template(handle_, (int)strand, &probe, 0, &len);
        std::string out(len + 1, '\0');
        detail::Check(pbccs_quiver_scorer_template(handle_, (int)strand, &out[0], (int)out.size(), &len));
        out.resize(len);
        return out;
    }
    // MultiReadMutationScorer.cpp:176-190: the window [templateStart, templateEnd) of the strand's template
    std::string Template(StrandEnum strand, int templateStart, int templateEnd) const override
    {
        const std::string fwd = Template(FORWARD_STRAND);
        const int len = (int)fwd.size();
        if (strand == FORWARD_STRAND) return fwd.substr(templateStart, templateEnd - templateStart);
        return Template(REVERSE_STRAND).substr(len - templateEnd, templateEnd - templateStart);
    }
    void ApplyMutations(const std::vector<Mutation>& muts) override
    {
        std::vector<pbccs_mutation> c;
        for (const Mutation& m : muts) c.push_back(m.ToC());
        detail::Check(pbccs_quiver_scorer_apply_mutations(handle_, c.data(), (int)c.size()));
    }
    bool AddRead(const MappedQvRead& mr, float threshold) override
    {
        const QvSequenceFeatures& f = mr.Features;
        int active = 0;
        detail::Check(pbccs_quiver_scorer_add_read(handle_, f.Sequence.data(), f.Length(), f.InsQv.data(),
                                                   f.SubsQv.data(), f.DelQv.data(), f.DelTag.data(),
                                                   f.MergeQv.data(), mr.Chemistry.c_str(), (int)mr.Strand,
                                                   mr.TemplateStart, mr.TemplateEnd, threshold, &active));
        return active != 0;
    }
    bool AddRead(const MappedQvRead& mr) override { return AddRead(mr, std::numeric_limits<float>::quiet_NaN()); }
    float Score(const Mutation& m) const override { return ScoreOne(m, false); }
    float FastScore(const Mutation& m) const override { return ScoreOne(m, true); }
    std::vector<float> Scores(const Mutation& m, float unscoredValue) const override
    {
        const pbccs_mutation c = m.ToC();
        std::vector<float> out(NumReads());
        detail::Check(pbccs_quiver_scorer_scores(handle_, &c, unscoredValue, out.data()));
        return out;
    }
    std::vector<float> Scores(const Mutation& m) const override { return Scores(m, 0.0f); }
    bool IsFavorable(const Mutation& m) const override { return Favorable(m, false); }
    bool FastIsFavorable(const Mutation& m) const override { return Favorable(m, true); }
    std::vector<int> AllocatedMatrixEntries() const override
    {
        std::vector<int> out;
        for (int i = 0; i < NumReads(); ++i) {
            long long a = 0, b = 0;
            detail::Check(pbccs_quiver_scorer_allocated_entries(handle_, i, &a, &b));
            out.push_back((int)(a + b));
        }
        return out;
    }
    std::vector<int> NumFlipFlops() const override
    {
        std::vector<int> out(NumReads());
        detail::Check(pbccs_quiver_scorer_num_flipflops(handle_, out.data()));
        return out;
    }
    float Score(MutationType t, int position, const std::string& newBases) const override
    {
        return Score(Mutation(t, position, newBases));   // Mutation-inl.hpp:66-77
    }
    std::vector<float> Scores(MutationType t, int position, const std::string& newBases,
                              float unscoredValue) const override
    {
        return Scores(Mutation(t, position, newBases), unscoredValue);
    }
    std::vector<float> Scores(MutationType t, int position, const std::string& newBases) const
    {
        return Scores(t, position, newBases, 0.0f);
    }
    float BaselineScore() const override
    {
        float v = 0.0f;
        detail::Check(pbccs_quiver_scorer_baseline_score(handle_, &v));
        return v;
    }
    std::vector<float> BaselineScores() const override
    {
        std::vector<float> out(NumReads());
        int n = 0;
        detail::Check(pbccs_quiver_scorer_baseline_scores(handle_, out.data(), (int)out.size(), &n));
        out.resize(n);
        return out;
    }
    // not in the reference's MRMS surface: MutationScorer<R>::ScoreMutation of read i's own scorer
    // (Quiver/MutationScorer.cpp:113-226), the mutation in the read's window coordinates
    float ReadScoreMutation(int i, const Mutation& m) const override
    {
        const pbccs_mutation c = m.ToC();
        float v = 0.0f;
        detail::Check(pbccs_quiver_scorer_read_score_mutation(handle_, i, &c, &v));
        return v;
    }
    // RecursorBase::Alignment (detail/RecursorBase.cpp:124-264) of read i: gapped target and query
    std::pair<std::string, std::string> Alignment(int i) const override
    {
        int len = 0;
        (void)pbccs_quiver_scorer_alignment(handle_, i, nullptr, nullptr, 0, &len);
        std::string t(len + 1, '\0'), q(len + 1, '\0');
        detail::Check(pbccs_quiver_scorer_alignment(handle_, i, &t[0], &q[0], (int)t.size(), &len));
        t.resize(len);
        q.resize(len);
        return std::make_pair(t, q);
    }
    pbccs_quiver_scorer* Handle() const override { return handle_; }

private:
    float ScoreOne(const Mutation& m, bool fast) const
    {
        const pbccs_mutation c = m.ToC();
        float v = 0.0f;
        detail::Check(pbccs_quiver_scorer_score_many(handle_, &c, 1, fast ? 1 : 0, &v));
        return v;
    }
    bool Favorable(const Mutation& m, bool fast) const
    {
        const pbccs_mutation c = m.ToC();
        int f = 0;
        detail::Check(pbccs_quiver_scorer_is_favorable(handle_, &c, fast ? 1 : 0, &f));
        return f != 0;
    }
    pbccs_quiver_scorer* handle_;
};

typedef MultiReadMutationScorer<SparseSseQvRecursor> SparseSseQvMultiReadMutationScorer;
typedef MultiReadMutationScorer<SparseSseQvSumProductRecursor> SparseSseQvSumProductMultiReadMutationScorer;

// RefineConsensus / ConsensusQVs over a Quiver scorer (Consensus.hpp:63-79, Consensus-inl.hpp:159-295)
inline bool RefineConsensus(AbstractMultiReadMutationScorer& mms, size_t* nTested, size_t* nApplied,
                            const RefineOptions& opts = DefaultRefineOptions)
{
    pbccs_refine_options o;
    o.max_iterations = opts.MaximumIterations;
    o.mutation_separation = opts.MutationSeparation;
    o.mutation_neighborhood = opts.MutationNeighborhood;
    long long nt = 0, na = 0;
    int conv = 0;
    detail::Check(pbccs_quiver_refine_consensus(mms.Handle(), &o, &nt, &na, &conv));
    *nTested += (size_t)nt;
    *nApplied += (size_t)na;
    return conv != 0;
}

inline std::vector<int> ConsensusQVs(AbstractMultiReadMutationScorer& mms)
{
    std::vector<int> q(mms.TemplateLength());
    int n = 0;
    detail::Check(pbccs_quiver_consensus_qvs(mms.Handle(), q.data(), (int)q.size(), &n));
    q.resize(n);
    return q;
}

}  // namespace ConsensusCore
