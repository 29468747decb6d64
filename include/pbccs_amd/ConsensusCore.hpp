// include/pbccs_amd/ConsensusCore.hpp -- header-only C++ facade with ConsensusCore's class names over
// the C ABI in include/pbccs_amd.h, so that pbccs' per-ZMW driver (include/pacbio/ccs/Consensus.h:436-512)
// compiles against the MI355X engine by swapping its ConsensusCore includes for this header.
//
// Mirrored surface (reference file:line):
//   Arrow::SNR, ContextParameters            Arrow/ContextParameterProvider.hpp, ContextParameters.hpp
//   Arrow::BandingOptions, Arrow::ArrowConfig Arrow/ArrowConfig.hpp:63-128
//   ArrowSequenceFeatures, ArrowRead, MappedArrowRead, StrandEnum   Features.hpp, Read.hpp:47-97
//   Mutation, MutationType                    Mutation.hpp:50-129
//   Arrow::AddReadResult, ArrowMultiReadMutationScorer   Arrow/MultiReadMutationScorer.hpp:60-284
//   RefineOptions, RefineConsensus, ConsensusQVs          Consensus.hpp:48-79
// The Quiver family's classes are in pbccs_amd/Quiver.hpp (as ConsensusCore keeps them under Quiver/).
// Errors surface as ConsensusCore-style exceptions on the C++ side (the ABI itself never throws).
#pragma once

#include <cfloat>
#include <limits>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../pbccs_amd.h"

namespace ConsensusCore {

class InvalidInputError : public std::runtime_error {
public:
    explicit InvalidInputError(const std::string& m = "invalid input") : std::runtime_error(m) {}
};

class DeviceError : public std::runtime_error {
public:
    explicit DeviceError(const std::string& m) : std::runtime_error(m) {}
};

namespace detail {
inline void Check(int rc)
{
    if (rc == PBCCS_OK) return;
    const std::string msg = pbccs_last_error();
    if (rc == PBCCS_EINVAL || rc == PBCCS_ERANGE) throw InvalidInputError(msg);
    throw DeviceError(msg);
}

// One engine per process and device (ccs: one device per worker process).
inline pbccs_engine* DefaultEngine(int device = 0)
{
    static pbccs_engine* eng = nullptr;
    if (!eng) Check(pbccs_engine_create(device, &eng));
    return eng;
}
}  // namespace detail

enum MutationType { INSERTION = PBCCS_INSERTION, DELETION = PBCCS_DELETION, SUBSTITUTION = PBCCS_SUBSTITUTION };
enum StrandEnum { FORWARD_STRAND = PBCCS_FORWARD_STRAND, REVERSE_STRAND = PBCCS_REVERSE_STRAND };

class Mutation {
public:
    Mutation(MutationType type, int position, char base)
        : type_(type), start_(position), end_(type == INSERTION ? position : position + 1),
          newBases_(type == DELETION ? std::string() : std::string(1, base))
    {}
    Mutation(MutationType type, int start, int end, const std::string& newBases)
        : type_(type), start_(start), end_(end), newBases_(newBases)
    {
        if (!CheckInvariants()) throw InvalidInputError();
    }
    // Mutation-inl.hpp:66-77: end from the new bases' length (an insertion's is its start), a deletion's bases dropped
    Mutation(MutationType type, int position, const std::string& newBases)
        : type_(type), start_(position),
          end_(type == INSERTION ? position : position + (int)newBases.size()),
          newBases_(type == DELETION ? std::string() : newBases)
    {
        if (!CheckInvariants()) throw InvalidInputError();
    }
    // Mutation-inl.hpp:103-115
    bool CheckInvariants() const
    {
        return (type_ == INSERTION && start_ == end_ && !newBases_.empty()) ||
               (type_ == DELETION && start_ < end_ && newBases_.empty()) ||
               (type_ == SUBSTITUTION && start_ < end_ && (int)newBases_.size() == end_ - start_);
    }
    MutationType Type() const { return type_; }
    int Start() const { return start_; }
    int End() const { return end_; }
    std::string NewBases() const { return newBases_; }
    bool IsInsertion() const { return type_ == INSERTION; }
    bool IsDeletion() const { return type_ == DELETION; }
    bool IsSubstitution() const { return type_ == SUBSTITUTION; }
    int LengthDiff() const
    {
        return type_ == INSERTION ? (int)newBases_.size() : (type_ == DELETION ? start_ - end_ : 0);
    }
    bool operator<(const Mutation& o) const
    {
        if (start_ != o.start_) return start_ < o.start_;
        if (end_ != o.end_) return end_ < o.end_;
        if (type_ != o.type_) return type_ < o.type_;
        return newBases_ < o.newBases_;
    }
    bool operator==(const Mutation& o) const
    {
        return start_ == o.start_ && end_ == o.end_ && type_ == o.type_ && newBases_ == o.newBases_;
    }
    pbccs_mutation ToC() const
    {
        if (newBases_.size() > 1) throw InvalidInputError("Only mutations of size 1 allowed");
        pbccs_mutation m;
        m.type = (int)type_;
        m.start = start_;
        m.end = end_;
        m.new_base = newBases_.empty() ? '-' : newBases_[0];
        return m;
    }

private:
    MutationType type_;
    int start_, end_;
    std::string newBases_;
};

struct ArrowSequenceFeatures {
    std::string Sequence;
    explicit ArrowSequenceFeatures(const std::string& seq) : Sequence(seq) {}
    int Length() const { return (int)Sequence.size(); }
};

struct ArrowRead {
    ArrowSequenceFeatures Features;
    std::string Name, Chemistry;
    ArrowRead(const ArrowSequenceFeatures& f, const std::string& name, const std::string& chem)
        : Features(f), Name(name), Chemistry(chem)
    {}
    int Length() const { return Features.Length(); }
};

struct MappedArrowRead : public ArrowRead {
    StrandEnum Strand;
    int TemplateStart, TemplateEnd;
    MappedArrowRead(const ArrowRead& r, StrandEnum strand, int ts, int te)
        : ArrowRead(r), Strand(strand), TemplateStart(ts), TemplateEnd(te)
    {}
};

struct RefineOptions {
    int MaximumIterations;
    int MutationSeparation;
    int MutationNeighborhood;
};
static const RefineOptions DefaultRefineOptions = {40, 10, 20};

namespace Arrow {

enum AddReadResult { SUCCESS = 0, ALPHABETAMISMATCH = 1, MEM_FAIL = 2, POOR_ZSCORE = 3, OTHER = 4 };
static const char* AddReadResultNames[] = {"SUCCESS", "ALPHA/BETA MISMATCH", "EXCESSIVE MEMORY USAGE",
                                           "POOR Z-SCORE", "OTHER"};

struct SNR {
    double A, C, G, T;
    SNR(double a, double c, double g, double t) : A(a), C(c), G(g), T(t) {}
};

struct ContextParameters {
    SNR snr;
    explicit ContextParameters(const SNR& s) : snr(s) {}
};

struct BandingOptions {
    double ScoreDiff;
    explicit BandingOptions(double scoreDiff) : ScoreDiff(scoreDiff)
    {
        if (scoreDiff < 0) throw InvalidInputError("ScoreDiff must be positive!");
    }
};

class ArrowConfig {
public:
    ContextParameters CtxParams;
    BandingOptions Banding;
    double FastScoreThreshold;
    double AddThreshold;
    ArrowConfig(const ContextParameters& ctx, const BandingOptions& b, double fastScoreThreshold = -12.5,
                double addThreshold = std::numeric_limits<double>::quiet_NaN())
        : CtxParams(ctx), Banding(b), FastScoreThreshold(fastScoreThreshold), AddThreshold(addThreshold)
    {}
    pbccs_arrow_config ToC() const
    {
        pbccs_arrow_config c;
        c.snr[0] = CtxParams.snr.A;
        c.snr[1] = CtxParams.snr.C;
        c.snr[2] = CtxParams.snr.G;
        c.snr[3] = CtxParams.snr.T;
        c.score_diff = Banding.ScoreDiff;
        c.fast_score_threshold = FastScoreThreshold;
        c.add_threshold = AddThreshold;
        return c;
    }
};

class ArrowMultiReadMutationScorer {
public:
    ArrowMultiReadMutationScorer(const ArrowConfig& config, const std::string& tpl)
        : config_(config), handle_(nullptr)
    {
        const pbccs_arrow_config c = config.ToC();
        detail::Check(pbccs_scorer_create(detail::DefaultEngine(), &c, tpl.data(), (int)tpl.size(), &handle_));
    }
    ~ArrowMultiReadMutationScorer()
    {
        if (handle_) pbccs_scorer_destroy(handle_);
    }
    ArrowMultiReadMutationScorer(ArrowMultiReadMutationScorer&& o) noexcept : config_(o.config_), handle_(o.handle_)
    {
        o.handle_ = nullptr;
    }
    ArrowMultiReadMutationScorer(const ArrowMultiReadMutationScorer&) = delete;
    ArrowMultiReadMutationScorer& operator=(const ArrowMultiReadMutationScorer&) = delete;

    AddReadResult AddRead(const MappedArrowRead& mr, double threshold)
    {
        int res = 0;
        const std::string& s = mr.Features.Sequence;
        detail::Check(pbccs_scorer_add_read(handle_, s.data(), (int)s.size(), (int)mr.Strand, mr.TemplateStart,
                                            mr.TemplateEnd, threshold, &res));
        return (AddReadResult)res;
    }
    AddReadResult AddRead(const MappedArrowRead& mr) { return AddRead(mr, config_.AddThreshold); }

    double Score(const Mutation& m, double fastScoreThreshold = -DBL_MAX)
    {
        const pbccs_mutation c = m.ToC();
        double v = 0.0;
        detail::Check(pbccs_scorer_score(handle_, &c, fastScoreThreshold, &v));
        return v;
    }
    double Score(MutationType t, int position, char base) { return Score(Mutation(t, position, base)); }
    double FastScore(const Mutation& m) { return Score(m, config_.FastScoreThreshold); }
    std::vector<double> Scores(const Mutation& m, double unscoredValue = 0.0)
    {
        const pbccs_mutation c = m.ToC();
        std::vector<double> out(NumReads());
        detail::Check(pbccs_scorer_scores(handle_, &c, unscoredValue, out.data()));
        return out;
    }
    bool IsFavorable(const Mutation& m) { return Score(m) > 0.04; }
    bool FastIsFavorable(const Mutation& m) { return FastScore(m) > 0.04; }
    void ApplyMutations(const std::vector<Mutation>& muts)
    {
        std::vector<pbccs_mutation> c;
        for (const Mutation& m : muts) c.push_back(m.ToC());
        detail::Check(pbccs_scorer_apply_mutations(handle_, c.data(), (int)c.size()));
    }
    std::string Template(StrandEnum strand = FORWARD_STRAND) const
    {
        int len = 0;
        std::string out(TemplateLength() + 1, '\0');
        detail::Check(pbccs_scorer_template(handle_, (int)strand, &out[0], (int)out.size(), &len));
        out.resize(len);
        return out;
    }
    int TemplateLength() const { return pbccs_scorer_template_length(handle_); }
    int NumReads() const { return pbccs_scorer_num_reads(handle_); }
    double BaselineScore() const
    {
        double v = 0.0;
        detail::Check(pbccs_scorer_baseline_score(handle_, &v));
        return v;
    }
    std::vector<double> BaselineScores() const
    {
        std::vector<double> out(NumReads());
        int n = 0;
        detail::Check(pbccs_scorer_baseline_scores(handle_, out.data(), (int)out.size(), &n));
        out.resize(n);
        return out;
    }
    std::pair<std::pair<double, double>, std::vector<double>> ZScores() const
    {
        double zg = 0.0, za = 0.0;
        std::vector<double> zs(NumReads());
        detail::Check(pbccs_scorer_zscores(handle_, &zg, &za, zs.data()));
        return std::make_pair(std::make_pair(zg, za), zs);
    }
    std::vector<int> NumFlipFlops() const
    {
        std::vector<int> out(NumReads());
        detail::Check(pbccs_scorer_num_flipflops(handle_, out.data()));
        return out;
    }
    pbccs_scorer* Handle() { return handle_; }

private:
    ArrowConfig config_;
    pbccs_scorer* handle_;
};

}  // namespace Arrow

// RefineConsensus / ConsensusQVs (Consensus.hpp:63-79)
inline bool RefineConsensus(Arrow::ArrowMultiReadMutationScorer& mms, size_t* nTested, size_t* nApplied,
                            const RefineOptions& opts = DefaultRefineOptions)
{
    pbccs_refine_options o;
    o.max_iterations = opts.MaximumIterations;
    o.mutation_separation = opts.MutationSeparation;
    o.mutation_neighborhood = opts.MutationNeighborhood;
    long long nt = 0, na = 0;
    int conv = 0;
    detail::Check(pbccs_refine_consensus(mms.Handle(), &o, &nt, &na, &conv));
    *nTested += (size_t)nt;
    *nApplied += (size_t)na;
    return conv != 0;
}

inline std::vector<int> ConsensusQVs(Arrow::ArrowMultiReadMutationScorer& mms)
{
    std::vector<int> q(mms.TemplateLength());
    int n = 0;
    detail::Check(pbccs_consensus_qvs(mms.Handle(), q.data(), (int)q.size(), &n));
    q.resize(n);
    return q;
}

}  // namespace ConsensusCore
