// include/pbccs_amd/SparsePoa.hpp -- header-only C++ facade for the POA draft step, with pbccs's and
// ConsensusCore's names, over the C ABI in include/pbccs_amd.h (pbccs_sparse_poa_*, pbccs_poa_consensus).
// Consensus.h's PoaConsensus template (include/pacbio/ccs/Consensus.h:352-390) compiles against it by
// swapping its SparsePoa include for this header (tests/cpp/poa_driver.cpp does exactly that).
//
// Mirrored surface (reference file:line):
//   PacBio::CCS::Interval (Left/Right/Length/Covers/==)   include/pacbio/ccs/Interval.h:55-200
//   PacBio::CCS::PoaAlignmentSummary / PoaAlignmentOptions include/pacbio/ccs/SparsePoa.h:57-85
//   PacBio::CCS::SparsePoa                                 include/pacbio/ccs/SparsePoa.h:87-131
//   ConsensusCore::PoaConsensus::FindConsensus             ConsensusCore/include/ConsensusCore/Poa/PoaConsensus.hpp:60-97
#pragma once

#include <climits>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "ConsensusCore.hpp"

namespace ConsensusCore {

enum AlignMode { GLOBAL = PBCCS_POA_GLOBAL, SEMIGLOBAL = PBCCS_POA_SEMIGLOBAL, LOCAL = PBCCS_POA_LOCAL };

// The consensus of a POA; Graph / Path stay inside the engine (ToGraphViz on the SparsePoa gives the dump).
struct PoaConsensus {
    const std::string Sequence;
    explicit PoaConsensus(std::string s) : Sequence(std::move(s)) {}

    // PoaConsensus::FindConsensus(reads, mode, minCoverage) (PoaConsensus.cpp:86-115); caller deletes
    static const PoaConsensus* FindConsensus(const std::vector<std::string>& reads, AlignMode mode = GLOBAL,
                                             int minCoverage = -INT_MAX)
    {
        std::vector<const char*> p;
        std::vector<int> n;
        size_t total = 16;
        for (const std::string& r : reads) {
            p.push_back(r.data());
            n.push_back((int)r.size());
            total += r.size();
        }
        std::string out(total, '\0');
        int len = 0, dlen = 0;
        detail::Check(pbccs_poa_consensus(detail::DefaultEngine(), p.data(), n.data(), (int)reads.size(), mode,
                                          minCoverage, &out[0], (int)out.size(), &len, 0, nullptr, 0, &dlen));
        out.resize(len);
        return new PoaConsensus(out);
    }
};

}  // namespace ConsensusCore

namespace PacBio {
namespace CCS {

class Interval {
public:
    Interval() : left_(0), right_(0) {}
    Interval(size_t l, size_t r) : left_(l), right_(r)
    {
        if (l > r) throw std::invalid_argument("invalid Interval");
    }
    size_t Left() const { return left_; }
    size_t Right() const { return right_; }
    size_t Length() const { return right_ - left_; }
    bool Covers(const Interval& o) const { return left_ <= o.left_ && o.right_ <= right_; }
    bool operator==(const Interval& o) const { return left_ == o.left_ && right_ == o.right_; }

private:
    size_t left_, right_;
};

struct PoaAlignmentSummary {
    bool ReverseComplementedRead = false;
    Interval ExtentOnRead;
    Interval ExtentOnConsensus;
    float AlignmentScore = 0;
    float AlignmentIdentity = 0;
};

struct PoaAlignmentOptions {
    bool ClipBegin = false;
    bool ClipEnd = false;
};

class SparsePoa {
public:
    using ReadKey = int;

    SparsePoa() { ConsensusCore::detail::Check(pbccs_sparse_poa_create(ConsensusCore::detail::DefaultEngine(), &h_)); }
    ~SparsePoa() { pbccs_sparse_poa_destroy(h_); }
    SparsePoa(const SparsePoa&) = delete;
    SparsePoa& operator=(const SparsePoa&) = delete;

    ReadKey OrientAndAddRead(const std::string& readSequence, const PoaAlignmentOptions& = PoaAlignmentOptions(),
                             float minScoreToAdd = 0)
    {
        int key = -1;
        ConsensusCore::detail::Check(pbccs_sparse_poa_orient_and_add_read(h_, readSequence.data(),
                                                                          (int)readSequence.size(), minScoreToAdd,
                                                                          &key));
        if (key >= 0) ++reads_;
        bases_ += readSequence.size();
        return key;
    }

    std::shared_ptr<const ConsensusCore::PoaConsensus> FindConsensus(
        int minCoverage, std::vector<PoaAlignmentSummary>* summaries = nullptr) const
    {
        std::vector<int> rc(reads_ + 1), ext(4 * reads_ + 4);
        std::string out(bases_ + 16, '\0');
        int len = 0, nk = 0;
        ConsensusCore::detail::Check(pbccs_sparse_poa_find_consensus(h_, minCoverage, &out[0], (int)out.size(), &len,
                                                                     rc.data(), ext.data(), &nk));
        out.resize(len);
        if (summaries) {
            summaries->clear();
            for (int k = 0; k < nk; ++k) {
                PoaAlignmentSummary s;
                s.ReverseComplementedRead = rc[k] != 0;
                s.ExtentOnRead = Interval(ext[4 * k], ext[4 * k + 1]);
                s.ExtentOnConsensus = Interval(ext[4 * k + 2], ext[4 * k + 3]);
                summaries->push_back(s);
            }
        }
        return std::make_shared<const ConsensusCore::PoaConsensus>(out);
    }

    std::string ToGraphViz(int flags = 0, int minCoverage = -INT_MAX) const
    {
        int len = 0;
        if (pbccs_sparse_poa_graphviz(h_, flags, minCoverage, nullptr, 0, &len) != PBCCS_ERANGE)
            ConsensusCore::detail::Check(pbccs_sparse_poa_graphviz(h_, flags, minCoverage, nullptr, 0, &len));
        std::string out(len, '\0');
        ConsensusCore::detail::Check(pbccs_sparse_poa_graphviz(h_, flags, minCoverage, &out[0], len, &len));
        return out;
    }

private:
    pbccs_sparse_poa* h_ = nullptr;
    int reads_ = 0;
    size_t bases_ = 0;
};

}  // namespace CCS
}  // namespace PacBio
