// pbccs_amd/csrc/arrow_model.hpp -- host-side Arrow model and mutation bookkeeping.
//
// Cheap per-ZMW work that stays on the host CPU next to the GPU engine: the SNR -> transition
// parameter model, z-score expectations, mutation ordering/enumeration for the neighbourhood
// rounds, and real template edits with coordinate remapping.  The DP work runs on the GPU.
#pragma once

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace pbccs {

constexpr double kMismatchProbability = 0.00505052456472967;   // ArrowConfig.hpp:54 (MISMATCH_PROBABILITY)
constexpr double kMinFavorableScoreDiff = 0.04;                // MultiReadMutationScorer.cpp:56

struct TransParams {
    double match = 0.0, stick = 0.0, branch = 0.0, deletion = 0.0;
};

// ContextParameterProvider::GetTransitionParameters (ContextParameterProvider.cpp:66-110) for the
// 8 contexts; slot order AA CC GG TT NA NC NG NT.
void transition_table(const double snr[4], TransParams out[8]);
// Device layout: 9 slots x {Match, Stick, Branch, Deletion, Stick / 3.0}; slot 8 = zeros.
void device_context_table(const TransParams t[8], double out[45]);

// ExpectedContextLL (Expectations.hpp:12-40)
std::pair<double, double> expected_context_ll(const TransParams& p, double eps);

// A single-base mutation (Mutation.hpp); ordered as in Mutation-inl.hpp:179-186.
struct Mutation {
    int type = 2;    // 0 insertion, 1 deletion, 2 substitution
    int start = 0;
    int end = 1;
    char base = 'A';   // '-' for deletions
    int LengthDiff() const { return type == 0 ? 1 : (type == 1 ? -1 : 0); }
    bool operator<(const Mutation& o) const
    {
        if (start != o.start) return start < o.start;
        if (end != o.end) return end < o.end;
        if (type != o.type) return type < o.type;
        const std::string a = type == 1 ? std::string() : std::string(1, base);
        const std::string b = o.type == 1 ? std::string() : std::string(1, o.base);
        return a < b;
    }
    bool operator==(const Mutation& o) const
    {
        return type == o.type && start == o.start && end == o.end && (type == 1 || base == o.base);
    }
    static Mutation Make(int type, int pos, char base)
    {
        Mutation m;
        m.type = type;
        m.start = pos;
        m.end = type == 0 ? pos : pos + 1;
        m.base = type == 1 ? '-' : base;
        return m;
    }
};

int mutation_code(const Mutation& m);
Mutation mutation_from_code(int code);

bool is_acgt(const std::string& s);
std::string reverse_complement(const std::string& s);

// Count of UniqueSingleBaseMutationEnumerator::Mutations() for an ACGT template.
long long unique_mutation_count(const std::string& tpl);
// UniqueSingleBaseMutationEnumerator::Mutations(b, e) (MutationEnumerator.cpp:114-145), as codes.
void unique_mutations(const std::string& tpl, int b, int e, std::vector<int>* codes);
// UniqueNearbyMutations (MutationEnumerator-inl.hpp:50-68): std::set<Mutation> order, as codes.
void nearby_mutations(const std::string& tpl, const std::vector<int>& centerStarts, int nbhd,
                      std::vector<int>* codes);

// ApplyMutations (Mutation.cpp:115-128) and TargetToQueryPositions (Mutation.cpp:193-197).
// Returns false when an edit is out of range (the reference would throw).
bool apply_mutations(const std::string& tpl, std::vector<Mutation> muts, std::string* out, std::vector<int>* mtp);

// ProbabilityToQV (Consensus-inl.hpp:130-138)
int probability_to_qv(double p);

}  // namespace pbccs
