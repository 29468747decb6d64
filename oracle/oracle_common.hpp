// oracle/oracle_common.hpp -- TEST INFRASTRUCTURE ONLY (see arrow_oracle.cpp's header).
// Mutation type, edits, enumerators and BestSubset shared by the Arrow and Quiver CPU restatements;
// each routine cites the reference file:line it follows.
#pragma once

#include <algorithm>
#include <set>
#include <string>
#include <vector>

namespace orc {

enum { INS = 0, DEL = 1, SUB = 2 };                    // CC/include/ConsensusCore/Mutation.hpp:50-53
enum { FWD = 0, REV = 1 };                             // CC/include/ConsensusCore/Read.hpp:66-70

// ------------------------------------------------------------------ mutation
struct Mut {
    int type = SUB, start = 0, end = 1;
    std::string bases = "A";
    Mut() {}
    Mut(int t, int s, int e, const std::string& nb) : type(t), start(s), end(e), bases(nb) {}
    static Mut Single(int t, int pos, char base)   // Mutation-inl.hpp (MutationType, int, char) ctor
    {
        Mut m;
        m.type = t;
        m.start = pos;
        m.end = (t == INS) ? pos : pos + 1;
        m.bases = (t == DEL) ? std::string() : std::string(1, base);
        return m;
    }
    int LengthDiff() const   // Mutation-inl.hpp LengthDiff
    {
        if (type == INS) return (int)bases.size();
        if (type == DEL) return start - end;
        return 0;
    }
    bool operator<(const Mut& o) const   // Mutation-inl.hpp:179-186
    {
        if (start != o.start) return start < o.start;
        if (end != o.end) return end < o.end;
        if (type != o.type) return type < o.type;
        return bases < o.bases;
    }
    bool operator==(const Mut& o) const
    {
        return start == o.start && end == o.end && type == o.type && bases == o.bases;
    }
};

inline char Complement(char c)
{
    switch (c) {   // CC/src/C++/Sequence.cpp:44-86
        case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C'; case 'T': return 'A';
        case 'a': return 't'; case 'c': return 'g'; case 'g': return 'c'; case 't': return 'a';
        case 'N': return 'M'; case 'M': return 'N'; case 'n': return 'm'; case 'm': return 'n';
        case '-': return '-';
    }
    return (char)127;
}

inline std::string RevComp(const std::string& s)
{
    std::string r(s.size(), ' ');
    for (size_t i = 0; i < s.size(); ++i) r[s.size() - 1 - i] = Complement(s[i]);
    return r;
}

// Mutation.cpp:60-100 (ApplyMutation(s) on a plain string).
inline void ApplyInPlace(const Mut& m, int at, std::string* t)
{
    if (m.type == SUB) t->replace(at, m.end - m.start, m.bases);
    else if (m.type == DEL) t->erase(at, m.end - m.start);
    else t->insert(at, m.bases);
}

inline std::string ApplyMuts(std::vector<Mut> muts, const std::string& tpl)
{
    std::string out(tpl);
    std::sort(muts.begin(), muts.end());
    int shift = 0;
    for (const Mut& m : muts) {
        ApplyInPlace(m, m.start + shift, &out);
        shift += m.LengthDiff();
    }
    return out;
}

// Mutation.cpp:102-140 (MutationsToTranscript) + Align/PairwiseAlignment.cpp:264-297.
inline std::vector<int> TargetToQuery(std::vector<Mut> muts, const std::string& tpl)
{
    std::sort(muts.begin(), muts.end());
    std::string tx;
    int tpos = 0;
    for (const Mut& m : muts) {
        for (; tpos < m.start; ++tpos) tx.push_back('M');
        if (m.type == INS) {
            tx += std::string(m.LengthDiff(), 'I');
        } else if (m.type == DEL) {
            tx += std::string(-m.LengthDiff(), 'D');
            tpos += -m.LengthDiff();
        } else {
            tx += std::string(m.end - m.start, 'R');
            tpos += m.end - m.start;
        }
    }
    for (; tpos < (int)tpl.size(); ++tpos) tx.push_back('M');
    std::vector<int> ntp;
    int q = 0;
    for (char c : tx) {
        if (c == 'M' || c == 'R') { ntp.push_back(q); ++q; }
        else if (c == 'D') { ntp.push_back(q); }
        else { ++q; }
    }
    ntp.push_back(q);
    return ntp;
}

// UniqueSingleBaseMutationEnumerator::Mutations (CC/src/C++/MutationEnumerator.cpp:114-145).
inline std::vector<Mut> UniqueMutations(const std::string& tpl, int b, int e)
{
    static const char kBases[4] = {'A', 'C', 'G', 'T'};
    const int L = (int)tpl.size();
    b = std::max(0, std::min(b, L));
    e = std::max(0, std::min(e, L));
    std::vector<Mut> out;
    for (int p = b; p < e; ++p) {
        const char prev = p > 0 ? tpl[p - 1] : '-';
        for (char x : kBases)
            if (x != tpl[p]) out.push_back(Mut::Single(SUB, p, x));
        for (char x : kBases)
            if (x != prev) out.push_back(Mut::Single(INS, p, x));
        if (tpl[p] != prev) out.push_back(Mut::Single(DEL, p, '-'));
    }
    return out;
}

// UniqueNearbyMutations (CC/include/ConsensusCore/MutationEnumerator-inl.hpp:50-68).
inline std::vector<Mut> NearbyMutations(const std::string& tpl, const std::vector<Mut>& centers, int nbhd)
{
    std::set<Mut> acc;
    for (const Mut& c : centers) {
        std::vector<Mut> v = UniqueMutations(tpl, c.start - nbhd, c.start + nbhd);
        acc.insert(v.begin(), v.end());
    }
    return std::vector<Mut>(acc.begin(), acc.end());
}

struct Scored { Mut m; float score; };

inline std::vector<Scored> BestSubset(std::vector<Scored> in, int sep)
{
    if (sep == 0) return in;
    std::vector<Scored> out;
    while (!in.empty()) {
        size_t best = 0;   // std::max_element: first maximum
        for (size_t k = 1; k < in.size(); ++k)
            if (in[best].score < in[k].score) best = k;
        const Scored b = in[best];
        out.push_back(b);
        const int lo = b.m.start - sep, hi = b.m.start + sep;
        std::vector<Scored> keep;
        for (const Scored& s : in)
            if (!(lo <= s.m.start && s.m.start <= hi)) keep.push_back(s);
        in.swap(keep);
    }
    return out;
}

}  // namespace orc
