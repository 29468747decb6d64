// pbccs_amd/csrc/driver.hpp -- the per-ZMW driver steps of include/pacbio/ccs/Consensus.h that sit around
// the POA and the polish: FilterReads (:223-292) and ExtractMappedRead (:294-325).  Host code; the
// batched ccs entry point (pbccs_ccs_batch, capi.hip) composes them with the GPU POA and polish.
#pragma once

#include <algorithm>
#include <cstdint>
#include <string>
#include <tuple>
#include <vector>

namespace pbccs {
namespace driver {

constexpr unsigned kAdapterBefore = 1, kAdapterAfter = 2;   // pbbam LocalContextFlags

struct Subread {
    std::string seq;
    unsigned flags = kAdapterBefore | kAdapterAfter;
    bool FullPass() const { return (flags & kAdapterBefore) && (flags & kAdapterAfter); }
};

// Median (Consensus.h:213-221): the middle element, or 0.5 * (sum of the two middle ones) in double, as float
inline float Median(std::vector<size_t> v)
{
    const size_t n = v.size();
    std::sort(v.begin(), v.end());
    if (n % 2 == 1) return static_cast<float>(v[n / 2]);
    return static_cast<float>(0.5 * (v[n / 2 - 1] + v[n / 2]));
}

// FilterReads (Consensus.h:223-292): indices into `reads` in priority order -- full passes first by
// closeness of their length to the median full-pass length, then the others -- with -1 (nullptr) for reads
// of at least twice the median, sorted last.  Empty when the median is shorter than minLength.
inline std::vector<int> FilterReads(const std::vector<Subread>& reads, size_t minLength)
{
    std::vector<int> results;
    if (reads.empty()) return results;
    std::vector<size_t> lengths;
    size_t longest = 0;
    for (const Subread& r : reads) {
        longest = std::max(longest, r.seq.length());
        if (r.FullPass()) lengths.push_back(r.seq.length());
    }
    const float median = lengths.empty() ? static_cast<float>(longest) : Median(lengths);
    const size_t maxLen = 2 * static_cast<size_t>(median);
    if (median < static_cast<float>(minLength)) return results;
    for (size_t k = 0; k < reads.size(); ++k) results.push_back(reads[k].seq.length() < maxLen ? (int)k : -1);
    auto lex = [&](int k) {
        const float l = static_cast<float>(reads[k].seq.length());
        const float v = std::min(l / median, median / l);
        return reads[k].FullPass() ? std::make_tuple(v, 0.0f) : std::make_tuple(0.0f, v);
    };
    std::stable_sort(results.begin(), results.end(), [&](int a, int b) {
        if (a < 0) return false;
        if (b < 0) return true;
        return lex(a) > lex(b);
    });
    return results;
}

struct MappedRead {
    std::string seq;
    int strand = 0, ts = 0, te = 0;
};

// ExtractMappedRead (Consensus.h:294-325): the read's extent-clipped bases, mapped over the consensus
// extent.  Quirk: the substring is taken from the read as given even when the POA
// added it reverse-complemented and the extent is in the reverse complement's coordinates.
inline bool ExtractMappedRead(const Subread& read, bool rc, int readStart, int readEnd, int tplStart, int tplEnd,
                              size_t minLength, MappedRead* out)
{
    if (readStart > readEnd || (size_t)(readEnd - readStart) < minLength) return false;
    out->seq = read.seq.substr(readStart, readEnd - readStart);
    out->strand = rc ? 1 : 0;
    out->ts = tplStart;
    out->te = tplEnd;
    return true;
}

}  // namespace driver
}  // namespace pbccs
