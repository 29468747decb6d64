// Consensus.h's PoaConsensus step (include/pacbio/ccs/Consensus.h:352-390) written against
// include/pbccs_amd/SparsePoa.hpp the way pbccs drives its SparsePoa: reads added in order with
// OrientAndAddRead (an empty line = a read FilterReads dropped, key -1) until maxPoaCov were taken, then
// FindConsensus with the minimum-coverage rule.  Input (stdin): line 1 = maxPoaCov, then one read per
// line.  Output: the consensus, the keys, then one "rc readBegin readEnd cssBegin cssEnd" line per key.
#include <pbccs_amd/SparsePoa.hpp>

#include <iostream>
#include <string>
#include <vector>

using namespace PacBio::CCS;

int main()
{
    size_t maxPoaCov = 0;
    std::string line;
    if (!std::getline(std::cin, line)) return 2;
    maxPoaCov = std::stoul(line);
    std::vector<std::string> reads;
    while (std::getline(std::cin, line)) reads.push_back(line);

    SparsePoa poa;
    size_t cov = 0;
    std::vector<SparsePoa::ReadKey> readKeys;
    for (const std::string& r : reads) {
        const SparsePoa::ReadKey key = r.empty() ? -1 : poa.OrientAndAddRead(r);
        readKeys.emplace_back(key);
        if (key >= 0 && (++cov) >= maxPoaCov) break;
    }
    const size_t minCov = (cov < 5) ? 1 : (cov + 1) / 2 - 1;
    std::vector<PoaAlignmentSummary> summaries;
    const std::string css = poa.FindConsensus((int)minCov, &summaries)->Sequence;
    std::cout << css << "\n";
    for (size_t k = 0; k < readKeys.size(); ++k) std::cout << (k ? " " : "") << readKeys[k];
    std::cout << "\n";
    for (const PoaAlignmentSummary& s : summaries)
        std::cout << s.ReverseComplementedRead << " " << s.ExtentOnRead.Left() << " " << s.ExtentOnRead.Right() << " "
                  << s.ExtentOnConsensus.Left() << " " << s.ExtentOnConsensus.Right() << "\n";
    // ConsensusCore's own entry point agrees on a forward-only read set
    const ConsensusCore::PoaConsensus* pc = ConsensusCore::PoaConsensus::FindConsensus({"GGG", "TGGG"});
    std::cout << pc->Sequence << "\n";
    delete pc;
    return 0;
}
