// A pbccs-style per-ZMW driver written against include/pbccs_amd/ConsensusCore.hpp exactly the way
// include/pacbio/ccs/Consensus.h:436-512 drives ConsensusCore (scorer setup, AddRead with MinZScore,
// ZScores, RefineConsensus, ConsensusQVs, predicted accuracy).  Input (stdin):
//   line 1: <draft> <snrA> <snrC> <snrG> <snrT> <minZScore>
//   then  : <strand 0|1> <tstart> <tend> <read bases>
// Output: key=value lines.
#include <pbccs_amd/ConsensusCore.hpp>

#include <cmath>
#include <iostream>
#include <string>
#include <vector>

using namespace ConsensusCore;
using namespace ConsensusCore::Arrow;

int main()
{
    std::string draft;
    double a, c, g, t, minZ;
    if (!(std::cin >> draft >> a >> c >> g >> t >> minZ)) return 2;
    ContextParameters ctxParams(SNR(a, c, g, t));
    ArrowConfig config(ctxParams, BandingOptions(12.5));
    ArrowMultiReadMutationScorer scorer(config, draft);
    int strand, ts, te;
    std::string seq;
    std::vector<int> statusCounts(OTHER + 1, 0);
    while (std::cin >> strand >> ts >> te >> seq) {
        MappedArrowRead mr(ArrowRead(ArrowSequenceFeatures(seq), "read", "N/A"),
                           strand ? REVERSE_STRAND : FORWARD_STRAND, ts, te);
        statusCounts[scorer.AddRead(mr, minZ)] += 1;
    }
    const auto zdata = scorer.ZScores();
    size_t nTested = 0, nApplied = 0;
    const bool converged = RefineConsensus(scorer, &nTested, &nApplied);
    std::vector<int> qvs = ConsensusQVs(scorer);
    double predAcc = 0.0;
    for (int qv : qvs) predAcc += std::pow(10.0, static_cast<double>(qv) / -10.0);
    predAcc = 1.0 - predAcc / qvs.size();
    std::cout.precision(17);
    std::cout << "converged=" << converged << "\n"
              << "n_tested=" << nTested << "\nn_applied=" << nApplied << "\n"
              << "zg=" << zdata.first.first << "\nza=" << zdata.first.second << "\n"
              << "pred_acc=" << predAcc << "\n"
              << "success=" << statusCounts[SUCCESS] << "\n"
              << "consensus=" << scorer.Template() << "\n";
    return 0;
}
