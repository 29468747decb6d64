// A ConsensusCore Quiver caller written against include/pbccs_amd/Quiver.hpp only: QuiverConfigTable, a
// MultiReadMutationScorer<R> of the recursor type asked for, MappedQvRead / QvSequenceFeatures, Score / FastScore /
// ApplyMutations / BaselineScore, RefineConsensus + ConsensusQVs, and QvEvaluator.  It reads one command per line on
// stdin and answers one line each (floats as C99 hex, exact), so a test can drive the reference's gtest KATs
// through the C++ facade interactively:
//   new <sum_product> <recursor 0-3> <moves> <score_diff> <fast> <add_thr> <18 params> <tpl>
//   add <strand> <ts> <te> <threshold|nan> <seq> <ins> <subs> <del> <tag> <merge>    (tracks: a,b,... or -)
//   score <type> <pos> <base> <fast 0|1> | rsm <read> <type> <pos> <base> | baseline | template | flips
//   apply <n> (<type> <pos> <base>)... | align <read> | refine | qvs
//   moves <pin_start> <pin_end> <tpl> <seq> <ins> <subs> <del> <tag> <merge> <n> (<i> <j>)... <18 params>
// (18 params: Match Mismatch MismatchS Branch BranchS DeletionN DeletionWithTag DeletionWithTagS Nce NceS,
// Merge A C G T, MergeS A C G T)
#include <pbccs_amd/Quiver.hpp>

#include <cstdio>
#include <iostream>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

using namespace ConsensusCore;

namespace {

std::vector<float> track(const std::string& s, size_t n)
{
    std::vector<float> v;
    if (s == "-") return std::vector<float>(n, 0.0f);
    std::stringstream ss(s);
    std::string x;
    while (std::getline(ss, x, ',')) v.push_back(std::stof(x));
    return v;
}

std::string hexf(float f)
{
    char b[64];
    std::snprintf(b, sizeof(b), "%a", (double)f);
    return b;
}

template <int K>
AbstractMultiReadMutationScorer* make(bool sp, const QuiverConfigTable& t, const std::string& tpl)
{
    if (sp) return new MultiReadMutationScorer<QvRecursorType<K, true>>(t, tpl);
    return new MultiReadMutationScorer<QvRecursorType<K, false>>(t, tpl);
}

QvSequenceFeatures features(const std::string& seq, std::istream& in)
{
    std::string f[5];
    for (auto& x : f) in >> x;
    std::vector<float> tr[5];
    for (int k = 0; k < 5; ++k) tr[k] = track(f[k], seq.size());
    return QvSequenceFeatures(seq, tr[0].data(), tr[1].data(), tr[2].data(), tr[3].data(), tr[4].data());
}

Mutation mutation(std::istream& in)
{
    int t, p;
    std::string b;
    in >> t >> p >> b;
    return Mutation((MutationType)t, p, b == "-" ? 'A' : b[0]);
}

}  // namespace

int main()
{
    std::unique_ptr<AbstractMultiReadMutationScorer> s;
    std::string line;
    while (std::getline(std::cin, line)) {
        std::istringstream in(line);
        std::string cmd;
        in >> cmd;
        try {
            if (cmd == "new") {
                int sp, rec, moves;
                float sd, fast, add, p[18];
                in >> sp >> rec >> moves >> sd >> fast >> add;
                for (float& x : p) in >> x;
                std::string tpl;
                in >> tpl;
                QvModelParams qp("*", "test", p[0], p[1], p[2], p[3], p[4], p[5], p[6], p[7], p[8], p[9], p[10], p[11],
                                 p[12], p[13], p[14], p[15], p[16], p[17]);
                QuiverConfigTable table;
                table.InsertDefault(QuiverConfig(qp, moves, BandingOptions(4, sd), fast, add));
                AbstractMultiReadMutationScorer* m = nullptr;
                switch (rec) {
                    case PBCCS_QV_RECURSOR_SPARSE_SSE: m = make<PBCCS_QV_RECURSOR_SPARSE_SSE>(sp, table, tpl); break;
                    case PBCCS_QV_RECURSOR_SPARSE_SIMPLE: m = make<PBCCS_QV_RECURSOR_SPARSE_SIMPLE>(sp, table, tpl); break;
                    case PBCCS_QV_RECURSOR_DENSE_SSE: m = make<PBCCS_QV_RECURSOR_DENSE_SSE>(sp, table, tpl); break;
                    default: m = make<PBCCS_QV_RECURSOR_DENSE_SIMPLE>(sp, table, tpl); break;
                }
                s.reset(m);
                std::cout << "ok\n";
            } else if (cmd == "add") {
                int strand, ts, te;
                std::string thr, seq;
                in >> strand >> ts >> te >> thr >> seq;
                const QvSequenceFeatures f = features(seq, in);
                MappedQvRead mr(QvRead(f, "read", "*"), strand ? REVERSE_STRAND : FORWARD_STRAND, ts, te);
                const bool a = thr == "nan" ? s->AddRead(mr) : s->AddRead(mr, std::stof(thr));
                std::cout << (a ? 1 : 0) << "\n";
            } else if (cmd == "score") {
                const Mutation m = mutation(in);
                int fast = 0;
                in >> fast;
                std::cout << hexf(fast ? s->FastScore(m) : s->Score(m)) << "\n";
            } else if (cmd == "rsm") {
                int r;
                in >> r;
                const Mutation m = mutation(in);
                std::cout << hexf(s->ReadScoreMutation(r, m)) << "\n";
            } else if (cmd == "baseline") {
                std::cout << hexf(s->BaselineScore()) << "\n";
            } else if (cmd == "template") {
                std::cout << s->Template() << "\n";
            } else if (cmd == "flips") {
                for (int x : s->NumFlipFlops()) std::cout << x << " ";
                std::cout << "\n";
            } else if (cmd == "apply") {
                int n;
                in >> n;
                std::vector<Mutation> muts;
                for (int k = 0; k < n; ++k) muts.push_back(mutation(in));
                s->ApplyMutations(muts);
                std::cout << "ok\n";
            } else if (cmd == "align") {
                int r;
                in >> r;
                const auto a = s->Alignment(r);
                std::cout << a.first << " " << a.second << "\n";
            } else if (cmd == "refine") {
                size_t nt = 0, na = 0;
                const bool conv = RefineConsensus(*s, &nt, &na);
                std::cout << conv << " " << nt << " " << na << "\n";
            } else if (cmd == "qvs") {
                for (int q : ConsensusQVs(*s)) std::cout << q << " ";
                std::cout << "\n";
            } else if (cmd == "moves") {
                int ps, pe, n;
                std::string tpl, seq;
                in >> ps >> pe >> tpl >> seq;
                const QvSequenceFeatures f = features(seq, in);
                in >> n;
                std::vector<int> ci(n), cj(n);
                for (int k = 0; k < n; ++k) in >> ci[k] >> cj[k];
                float p[18];   // after the cells
                for (float& x : p) in >> x;
                const QvModelParams qp("*", "test", p[0], p[1], p[2], p[3], p[4], p[5], p[6], p[7], p[8], p[9], p[10],
                                       p[11], p[12], p[13], p[14], p[15], p[16], p[17]);
                QvEvaluator ev(QvRead(f, "read", "*"), tpl, qp, ps != 0, pe != 0);
                std::vector<float> out[4];
                ev.Moves(ci, cj, &out[0], &out[1], &out[2], &out[3]);
                for (int k = 0; k < 4; ++k)
                    for (float v : out[k]) std::cout << hexf(v) << " ";
                // single-cell forms agree with the batched one
                if (n > 0 && !(ev.Inc(ci[0], cj[0]) == out[0][0] || std::isnan(out[0][0]))) std::cout << "single-cell-mismatch";
                if (n > 0 && !(ev.Merge(ci[0], cj[0]) == out[3][0] || std::isnan(out[3][0]))) std::cout << "single-cell-mismatch";
                std::cout << "\n";
            } else if (cmd == "quit") {
                break;
            } else {
                std::cout << "error unknown command\n";
            }
        } catch (const std::exception& e) {
            std::cout << "error " << e.what() << "\n";
        }
        std::cout.flush();
    }
    return 0;
}
