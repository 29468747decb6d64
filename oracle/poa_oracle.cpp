// oracle/poa_oracle.cpp -- TEST INFRASTRUCTURE ONLY: the CPU restatement of the POA draft step that the
// tests (and bench.py's cpu_baseline leg for the POA workload) use as the checker.  The product
// (pbccs_amd/csrc/poa*.{hip,cpp}) never links or calls it; it shares no code with it.
//
// What it restates:
//   * ConsensusCore's partial-order graph: PoaGraphImpl (CC/src/C++/Poa/PoaGraphImpl.cpp:106-447,
//     PoaGraphImpl.hpp:57-298) and its traversals (PoaGraphTraversals.cpp:50-369): the
//     vertex/edge bookkeeping of a boost adjacency_list<setS, listS, bidirectionalS> (vertex index =
//     creation order, duplicate edges ignored, edges(g) in insertion order), the read-vs-graph DP
//     columns for GLOBAL / SEMIGLOBAL / LOCAL, the traceback that threads a read into the graph,
//     tagSpan, and the consensus path;
//   * PoaConsensus::FindConsensus(reads, mode, minCov) (PoaConsensus.cpp:60-115, DefaultPoaConfig
//     AlignParams(3, -5, -4, -4));
//   * pbccs's SparsePoa (src/SparsePoa.cpp:95-201): OrientAndAddRead and FindConsensus with the
//     per-read PoaAlignmentSummary extents;
//   * PoaGraphImpl::ToGraphViz in boost write_graphviz's format (PoaGraphImpl.cpp:13-80, 454-462),
//     which the reference's POA gtests compare verbatim.
// The SdpRangeFinder that SparsePoa passes to TryAddRead does not change any result: makeAlignmentColumn
// (PoaGraphImpl.cpp:236-352) ignores the beginRow/endRow it is given and fills every row, and the
// intermediate consensusPath it triggers only rewrites the Score/ReachingScore fields that FindConsensus
// rewrites again.  So this restatement fills full columns and skips the range finder.
//
// Parity pin: tests/test_poa_oracle_pins.py replays every case of the reference's own POA tests --
// CC/src/Tests/TestPoaConsensus.cpp (graph dumps, consensus sequences; GLOBAL, SEMIGLOBAL, LOCAL) and
// tests/TestSparsePoa.cpp (extents, orientation, ZMW 6251, the seeded SingleReadx100 and
// SingleAndHalfx100 cases, whose std::mt19937 streams tests/cpp/poa_kat_inputs.cpp regenerates).
#include <cfloat>
#include <climits>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "oracle_common.hpp"

namespace orc {
namespace poa {

enum Mode { GLOBAL = 0, SEMIGLOBAL = 1, LOCAL = 2 };   // CC/include/ConsensusCore/Align/AlignConfig.hpp:60-64
enum Move { InvalidMove, StartMove, EndMove, MatchMove, MismatchMove, DeleteMove, ExtraMove };  // PoaGraphImpl.hpp:45-55

struct Params { int match = 3, mismatch = -5, insert = -4, del = -4; };   // PoaConsensus.cpp DefaultPoaConfig

struct Node {                       // PoaNode (PoaGraphImpl.hpp:57-91)
    char base;
    int reads;
    int spanning = 0;
    float score = 0, reaching = 0;
};

struct Column {                     // AlignmentColumn (PoaGraphImpl.hpp:145-171), full rows
    std::vector<float> score;
    std::vector<unsigned char> move;
    std::vector<int> prev;
};

struct Matrix {                     // PoaAlignmentMatrixImpl
    std::vector<Column> cols;       // by vertex index
    std::string read;
    Mode mode;
    float score;
};

class Graph {
public:
    std::vector<Node> nodes;                         // index = vertex_index = creation order
    std::vector<std::vector<int>> outs, ins;         // setS: unique; kept sorted by vertex index
    std::vector<std::pair<int, int>> edgeList;       // edges(g): insertion order
    int enter, exit_;
    size_t numReads = 0;

    Graph()
    {
        enter = AddVertex('^', 0);
        exit_ = AddVertex('$', 0);
    }

    int AddVertex(char base, int reads = 1)          // PoaGraphImpl.hpp:229-237
    {
        nodes.push_back(Node{base, reads});
        outs.emplace_back();
        ins.emplace_back();
        return (int)nodes.size() - 1;
    }

    void AddEdge(int u, int v)                        // add_edge on setS: no duplicates
    {
        auto& o = outs[u];
        auto it = std::lower_bound(o.begin(), o.end(), v);
        if (it != o.end() && *it == v) return;
        o.insert(it, v);
        auto& in = ins[v];
        in.insert(std::lower_bound(in.begin(), in.end(), u), u);
        edgeList.emplace_back(u, v);
    }

    // boost::topological_sort (reverse DFS finish order); any topological order gives the same
    // DP values, and every order-dependent choice below breaks ties on vertex index.
    std::vector<int> TopoOrder() const
    {
        const int n = (int)nodes.size();
        std::vector<int> indeg(n), order;
        order.reserve(n);
        for (int v = 0; v < n; ++v) indeg[v] = (int)ins[v].size();
        std::vector<int> stack;
        for (int v = n - 1; v >= 0; --v)
            if (indeg[v] == 0) stack.push_back(v);
        while (!stack.empty()) {
            int v = stack.back();
            stack.pop_back();
            order.push_back(v);
            for (int w : outs[v])
                if (--indeg[w] == 0) stack.push_back(w);
        }
        return order;
    }

    // tagSpan / SpanningDFS (PoaGraphTraversals.cpp:62-113)
    void TagSpan(int start, int end)
    {
        const int n = (int)nodes.size();
        std::vector<char> fwd(n, 0), rev(n, 0);
        std::vector<int> stack{start};
        while (!stack.empty()) {
            int v = stack.back();
            stack.pop_back();
            if (fwd[v]) continue;
            fwd[v] = 1;
            for (int w : outs[v]) stack.push_back(w);
        }
        stack.push_back(end);
        while (!stack.empty()) {
            int v = stack.back();
            stack.pop_back();
            if (!fwd[v] || rev[v]) continue;
            rev[v] = 1;
            for (int u : ins[v]) stack.push_back(u);
        }
        for (int v = 0; v < n; ++v)
            if (rev[v]) nodes[v].spanning++;
    }

    // threadFirstRead (PoaGraphTraversals.cpp:194-225)
    void ThreadFirstRead(const std::string& seq, std::vector<int>* path)
    {
        int u = -1, start = -1;
        if (path) path->clear();
        for (size_t p = 0; p < seq.size(); ++p) {
            int v = AddVertex(seq[p]);
            if (path) path->push_back(v);
            if (p == 0) {
                AddEdge(enter, v);
                start = v;
            } else {
                AddEdge(u, v);
            }
            u = v;
        }
        AddEdge(u, exit_);
        TagSpan(start, u);
        numReads++;
    }

    // makeAlignmentColumn (PoaGraphImpl.cpp:236-352)
    void MakeColumn(int v, Matrix& M, const Params& P) const
    {
        const std::string& s = M.read;
        const int I = (int)s.size();
        Column& c = M.cols[v];
        c.score.assign(I + 1, -FLT_MAX);
        c.move.assign(I + 1, InvalidMove);
        c.prev.assign(I + 1, -1);
        const std::vector<int>& preds = ins[v];   // inEdges sorted by (source index, target index)
        const Node& node = nodes[v];
        if (preds.empty()) {
            c.score[0] = 0;
            c.move[0] = InvalidMove;
            c.prev[0] = -1;
        } else if (M.mode == SEMIGLOBAL || M.mode == LOCAL) {
            c.score[0] = 0;
            c.move[0] = StartMove;
            c.prev[0] = enter;
        } else {
            float best = -FLT_MAX;
            int pv = -1;
            int mv = InvalidMove;
            for (int u : preds) {
                float cand = M.cols[u].score[0] + (float)P.del;
                if (cand > best) { best = cand; pv = u; mv = DeleteMove; }
            }
            c.score[0] = best;
            c.move[0] = (unsigned char)mv;
            c.prev[0] = pv;
        }
        for (int i = 1; i <= I; ++i) {
            float best;
            int pv, mv;
            if (M.mode == LOCAL) { best = 0; pv = enter; mv = StartMove; }
            else { best = -FLT_MAX; pv = -1; mv = InvalidMove; }
            const bool isMatch = s[i - 1] == node.base;
            for (int u : preds) {
                const Column& pc = M.cols[u];
                float cand = pc.score[i - 1] + (float)(isMatch ? P.match : P.mismatch);
                if (cand > best) { best = cand; pv = u; mv = isMatch ? MatchMove : MismatchMove; }
                cand = pc.score[i] + (float)P.del;
                if (cand > best) { best = cand; pv = u; mv = DeleteMove; }
            }
            float cand = c.score[i - 1] + (float)P.insert;
            if (cand > best) { best = cand; pv = v; mv = ExtraMove; }
            c.score[i] = best;
            c.move[i] = (unsigned char)mv;
            c.prev[i] = pv;
        }
    }

    static int ArgMax(const std::vector<float>& v)     // VectorL.hpp:66-69: first maximum
    {
        return (int)(std::max_element(v.begin(), v.end()) - v.begin());
    }

    // makeAlignmentColumnForExit (PoaGraphImpl.cpp:177-233)
    void MakeExitColumn(Matrix& M) const
    {
        const int I = (int)M.read.size();
        Column& c = M.cols[exit_];
        c.score.assign(I + 1, -FLT_MAX);
        c.move.assign(I + 1, InvalidMove);
        c.prev.assign(I + 1, -1);
        float best = -FLT_MAX;
        int pv = -1;
        if (M.mode == SEMIGLOBAL || M.mode == LOCAL) {
            for (int u = 0; u < (int)nodes.size(); ++u) {      // vertices(g_): listS = creation order
                if (u == exit_) continue;
                const Column& pc = M.cols[u];
                const int row = M.mode == LOCAL ? ArgMax(pc.score) : I;
                if (pc.score[row] > best) { best = pc.score[row]; pv = u; }
            }
        } else {
            for (int u : ins[exit_]) {
                if (M.cols[u].score[I] > best) { best = M.cols[u].score[I]; pv = u; }
            }
        }
        c.score[I] = best;
        c.prev[I] = pv;
        c.move[I] = EndMove;
    }

    // TryAddRead (PoaGraphImpl.cpp:384-435), range finder skipped (see header)
    Matrix TryAddRead(const std::string& read, Mode mode, const Params& P) const
    {
        Matrix M;
        M.read = read;
        M.mode = mode;
        M.cols.resize(nodes.size());
        for (int v : TopoOrder()) {
            if (v != exit_) MakeColumn(v, M, P);
            else MakeExitColumn(M);
        }
        M.score = M.cols[exit_].score[read.size()];
        return M;
    }

    // tracebackAndThread (PoaGraphTraversals.cpp:227-369)
    void CommitAdd(const Matrix& M, std::vector<int>* path)
    {
        const std::string& seq = M.read;
        const int I = (int)seq.size();
        int i = I;
        int v = -1, fork = -1, u = exit_;
        const int endSpan = M.cols[exit_].prev[I];
        if (path) path->assign(I, -1);
        while (!(u == enter && i == 0)) {
            const Column& col = M.cols[u];
            const int prevV = col.prev[i];
            const int mv = col.move[i];
            if (mv == StartMove) {
                if (fork == -1) fork = v;
                while (i > 0) {
                    int nf = AddVertex(seq[i - 1]);
                    AddEdge(nf, fork);
                    if (path) (*path)[i - 1] = nf;
                    fork = nf;
                    i--;
                }
            } else if (mv == EndMove) {
                fork = exit_;
                if (M.mode == LOCAL) {
                    const int prevRow = ArgMax(M.cols[prevV].score);
                    while (i > prevRow) {
                        int nf = AddVertex(seq[i - 1]);
                        AddEdge(nf, fork);
                        if (path) (*path)[i - 1] = nf;
                        fork = nf;
                        i--;
                    }
                }
            } else if (mv == MatchMove) {
                if (path) (*path)[i - 1] = u;
                if (fork != -1) {
                    AddEdge(u, fork);
                    fork = -1;
                }
                nodes[u].reads++;
                i--;
            } else if (mv == DeleteMove) {
                if (fork == -1) fork = v;
            } else if (mv == ExtraMove || mv == MismatchMove) {
                int nf = AddVertex(seq[i - 1]);
                if (fork == -1) fork = v;
                AddEdge(nf, fork);
                if (path) (*path)[i - 1] = nf;
                fork = nf;
                i--;
            } else {
                throw std::runtime_error("poa traceback: invalid move");
            }
            v = u;
            u = prevV;
        }
        int startSpan = v;
        if (fork != -1) {
            AddEdge(enter, fork);
            startSpan = fork;
        }
        if (startSpan != exit_) TagSpan(startSpan, endSpan);
        numReads++;
    }

    // consensusPath (PoaGraphTraversals.cpp:115-192)
    std::vector<int> ConsensusPath(Mode mode, int minCoverage)
    {
        const int totalReads = (int)numReads;
        std::vector<int> order = TopoOrder();
        std::vector<int> bestPrev(nodes.size(), -1);
        nodes[order.front()].reaching = 0;
        int bestVertex = -1;
        float bestReaching = -FLT_MAX;
        for (size_t k = 1; k + 1 < order.size(); ++k) {
            const int v = order[k];
            Node& n = nodes[v];
            const float score = (mode != GLOBAL)
                ? (2 * n.reads - 1 * std::max(n.spanning, minCoverage) - 0.0001f)
                : (2 * n.reads - 1 * totalReads - 0.0001f);
            n.score = score;
            n.reaching = score;
            bestPrev[v] = -1;
            for (int src : ins[v]) {
                const float rsc = score + nodes[src].reaching;
                if (rsc > n.reaching) {
                    n.reaching = rsc;
                    bestPrev[v] = src;
                }
                if (rsc > bestReaching) {
                    bestVertex = v;
                    bestReaching = rsc;
                } else if (rsc == bestReaching) {
                    if (v < bestVertex) bestVertex = v;
                }
            }
        }
        std::vector<int> path;
        for (int v = bestVertex; v != -1; v = bestPrev[v]) path.push_back(v);
        std::reverse(path.begin(), path.end());
        return path;
    }

    std::string Sequence(const std::vector<int>& path) const
    {
        std::string s;
        for (int v : path) s.push_back(nodes[v].base);
        return s;
    }

    // write_graphviz with my_label_writer (PoaGraphImpl.cpp:13-80), newlines as boost writes them
    std::string GraphViz(bool color, bool verbose, const std::vector<int>* cssPath) const
    {
        std::vector<char> inCss(nodes.size(), 0);
        if (cssPath)
            for (int v : *cssPath) inCss[v] = 1;
        std::string out = "digraph G {\n";
        char buf[512];
        for (size_t v = 0; v < nodes.size(); ++v) {
            const Node& n = nodes[v];
            const char* attr = (color && inCss[v]) ? " style=\"filled\", fillcolor=\"lightblue\" ," : "";
            if (!verbose)
                snprintf(buf, sizeof buf, "%zu[shape=Mrecord,%s label=\"{ %c | %d }\"];\n", v, attr, n.base,
                         n.reads);
            else
                snprintf(buf, sizeof buf,
                         "%zu[shape=Mrecord,%s label=\"{ { %zu | %c } | { %d | %d } | { %0.2f | %0.2f } }\"];\n",
                         v, attr, v, n.base, n.reads, n.spanning, (double)n.score, (double)n.reaching);
            out += buf;
        }
        for (auto& e : edgeList) {
            snprintf(buf, sizeof buf, "%d->%d ;\n", e.first, e.second);
            out += buf;
        }
        out += "}\n";
        return out;
    }
};

// src/SparsePoa.cpp:95-201
struct SparsePoa {
    Graph g;
    std::vector<std::vector<int>> readPaths;
    std::vector<char> rc;

    int OrientAndAddRead(const std::string& seq, float minScoreToAdd = 0)
    {
        Params P;
        std::vector<int> path;
        if (g.numReads == 0) {
            g.ThreadFirstRead(seq, &path);
            readPaths.push_back(path);
            rc.push_back(0);
            return (int)g.numReads - 1;
        }
        Matrix c1 = g.TryAddRead(seq, LOCAL, P);
        Matrix c2 = g.TryAddRead(RevComp(seq), LOCAL, P);
        if (c1.score >= c2.score && c1.score >= minScoreToAdd) {
            g.CommitAdd(c1, &path);
            readPaths.push_back(path);
            rc.push_back(0);
            return (int)g.numReads - 1;
        }
        if (c2.score >= c1.score && c2.score >= minScoreToAdd) {
            g.CommitAdd(c2, &path);
            readPaths.push_back(path);
            rc.push_back(1);
            return (int)g.numReads - 1;
        }
        return -1;
    }

    // FindConsensus + the per-read summaries: extents[4*r] = readS, readE, cssS, cssE
    std::string FindConsensus(int minCoverage, std::vector<int>* extents, std::vector<int>* cssPath)
    {
        std::vector<int> path = g.ConsensusPath(LOCAL, minCoverage);
        if (cssPath) *cssPath = path;
        std::vector<int> pos(g.nodes.size(), -1);
        for (size_t i = 0; i < path.size(); ++i) pos[path[i]] = (int)i;   // std::map: last write wins
        if (extents) {
            extents->clear();
            for (size_t r = 0; r < readPaths.size(); ++r) {
                int rs = 0, re = 0, cs = 0, ce = 0;
                bool found = false;
                const std::vector<int>& rp = readPaths[r];
                for (size_t p = 0; p < rp.size(); ++p) {
                    const int v = rp[p];
                    if (pos[v] >= 0) {
                        if (!found) { cs = pos[v]; rs = (int)p; found = true; }
                        ce = pos[v] + 1;
                        re = (int)p + 1;
                    }
                }
                extents->insert(extents->end(), {rs, re, cs, ce});
            }
        }
        return g.Sequence(path);
    }
};

}  // namespace poa
}  // namespace orc

using namespace orc::poa;

static int put_string(const std::string& s, char* out, int cap)
{
    if (out && cap > 0) {
        const int n = std::min((int)s.size(), cap - 1);
        memcpy(out, s.data(), n);
        out[n] = 0;
    }
    return (int)s.size();
}

extern "C" {

// PoaConsensus::FindConsensus(reads, mode, minCoverage) (PoaConsensus.cpp:86-115): the consensus into
// seq_out and, when dot_out is given, ToGraphViz(flags) (flags: 1 = COLOR_NODES, 2 = VERBOSE_NODES; the
// colouring uses the consensus path, as ToGraphViz(flags, pc) does).  Returns the consensus length,
// -1 for an empty read (InvalidInputError).
int orc_poa_consensus(const char** reads, int n, int mode, int min_cov, char* seq_out, int seq_cap,
                      char* dot_out, int dot_cap, int flags)
{
    Graph g;
    Params P;
    for (int r = 0; r < n; ++r) {
        const std::string s(reads[r]);
        if (s.empty()) return -1;
        if (g.numReads == 0) g.ThreadFirstRead(s, nullptr);
        else g.CommitAdd(g.TryAddRead(s, (Mode)mode, P), nullptr);
    }
    std::vector<int> path = g.ConsensusPath((Mode)mode, min_cov);
    if (dot_out) put_string(g.GraphViz(flags & 1, flags & 2, &path), dot_out, dot_cap);
    return put_string(g.Sequence(path), seq_out, seq_cap);
}

// SparsePoa, as Consensus.h's PoaConsensus drives it (include/pacbio/ccs/Consensus.h:352-390): reads added
// in order with OrientAndAddRead (nullptr and empty reads get key -1) until max_cov reads were
// taken, then FindConsensus(min_cov; < 0 -> Consensus.h's (cov < 5) ? 1 : (cov + 1) / 2 - 1).
// keys[r] per input read (-2: not reached); per POA key k: rc[k], extents[4k..4k+3] = read begin/end,
// consensus begin/end.  Returns the consensus length; *n_keys = number of POA keys.
int orc_sparse_poa(const char** reads, int n, int min_cov, long max_cov, int* keys, int* n_keys, int* rc,
                   int* extents, char* seq_out, int seq_cap)
{
    SparsePoa sp;
    long cov = 0;
    for (int r = 0; r < n; ++r) keys[r] = -2;
    for (int r = 0; r < n; ++r) {
        // An empty read gets key -1, as in the engine (pbccs_poa_batch / pbccs_ccs_batch): the reference asserts a
        // non-empty read in AddFirstRead and TryAddRead (PoaGraphImpl.cpp:375,391) and threads a null vertex for an
        // empty first read in a release build, so it defines no behaviour to restate.
        const int key = (reads[r] && reads[r][0]) ? sp.OrientAndAddRead(std::string(reads[r])) : -1;
        keys[r] = key;
        if (key >= 0 && (++cov) >= max_cov) break;
    }
    if (min_cov < 0) min_cov = (cov < 5) ? 1 : (int)((cov + 1) / 2 - 1);
    std::vector<int> ext;
    const std::string css = sp.FindConsensus(min_cov, &ext, nullptr);
    *n_keys = (int)sp.readPaths.size();
    for (size_t k = 0; k < sp.readPaths.size(); ++k) {
        rc[k] = sp.rc[k];
        for (int j = 0; j < 4; ++j) extents[4 * k + j] = ext[4 * k + j];
    }
    return put_string(css, seq_out, seq_cap);
}

}  // extern "C"

#include <random>

extern "C" {

// The seeded inputs of tests/TestSparsePoa.cpp:221-293 (SingleReadx100: kind 0; SingleAndHalfx100: kind 1),
// drawn with the same std::mt19937(42) / std::uniform_int_distribution<size_t> calls in the same order, so
// the pin test replays exactly the sequences the reference test saw.  Writes the 100 first sequences
// back to back into out (lens[k] each); returns the total length, or -1 when cap is too small.
long orc_poa_kat_reads(int kind, char* out, long cap, int* lens)
{
    std::mt19937 gen(42);
    std::uniform_int_distribution<size_t> d(kind == 0 ? 2000 : 1000, kind == 0 ? 20000 : 5000);
    std::uniform_int_distribution<size_t> b(0, 3);
    const char* bases = "ACGT";
    long total = 0;
    for (int i = 0; i < 100; ++i) {
        size_t len = 0;
        while (len < 300) len = d(gen);
        if (total + (long)len > cap) return -1;
        for (size_t j = 0; j < len; ++j) out[total + j] = bases[b(gen)];
        lens[i] = (int)len;
        total += (long)len;
    }
    return total;
}

}  // extern "C"
