// pbccs_amd/csrc/poa_graph.hpp -- the host half of the POA draft step.
//
// The partial-order graph of one ZMW lives on the host: it changes by a handful of vertices per read and
// every change is a serial walk (threading a traceback, tagging spans).  What it hands the device per read
// is a column program -- vertices in a topological order that follows chains (so a column's predecessor
// is usually the column before it), each column's predecessor columns in the reference's in-edge order,
// and the vertex bases.  The device fills the read-vs-graph DP over that program (poa_kernels.hip) and
// walks the traceback; the host replays the walk to thread the read in.
//
// Reference semantics kept (ConsensusCore/src/C++/Poa, pbccs src/SparsePoa.cpp):
//   * vertices are numbered in creation order, ^ = 0 and $ = 1 (PoaGraphImpl.cpp:106-115, .hpp:229-237);
//   * edges are a set per vertex (adjacency_list<setS, ...>): re-adding an edge is a no-op, and the graph
//     dump lists edges in insertion order (boost's global edge list);
//   * in-edges are visited in (source index) order -- PoaGraphImpl.hpp:130-143's sorted inEdges;
//   * tracebackAndThread / threadFirstRead / tagSpan / consensusPath as in PoaGraphTraversals.cpp:62-369.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

namespace pbccs {
namespace poa {

enum AlignMode { kGlobal = 0, kSemiGlobal = 1, kLocal = 2 };   // Align/AlignConfig.hpp:60-64
// PoaGraphImpl.hpp:45-55
enum Move : uint8_t { kInvalid = 0, kStart, kEnd, kMatch, kMismatch, kDelete, kExtra };

constexpr int kEnter = 0, kExit = 1;

// Traceback steps as the device reports them, one uint32 per visited cell: the vertex (low 28 bits) and
// the move that reached the cell (top 4 bits).  Step 0 is the End move into $; the walk's header gives
// the row that move comes from (LOCAL: ArgMax of the column it names) and that column's vertex.
constexpr uint32_t kStepVertexMask = 0x0FFFFFFFu;
__host__ __device__ inline uint32_t pack_step(int vertex, int move) { return ((uint32_t)move << 28) | (uint32_t)vertex; }

struct TraceHeader {
    int32_t nSteps;      // < 0: the walk failed
    int32_t endRow;      // row of the End move's source cell
    int32_t endVertex;   // vertex of the End move's source cell (tagSpan's end)
    int32_t pad;
};

// The per-read column program (device inputs).  Column 0 is always ^; $ is not a column.
struct ColumnProgram {
    std::vector<int32_t> vertexOfCol;   // column -> vertex id
    std::vector<int32_t> colOfVertex;   // vertex id -> column (-1 for $)
    std::vector<int32_t> predStart;     // CSR over columns, size cols + 1
    std::vector<int32_t> predCol;       // predecessor columns, sorted by predecessor vertex id
    std::vector<uint8_t> base;          // per column
    std::vector<int32_t> exitPredCol;   // columns of $'s predecessors, by vertex id (GLOBAL end move)
};

class PoaGraph {
public:
    struct Vertex {
        char base;
        int reads;
        int spanning;
        float score, reaching;
        int outHead, inHead;   // edge lists in the pool: out-edges by descending target, in-edges by ascending source
    };

    PoaGraph()
    {
        AddVertex('^', 0);
        AddVertex('$', 0);
    }

    size_t NumReads() const { return numReads_; }
    size_t NumVertices() const { return v_.size(); }
    const Vertex& V(int v) const { return v_[v]; }

    // threadFirstRead (PoaGraphTraversals.cpp:194-225)
    void AddFirstRead(const std::string& seq, std::vector<int>* path)
    {
        // callers never add an empty read (key -1); TagSpan(-1, ^) below would index mark[-1]
        if (seq.empty()) throw std::invalid_argument("AddFirstRead: empty read");
        if (path) path->clear();
        int prev = kEnter, first = -1;
        for (char b : seq) {
            const int v = AddVertex(b, 1);
            if (path) path->push_back(v);
            if (first < 0) first = v;
            AddEdge(prev, v);
            prev = v;
        }
        AddEdge(prev, kExit);
        TagSpan(first, prev);
        numReads_++;
    }

    // The DP's column program: a topological order from a depth-first walk out of ^ (reverse postorder,
    // as boost::topological_sort produces), which keeps a chain's vertices in consecutive columns.
    void Program(ColumnProgram* P) const
    {
        const int n = (int)v_.size();
        // scratch kept per host thread: a program is built for every read of every ZMW
        static thread_local std::vector<int> order;
        static thread_local std::vector<uint8_t> state;
        static thread_local std::vector<std::pair<int, int>> stack;   // (vertex, next out-edge)
        order.clear();
        order.reserve(n);
        state.assign(n, 0);
        stack.clear();
        stack.emplace_back(kEnter, 0);
        state[kEnter] = 1;
        // (vertex, next out-edge): successors taken largest id first, so a vertex's oldest successor -- the
        // chain it lies on -- is finished first and follows it directly in the reversed order
        stack[0].second = v_[kEnter].outHead;
        while (!stack.empty()) {
            auto& top = stack.back();
            if (top.second >= 0) {
                const int w = e_[top.second].dst;
                top.second = e_[top.second].nextOut;
                if (!state[w]) {
                    state[w] = 1;
                    stack.emplace_back(w, v_[w].outHead);
                }
            } else {
                order.push_back(top.first);
                stack.pop_back();
            }
        }
        std::reverse(order.begin(), order.end());
        P->vertexOfCol.clear();
        P->colOfVertex.assign(n, -1);
        for (int v : order)
            if (v != kExit) {
                P->colOfVertex[v] = (int)P->vertexOfCol.size();
                P->vertexOfCol.push_back(v);
            }
        const int cols = (int)P->vertexOfCol.size();
        P->predStart.assign(cols + 1, 0);
        P->predCol.clear();
        P->base.resize(cols);
        for (int c = 0; c < cols; ++c) {
            const int v = P->vertexOfCol[c];
            P->base[c] = (uint8_t)v_[v].base;
            for (int e = v_[v].inHead; e >= 0; e = e_[e].nextIn) P->predCol.push_back(P->colOfVertex[e_[e].src]);
            P->predStart[c + 1] = (int)P->predCol.size();
        }
        P->exitPredCol.clear();
        for (int e = v_[kExit].inHead; e >= 0; e = e_[e].nextIn) P->exitPredCol.push_back(P->colOfVertex[e_[e].src]);
    }

    // tracebackAndThread (PoaGraphTraversals.cpp:227-369), replaying the device's walk: steps[0] is the
    // End move into $, then one step per visited cell until (^, 0).
    void ThreadTraceback(const std::string& seq, AlignMode mode, const uint32_t* steps, const TraceHeader& h,
                         std::vector<int>* path)
    {
        const int I = (int)seq.size();
        int i = I, v = -1, fork = -1;
        const int endSpan = h.endVertex;
        if (path) path->assign(I, -1);
        for (int s = 0; s < h.nSteps; ++s) {
            const int u = (int)(steps[s] & kStepVertexMask);
            switch (steps[s] >> 28) {
                case kStart:
                    if (fork < 0) fork = v;
                    while (i > 0) fork = Fork(seq, --i, fork, path);
                    break;
                case kEnd:
                    fork = kExit;
                    if (mode == kLocal)
                        while (i > h.endRow) fork = Fork(seq, --i, fork, path);
                    break;
                case kMatch:
                    if (path) (*path)[i - 1] = u;
                    if (fork >= 0) {
                        AddEdge(u, fork);
                        fork = -1;
                    }
                    v_[u].reads++;
                    i--;
                    break;
                case kDelete:
                    if (fork < 0) fork = v;
                    break;
                case kExtra:
                case kMismatch:
                    if (fork < 0) fork = v;
                    fork = Fork(seq, --i, fork, path);
                    break;
                default:
                    throw std::runtime_error("POA traceback: invalid move");
            }
            v = u;
        }
        int startSpan = v;
        if (fork >= 0) {
            AddEdge(kEnter, fork);
            startSpan = fork;
        }
        if (startSpan != kExit) TagSpan(startSpan, endSpan);
        numReads_++;
    }

    // consensusPath (PoaGraphTraversals.cpp:115-192).  Every choice that could depend on the visiting
    // order breaks ties on vertex index, so any topological order gives the reference's path.
    std::vector<int> ConsensusPath(AlignMode mode, int minCoverage)
    {
        ColumnProgram P;
        Program(&P);
        const int total = (int)numReads_;
        std::vector<int> bestPrev(v_.size(), -1);
        v_[kEnter].reaching = 0;
        int best = -1;
        float bestScore = -FLT_MAX;
        for (size_t c = 1; c < P.vertexOfCol.size(); ++c) {
            const int v = P.vertexOfCol[c];
            Vertex& x = v_[v];
            const float score = (mode != kGlobal) ? (2 * x.reads - 1 * std::max(x.spanning, minCoverage) - 0.0001f)
                                                  : (2 * x.reads - 1 * total - 0.0001f);
            x.score = score;
            x.reaching = score;
            for (int e = x.inHead; e >= 0; e = e_[e].nextIn) {
                const int u = e_[e].src;
                const float rsc = score + v_[u].reaching;
                if (rsc > x.reaching) {
                    x.reaching = rsc;
                    bestPrev[v] = u;
                }
                if (rsc > bestScore || (rsc == bestScore && v < best)) {
                    best = v;
                    bestScore = rsc;
                }
            }
        }
        std::vector<int> path;
        for (int v = best; v >= 0; v = bestPrev[v]) path.push_back(v);
        std::reverse(path.begin(), path.end());
        return path;
    }

    std::string Sequence(const std::vector<int>& path) const
    {
        std::string s;
        s.reserve(path.size());
        for (int v : path) s.push_back(v_[v].base);
        return s;
    }

    // ToGraphViz (PoaGraphImpl.cpp:13-80, 454-462): boost write_graphviz with the vertex label writer.
    std::string GraphViz(bool color, bool verbose, const std::vector<int>* css) const
    {
        std::vector<uint8_t> in(v_.size(), 0);
        if (css)
            for (int v : *css) in[v] = 1;
        std::string s = "digraph G {\n";
        char buf[256];
        for (size_t v = 0; v < v_.size(); ++v) {
            const Vertex& x = v_[v];
            const char* fill = (color && in[v]) ? " style=\"filled\", fillcolor=\"lightblue\" ," : "";
            if (verbose)
                snprintf(buf, sizeof buf,
                         "%zu[shape=Mrecord,%s label=\"{ { %zu | %c } | { %d | %d } | { %0.2f | %0.2f } }\"];\n", v,
                         fill, v, x.base, x.reads, x.spanning, (double)x.score, (double)x.reaching);
            else
                snprintf(buf, sizeof buf, "%zu[shape=Mrecord,%s label=\"{ %c | %d }\"];\n", v, fill, x.base, x.reads);
            s += buf;
        }
        for (const Edge& e : e_) {   // edge pool index = insertion order
            snprintf(buf, sizeof buf, "%d->%d ;\n", e.src, e.dst);
            s += buf;
        }
        return s + "}\n";
    }

private:
    // Edges live in one pool (index = insertion order, which the graph dump follows) threaded into a
    // sorted singly linked out-list and in-list per vertex: a graph is a handful of contiguous arrays,
    // whatever its size, so building and freeing thousands of graphs costs no per-vertex allocations.
    struct Edge {
        int src, dst, nextOut, nextIn;
    };
    std::vector<Vertex> v_;
    std::vector<Edge> e_;
    std::vector<uint8_t> mark_;   // TagSpan scratch
    size_t numReads_ = 0;

    int AddVertex(char base, int reads)
    {
        v_.push_back(Vertex{base, reads, 0, 0.f, 0.f, -1, -1});
        return (int)v_.size() - 1;
    }

    void AddEdge(int u, int w)   // add_edge on setS: a present edge is not added again
    {
        int* link = &v_[u].outHead;   // descending targets
        while (*link >= 0 && e_[*link].dst > w) link = &e_[*link].nextOut;
        if (*link >= 0 && e_[*link].dst == w) return;
        const int id = (int)e_.size();
        e_.push_back(Edge{u, w, *link, -1});
        *link = id;
        int* in = &v_[w].inHead;      // ascending sources (PoaGraphImpl.hpp:130-143)
        while (*in >= 0 && e_[*in].src < u) in = &e_[*in].nextIn;
        e_[id].nextIn = *in;
        *in = id;
    }

    // a new vertex for read base seq[pos] in front of `fork`
    int Fork(const std::string& seq, int pos, int fork, std::vector<int>* path)
    {
        const int nv = AddVertex(seq[pos], 1);
        AddEdge(nv, fork);
        if (path) (*path)[pos] = nv;
        return nv;
    }

    // SpanningDFS + tagSpan (PoaGraphTraversals.cpp:62-113): vertices reachable from `start` that reach `end`
    void TagSpan(int start, int end)
    {
        std::vector<uint8_t>& mark = mark_;   // bit 0: reachable from start, bit 1: also reaches end
        mark.assign(v_.size(), 0);
        std::vector<int> st{start};
        while (!st.empty()) {
            const int x = st.back();
            st.pop_back();
            if (mark[x] & 1) continue;
            mark[x] |= 1;
            for (int e = v_[x].outHead; e >= 0; e = e_[e].nextOut) st.push_back(e_[e].dst);
        }
        st.push_back(end);
        while (!st.empty()) {
            const int x = st.back();
            st.pop_back();
            if (!(mark[x] & 1) || (mark[x] & 2)) continue;
            mark[x] |= 2;
            v_[x].spanning++;
            for (int e = v_[x].inHead; e >= 0; e = e_[e].nextIn) st.push_back(e_[e].src);
        }
    }
};

}  // namespace poa
}  // namespace pbccs
