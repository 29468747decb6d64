// pbccs_amd/csrc/poa_engine.hpp -- POA draft step on the device.
//
// PoaRunner aligns reads against their ZMWs' partial-order graphs in batches: the host builds each
// graph's column program (poa_graph.hpp), k_poa_fill fills the read-vs-graph DP of every (ZMW, read
// orientation) pair at once -- one wavefront per pair -- and k_poa_trace walks the chosen orientation's
// traceback, which the host then threads into the graph.  ZmwPoa drives SparsePoa's OrientAndAddRead /
// FindConsensus (src/SparsePoa.cpp:95-201) for a whole batch of ZMWs in lock-step read rounds.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "engine.hpp"
#include "poa_graph.hpp"

namespace pbccs {
namespace poa {

constexpr int kChunkRows = 1024;   // rows per wave pass: 64 lanes x 16 rows

// One read-vs-graph alignment on the device.
struct PoaJob {
    long long scoreOff;   // element offset of the alignment's score matrix (ST units), nCols x colStride
    int nCols, colStride, I, mode;
    int progOff;          // into base[] / vertexOfCol[]  (nCols entries)
    int predStartOff;     // into predStart[]             (nCols + 1 entries, values index predCol[])
    int exitOff, nExit;   // into exitPred[]              ($'s predecessor columns, GLOBAL end move)
    long long readOff;    // into rowBase[]: byte i = read[i - 1] for rows 1..I, colStride bytes
    long long stepOff;    // into the traceback step pool (I + nCols + 2 steps)
    int traceSlot;        // this job's TraceHeader (committed jobs), else -1
    int wide;             // score matrix stored as int32 (else uint16)
    int variant;          // k_poa_fill variant (see fill_variant)
    int rowsPerLane;      // ring variants: rows per lane R; cell (column c, row i) at c * colStride + (i % R) * 64 + i / R
};

// Page-locked host staging (hipHostMalloc): the per-round program uploads and traceback downloads run at
// DMA speed, and the buffers persist across rounds.
template <class T>
struct HostVec {
    T* ptr = nullptr;
    size_t cap = 0;
    void reserve(size_t n)
    {
        if (n <= cap) return;
        const size_t nc = std::max(n, cap + cap / 2 + 1024);
        T* p = nullptr;
        if (hipHostMalloc((void**)&p, nc * sizeof(T), hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            throw DeviceOom("hipHostMalloc failed: " + std::to_string((nc * sizeof(T)) >> 20) + " MB");
        }
        if (ptr) (void)hipHostFree(ptr);
        ptr = p;
        cap = nc;
    }
    HostVec() = default;
    HostVec(const HostVec&) = delete;
    HostVec& operator=(const HostVec&) = delete;
    ~HostVec()
    {
        if (ptr) (void)hipHostFree(ptr);
    }
};

// A runner's host workers, started once: every round's column programs, staging copies and graph threading
// are spread over them (the calling thread takes indices too) instead of spawning threads per round.
class WorkerPool {
public:
    explicit WorkerPool(int threads)
    {
        for (int t = 1; t < threads; ++t) th_.emplace_back([this] { Loop(); });
    }
    ~WorkerPool()
    {
        {
            std::lock_guard<std::mutex> lk(mu_);
            quit_ = true;
        }
        cv_.notify_all();
        for (std::thread& t : th_) t.join();
    }
    WorkerPool(const WorkerPool&) = delete;
    WorkerPool& operator=(const WorkerPool&) = delete;
    int Size() const { return (int)th_.size() + 1; }
    // f(k) for k in [0, n); the first exception stops the hand-out and is rethrown here
    void Run(int n, const std::function<void(int)>& f)
    {
        if (n <= 0) return;
        if (th_.empty() || n < 2) {
            for (int k = 0; k < n; ++k) f(k);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &f;
            n_ = n;
            next_.store(0);
            err_ = nullptr;
            busy_ = (int)th_.size();
            gen_++;
        }
        cv_.notify_all();
        Work();
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return busy_ == 0; });
        job_ = nullptr;
        if (err_) std::rethrow_exception(err_);
    }

private:
    void Work()
    {
        for (int k; (k = next_.fetch_add(1)) < n_;) {
            try {
                (*job_)(k);
            } catch (...) {
                std::lock_guard<std::mutex> lk(mu_);
                if (!err_) err_ = std::current_exception();
                next_.store(n_);
            }
        }
    }
    void Loop()
    {
        long long seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return quit_ || gen_ != seen; });
                if (quit_) return;
                seen = gen_;
            }
            Work();
            std::lock_guard<std::mutex> lk(mu_);
            if (--busy_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* job_ = nullptr;
    int n_ = 0, busy_ = 0;
    std::atomic<int> next_{0};
    long long gen_ = 0;
    bool quit_ = false;
    std::exception_ptr err_;
};

struct PoaPools {
    const uint8_t* base;
    const int* vertexOfCol;
    const int* predStart;
    const int* predCol;
    const int* exitPred;
    const uint8_t* rowBase;
};

struct AlignRequest {
    PoaGraph* graph;
    std::string read;   // forward orientation as given
    AlignMode mode;
    bool orient;        // SparsePoa::OrientAndAddRead (also try the reverse complement)
    float minScore;     // minScoreToAdd
};

struct AlignResult {
    int chosen = -1;    // 0 forward, 1 reverse complement, -1 not added
    float score[2] = {0.f, 0.f};
    std::vector<int> path;   // per read position, the vertex it was threaded through
};

struct PoaStats {
    long long alignments = 0, cells = 0, launches = 0, traceSteps = 0;
    double fillMs = 0.0, traceMs = 0.0;
    double bytes = 0.0;   // algorithmic score-matrix bytes written by the fills
    // host wall time (ms): column programs + staging, device phase (uploads, kernels, downloads),
    // threading the reads into the graphs, FindConsensus
    double progMs = 0.0, deviceMs = 0.0, threadMs = 0.0, consensusMs = 0.0, totalMs = 0.0;
};

class PoaRunner {
public:
    explicit PoaRunner(int device, int hostThreads = 0);
    ~PoaRunner();
    PoaRunner(const PoaRunner&) = delete;
    PoaRunner& operator=(const PoaRunner&) = delete;

    // TryAddRead for every request (both orientations when orient), the SparsePoa choice, CommitAdd of
    // the chosen orientation.  Graphs of different requests must be distinct.
    void Align(std::vector<AlignRequest>& reqs, std::vector<AlignResult>* out);

    void SetPoolBudget(size_t bytes) { budget_ = bytes; }
    // Unmap the score-matrix pool (the address reservation stays): the polish that follows the POA in a
    // ccs run then has the device memory to itself.
    void ReleasePool() { dPool_.unmap_all(stream_); }   // only this runner's stream uses the pool
    size_t PoolMappedBytes() const { return dPool_.mapped_bytes(); }
    int HostThreads() const { return threads_; }
    void ParallelFor(int n, const std::function<void(int)>& f) { workers_->Run(n, f); }
    PoaStats stats;
    bool profiling = false;

private:
    int device_;
    int threads_;
    std::unique_ptr<WorkerPool> workers_;
    std::vector<ColumnProgram> prog_;   // per request, reused across rounds (their vectors keep their capacity)
    size_t budget_ = 0;   // cap on the score-matrix bytes per launch group (0 = 64 GB); also <= 0.6 x free HBM
    hipStream_t stream_ = nullptr;
    hipEvent_t ev_[4] = {nullptr, nullptr, nullptr, nullptr};
    DevVec<uint8_t> dBase_, dRowBase_;
    VmPool dPool_;   // score matrices: 1 GB granules mapped as rounds grow, never copied or freed between rounds
    DevVec<int> dVertexOfCol_, dPredStart_, dPredCol_, dExitPred_, dScore_, dExitCol_, dTraceJobs_;
    DevVec<PoaJob> dJobs_;
    DevVec<uint32_t> dSteps_;
    DevVec<TraceHeader> dHeads_;
    HostVec<uint8_t> hBase_, hRowBase_;
    HostVec<int> hVertex_, hPredStart_, hPredCol_, hExit_, hScore_, hExitCol_, hTraceJobs_;
    HostVec<PoaJob> hJobs_;
    HostVec<uint32_t> hSteps_;
    HostVec<TraceHeader> hHeads_;
};

// SparsePoa state of one ZMW (src/SparsePoa.cpp:60-201).
struct ZmwPoa {
    PoaGraph graph;
    std::vector<std::vector<int>> readPaths;   // per key
    std::vector<char> rc;                      // per key
    // FindConsensus (src/SparsePoa.cpp:140-201): the consensus and, per key, the read extent and
    // consensus extent (PoaAlignmentSummary); extents[4k..4k+3] = read begin, end, consensus begin, end.
    std::string FindConsensus(int minCoverage, std::vector<int>* extents, std::vector<int>* cssPath = nullptr);
};

// Consensus.h's PoaConsensus (include/pacbio/ccs/Consensus.h:352-390) over a batch of ZMWs: reads
// (nullptr = dropped by FilterReads, key -1) are added in order with OrientAndAddRead until maxCov were
// taken; keys[z][r] = key, -2 past the coverage stop.  minCov < 0: (cov < 5) ? 1 : (cov + 1) / 2 - 1.
// The ZMWs are split into one slice per runner (about equal read bases each); the slices run concurrently,
// so one slice's host work (column programs, threading) overlaps the other's kernels.
void PoaBatch(const std::vector<PoaRunner*>& runners, const std::vector<std::vector<const std::string*>>& reads,
              long long maxCov, int minCov, std::vector<std::string>* consensus, std::vector<std::vector<int>>* keys,
              std::vector<std::vector<char>>* rc, std::vector<std::vector<int>>* extents);

}  // namespace poa
}  // namespace pbccs
