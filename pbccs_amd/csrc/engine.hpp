// pbccs_amd/csrc/engine.hpp -- the batch engine behind the C ABI.
//
// ArrowBatch keeps any number of ZMWs (template + mapped reads) resident in HBM and runs the
// polishing hot path on them: read fills (AddRead / template refills), mutation-scoring rounds,
// the refine loop and QVs.  The fine-grained ConsensusCore-shaped scorer API is a batch of one ZMW;
// the ccs-style batch entry point polishes thousands of ZMWs per round trip.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <limits>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "arrow_device.hpp"
#include "arrow_kernels.hpp"
#include "arrow_model.hpp"

namespace pbccs {

struct ArrowOptions {   // ArrowConfig (ArrowConfig.hpp:104-128) + BandingOptions
    double scoreDiff = 12.5;
    double fastScoreThreshold = -12.5;
    double addThreshold = std::numeric_limits<double>::quiet_NaN();
};

struct RefineOptions {   // Consensus.hpp:48-60
    int maxIterations = 40;
    int mutationSeparation = 10;
    int mutationNeighborhood = 20;
};

enum AddReadResult { kSuccess = 0, kAlphaBetaMismatch = 1, kMemFail = 2, kPoorZScore = 3, kOther = 4 };

class DeviceError : public std::exception {
public:
    explicit DeviceError(const char* what) : what_(what) {}
    explicit DeviceError(std::string what) : what_(std::move(what)) {}
    const char* what() const noexcept override { return what_.c_str(); }
private:
    std::string what_;
};

// Device memory exhausted (hipMalloc / hipMemCreate): PBCCS_EOOM at the C ABI, so the work queue can
// retry the batch once the other slots' pools are unmapped.
class DeviceOom : public DeviceError {
public:
    explicit DeviceOom(std::string what) : DeviceError(std::move(what)) {}
};

// The stream a growing DevVec orders its copy after: the batch doing device work on this thread sets it
// (ArrowBatch::Bind).  With none set, growth synchronises the whole device (the old, conservative behaviour).
inline hipStream_t& devvec_stream()
{
    static thread_local hipStream_t s = nullptr;
    return s;
}
// Binds a stream for the scope (restoring the previous binding on exit, so nested calls and other engines'
// buffers on the same thread keep their own ordering).
struct StreamScope {
    hipStream_t prev;
    explicit StreamScope(hipStream_t s) : prev(devvec_stream()) { devvec_stream() = s; }
    ~StreamScope() { devvec_stream() = prev; }
    StreamScope(const StreamScope&) = delete;
    StreamScope& operator=(const StreamScope&) = delete;
};

// Device buffer with geometric growth (contents optionally preserved).  With a stream bound (devvec_stream) the
// growth is stream-ordered: the copy of the old contents is queued on that stream, and the old buffer -- which
// work still queued may read -- is kept until release() instead of freed at once.  Nothing synchronises the
// device: a hipDeviceSynchronize + hipFree per growth stalled every other workspace slot's work.
template <class T>
struct DevVec {
    T* ptr = nullptr;
    size_t cap = 0;
    void reserve(size_t n, bool keep)
    {
        if (n <= cap) return;
        const size_t nc = std::max(n, cap + cap / 2 + 256);
        T* p = nullptr;
        if (hipMalloc(&p, nc * sizeof(T)) != hipSuccess) {
            (void)hipGetLastError();
            size_t fr = 0, tot = 0;
            (void)hipMemGetInfo(&fr, &tot);
            throw DeviceOom("hipMalloc failed (device memory): " + std::to_string(nc * sizeof(T) >> 20) +
                              " MB requested, " + std::to_string(fr >> 20) + " MB free");
        }
        // PBCCS_DEVVEC_SYNC=1 (A/B): the old device-wide synchronising growth
        static const bool forceSync = std::getenv("PBCCS_DEVVEC_SYNC") && std::getenv("PBCCS_DEVVEC_SYNC")[0] == '1';
        const hipStream_t st = forceSync ? nullptr : devvec_stream();
        if (st) {
            if (keep && ptr && cap &&
                hipMemcpyAsync(p, ptr, cap * sizeof(T), hipMemcpyDeviceToDevice, st) != hipSuccess)
                throw DeviceError("device copy failed");
            if (ptr) {
                retired_.push_back(ptr);
                retiredCap_.push_back(cap);
            }
        } else {
            if (keep && ptr && cap) {
                if (hipDeviceSynchronize() != hipSuccess ||
                    hipMemcpy(p, ptr, cap * sizeof(T), hipMemcpyDeviceToDevice) != hipSuccess)
                    throw DeviceError("device copy failed");
            }
            if (ptr) {
                (void)hipDeviceSynchronize();
                (void)hipFree(ptr);
            }
        }
        ptr = p;
        cap = nc;
    }
    void release()
    {
        if (ptr) (void)hipFree(ptr);
        trim();
        ptr = nullptr;
        cap = 0;
    }
    // Free the buffers stream-ordered growth retired.  Only where no queued work can still read them: the caller
    // has synchronised every stream that used this buffer (a hipFree also waits for the whole device, so the
    // engine does this where the device is idle anyway: after a multi-batch call's slots joined, before an
    // out-of-memory rerun).  Returns the bytes freed.
    size_t trim()
    {
        size_t b = 0;
        for (size_t k = 0; k < retired_.size(); ++k) {
            b += retiredCap_[k] * sizeof(T);
            (void)hipFree(retired_[k]);
        }
        retired_.clear();
        retiredCap_.clear();
        return b;
    }
    size_t retired_bytes() const
    {
        size_t b = 0;
        for (size_t c : retiredCap_) b += c * sizeof(T);
        return b;
    }
    DevVec() = default;
    DevVec(const DevVec&) = delete;
    DevVec& operator=(const DevVec&) = delete;
    ~DevVec() { release(); }

private:
    std::vector<T*> retired_;   // outgrown buffers of stream-ordered growth (freed by trim / release)
    std::vector<size_t> retiredCap_;
};

// Page-locked host staging (grow-only): copies from it go to the DMA engines asynchronously, where a copy from
// pageable memory is staged by the runtime through a copy kernel that has to find room on the CUs.
struct PinnedBuf {
    char* ptr = nullptr;
    size_t cap = 0;
    void reserve(size_t n)
    {
        if (n <= cap) return;
        const size_t nc = std::max(n, cap + cap / 2 + 4096);
        char* p = nullptr;
        if (hipHostMalloc(reinterpret_cast<void**>(&p), nc, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            throw DeviceError("hipHostMalloc failed (" + std::to_string(nc >> 20) + " MB)");
        }
        // the old buffer is retired, not freed: hipHostFree waits for the whole device -- 14 s for one slot behind
        // the other slots' tall fills at configs[3] (gpurun_out/r9ze/api_gaps.json) -- and a queued copy may still
        // read it.  trim() frees the retired buffers where the device is idle (Workspace::TrimRetired).
        if (ptr) retired_.push_back(ptr);
        ptr = p;
        cap = nc;
    }
    size_t trim()
    {
        for (char* r : retired_) (void)hipHostFree(r);
        retired_.clear();
        return 0;   // host memory: not counted with the device bytes TrimRetired returns
    }
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    ~PinnedBuf()
    {
        trim();
        if (ptr) (void)hipHostFree(ptr);
    }

private:
    std::vector<char*> retired_;
};

// Band value pool: a large virtual-address reservation whose physical backing is mapped in 1 GB
// granules as the batch's bands grow (hipMemAddressReserve / hipMemCreate / hipMemMap).  Growth never
// copies and never needs old + new copies side by side, so several batches can keep tens of GB of bands
// resident each.  Falls back to DevVec growth where the virtual-memory API is unavailable.
struct VmPool {
    double* ptr = nullptr;
    size_t cap = 0;   // doubles mapped
    bool allowVmm = false;   // only long-lived engine workspaces map 1 GB granules; scorers use hipMalloc
    void reserve(size_t n, bool keep);
    // Best effort: map granules towards n doubles until the device runs out of memory (no throw).
    // Only meaningful on the VMM path (the hipMalloc fallback would have to copy): there it is a no-op.
    void try_reserve(size_t n);
    // Unmap every granule; the next reserve maps afresh at a new address range (never at addresses this pool has
    // mapped before, see unmap_all).  Synchronises.
    // s: the stream whose work last used the pool (synchronised instead of the whole device); nullptr: the device
    void unmap_all(hipStream_t s = nullptr);
    size_t mapped_bytes() const { return vmm_ ? mappedBytes_ : cap * sizeof(double); }
    size_t trim_fallback() { return fallback_.trim(); }   // the hipMalloc fallback's retired buffers (DevVec::trim)
    ~VmPool();
    VmPool() = default;
    VmPool(const VmPool&) = delete;
    VmPool& operator=(const VmPool&) = delete;
private:
    void map_to(size_t n, bool soft);
    static constexpr size_t kVaBytes = 1ull << 39;      // 512 GB of address space
    static constexpr size_t kChunkBytes = 1ull << 30;   // mapping granule
    bool tried_ = false, vmm_ = false;
    // A range mapped again while the streams that used it live on reads wrong values ("same-VA
    // remap"): every range any pool of the process has mapped is recorded (va_used_before, engine.hip), and a
    // reservation the allocator hands back as one of them is parked -- kept reserved, never mapped (address space
    // only) -- until the pool is destroyed.
    std::vector<void*> parkedVas_;
public:
    long long reusedVas_ = 0;      // reservations that returned such a range (parked, not mapped)
private:
    size_t mappedBytes_ = 0;
    std::vector<hipMemGenericAllocationHandle_t> handles_;
    std::vector<size_t> sizes_;
    DevVec<double> fallback_;
};

struct Counters {   // work counters for the roofline report (bench.py)
    long long fillCells = 0, fillLaunches = 0;
    long long scoreTasks = 0, scoreLaunches = 0;
    long long mutations = 0;
    long long bandGrowths = 0;   // fill launch sets in which some read grew its band region in-kernel
    long long relayouts = 0;     // fills that laid the band pool out afresh (ArrowBatch::Relayout)
    // band value pool of the batch, bytes (maxima over the batches merged into an engine's counters):
    // bump top (everything ever handed out), current regions (2 x capacity per read), cells in use
    long long bandTopBytes = 0, bandRegionBytes = 0, bandUsedBytes = 0;
    long long deriveNs = 0;      // DeriveZmws: the per-ZMW setup of Consensus.h:437-453 (host)
    // certified fast path: reads it filled, reads re-run exactly (an uncertain fill decision or
    // AddRead gate), ZMW rounds re-scored on exact bands (an uncertain score decision)
    long long scanReads = 0, uncertainReads = 0, exactRounds = 0;
    long long uncertainWhy[4] = {};   // uncertain fills by decision: band end, begin hint, loop entry, final mismatch
    long long fillWork[16] = {}; // PBCCS_FILL_WORK=1: CoopFill::work summed (2 kinds x kFillWorkSlots)
};

// Checkpointed-band policy: interval K (0 = off) and the shortest window it applies to;
// PBCCS_CKPT_K / PBCCS_CKPT_MIN_LEN override the defaults.
void ckpt_policy(int* K, int* minLen);

// kKFill: the 16-lane (and opt-in lane) fills of typical bands; kKFillTall: the 64-lane and lane-serial fills of
// tall bands (launched on their own streams), reported apart so each kind's launches never overlap each other
// within one workspace slot
// The Quiver family's kinds (kKQ*) are the QuiverBatch fills (four reads per wavefront, a wave per read on the side
// stream, the lane-serial fill) and its batched middle-case scoring.
enum KernelKind {
    kKFill = 0, kKSuffix, kKEnumerate, kKScore, kKReduce, kKQv, kKSelect, kKCompact, kKFillTall,
    kKQFillGrp, kKQFillCoop, kKQFillLane, kKQScoreMid, kKernelKinds
};
extern const char* const kKernelNames[kKernelKinds];

struct KernelStat {
    long long launches = 0;
    double ms = 0.0;      // summed HIP-event time on the engine stream
    double cells = 0.0;   // algorithmic DP cell-updates (in-kernel counters)
    double bytes = 0.0;   // algorithmic band bytes
    double waveTicks = 0.0;   // resident wavefront time, s_memrealtime ticks (arrow_device.hpp WaveSlot)
};

// Large device pools.  A batch either owns one (fine-grained scorers) or borrows its engine's (batch
// polish): batches polish one after another, so they stream through one resident workspace.  The workspace also
// keeps the batches' HIP streams, events and per-round scratch, so a slot that polishes one batch after another
// (the work queue, ccs chunks) allocates, frees and creates nothing in steady state: a hipFree or a stream
// destroy between batches synchronises with every other slot's work.
struct Workspace {
    explicit Workspace(bool vmm = false) { val.allowVmm = vmm; }
    ~Workspace();
    Workspace(const Workspace&) = delete;
    Workspace& operator=(const Workspace&) = delete;
    void EnsureStreams();   // creates the streams and fork/join events once
    // Free every buffer the slot's stream-ordered growth retired (DevVec::trim): call only with the slot's work
    // drained.  Returns the bytes freed (outgrown buffers otherwise stayed mapped for the engine's life).
    size_t TrimRetired();
    hipStream_t stream = nullptr, stream2 = nullptr;   // a batch's main stream; the tall fills' stream
    hipEvent_t evFork = nullptr, evJoin = nullptr;
    std::vector<hipEvent_t> eventPool;                 // timing events (profiling)
    // per-round scratch of the batch polishing on this slot
    DevVec<long long> selBase;
    DevVec<int> nSel;
    DevVec<double> colScratch;
    DevVec<unsigned long long> bump;
    PinnedBuf hDesc;
    DevVec<char> desc, seq;   // the descriptor arena and read pool of the slot's current batch (wsBuffers)
    DevVec<int2> ckPairs;
    DevVec<long long> ckStart;
    DevVec<double> rBaseline, rDev;
    DevVec<double> wDev;   // per scoring work item: the bound on its mutations' summed score deviations (certified path)
    DevVec<int> wAmb;      // per scoring work item: a decision of k_reduce lay within that bound
    DevVec<int> rFlips, rStatus, usedA, usedB, maxH;
    DevVec<int> wZmw, wNMut;
    DevVec<long long> wMutBase, wDeltaBase, wWaveStart, wMutStart, wPosStart, wPosBase, wQvBase;
    DevVec<unsigned long long> stats;
    // per-read compact bands (what scoring reads)
    DevVec<int2> aRange, bRange;
    DevVec<int> aOff, bOff;
    DevVec<double> aLs, bLs, aPre, bSuf;
    VmPool val;
    // lane-interleaved fill scratch
    DevVec<double> fVal, fLs, fPre;
    DevVec<int2> fRange;
    DevVec<int> fOff;
    // scoring rounds
    DevVec<int> codes, posOff, qv, list, edge, edgeCount;
    DevVec<double> ckSlots;                    // k_score_ckpt replay slots
    DevVec<unsigned long long> ckCounter;      // [0] task counter, [1] largest slot need
    DevVec<double> delta, score;
    DevVec<unsigned char> fav;
    DevVec<double> scratch;
    DevVec<unsigned long long> scratchTop;
    DevVec<int> scratchOverflow;
    // favourable-mutation selection (persistent: a per-round hipFree would synchronise the whole device)
    DevVec<unsigned char> xStage;   // packed transfers (download_packed / upload_packed, engine.hip)
    DevVec<long long> sel, selCount;
    DevVec<double> selScore;
    DevVec<int> selCode, selRank;
    DevVec<unsigned char> selTmp;
};

class ArrowBatch {
public:
    // ownStreams: the batch creates (and destroys) its own streams; otherwise it uses the workspace's.  The batch
    // polish passes true: with the slot's streams shared by its batches, a batch rerun after another ran the device
    // out of memory (pools unmapped and mapped again) scored wrong (tools/oom_dbg.py: 23 of 26 ZMWs; cause not
    // found -- own streams, or own per-round buffers, each made it exact), and own streams measured +2.6% at the
    // driver's command (interleaved A/B).  The fine-grained scorers keep the workspace's.
    // wsBuffers: the descriptor arena and read pool are the workspace's (a slot's batches made and polished one after
    // another: no hipMalloc / hipFree per batch -- 13.5 ms each on a busy device, 508 per ccs run); otherwise the
    // batch's own (batches made ahead, several alive per slot)
    explicit ArrowBatch(int device, Workspace* shared = nullptr, bool ownStreams = false, bool wsBuffers = false);
    ~ArrowBatch();
    ArrowBatch(const ArrowBatch&) = delete;
    ArrowBatch& operator=(const ArrowBatch&) = delete;

    // ---- host description -------------------------------------------------------------
    int AddZmw(const std::string& tpl, const double snr[4], const ArrowOptions& opt);
    // Reads are appended to the most recently added ZMW (reads of a ZMW are contiguous).
    int AppendRead(int z, const std::string& seq, int strand, int ts, int te);

    // ---- device operations ------------------------------------------------------------
    // Fill the given reads (AddRead / Template() semantics); refreshes baseline, flips, status.
    void FillReads(const std::vector<int>& reads);
    // lane-serial fallback for bands taller than the cooperative paths hold (k_fill + k_compact)
    void FillReadsSerial(const std::vector<int>& reads);
    // AddRead bookkeeping after FillReads (z-score gate, active flag).  Returns AddReadResult.
    int FinishAddRead(int r, double threshold);
    // Score explicit mutation lists (one list per ZMW); returns the summed score per mutation.
    void ScoreLists(const std::vector<int>& zmws, const std::vector<std::vector<int>>& codes, double fastThr,
                    std::vector<std::vector<double>>* scores, std::vector<std::vector<double>>* perRead = nullptr);
    // RefineConsensus for the listed ZMWs (all in lock-step rounds).
    // needFinalState = false: ZMWs that end NonConvergent may be left without the bands of their final
    // template (the batch polish never reads them).
    // qvsOnConverge != nullptr: ConsensusQVs of each ZMW in the round it converges (its bands are final then),
    // per listed ZMW (empty for the ones that do not converge); with reclaim on, their bands are then dropped.
    void Refine(const std::vector<int>& zmws, const RefineOptions& ro, std::vector<int>* converged,
                std::vector<long long>* nTested, std::vector<long long>* nApplied, bool needFinalState = true,
                std::vector<std::vector<int>>* qvsOnConverge = nullptr);
    // Band reclaim (batch polish): a fill whose list holds every read with live bands lays the value pool out
    // afresh from offset 0, each region sized from the read's last band.  Live = filled, active
    // and not retired; the caller retires the ZMWs whose bands it will not read again.
    void SetReclaim(bool on) { reclaim_ = on; }
    // The certified fast path: tall reads on the LDS-only 64-lane path fill with the reassociated
    // chain, every fill decision certified against a deviation bound (uncertain reads re-run exactly), and every
    // score decision the refine loop takes certified the same way (an uncertain ZMW round re-runs on exact bands).
    // Only for whole-batch polish: the fine-grained scorer API keeps every value the reference's bit for bit.
    void SetCertifiedScan(bool on) { scan_ = on; }
    // AddRead's z-score gate (MultiReadMutationScorer.cpp:296-318) certified: reads whose z-score lies within their
    // LL bound of `threshold` are re-filled exactly before FinishAddRead decides.
    void CertifyAddReads(const std::vector<int>& reads, double threshold);
    void Retire(const std::vector<int>& zmws);
    // ConsensusQVs for the listed ZMWs.
    void QVs(const std::vector<int>& zmws, std::vector<std::vector<int>>* qvs);
    // ApplyMutations (MultiReadMutationScorer.cpp:235-267).  Returns false on an invalid edit.
    bool ApplyMutations(int z, const std::vector<Mutation>& muts);

    // ---- host queries (MultiReadMutationScorer surface) -------------------------------
    int NumZmws() const { return (int)zmws_.size(); }
    int NumReads(int z) const { return zmws_[z].nReads; }
    int ReadIndex(int z, int k) const { return zmws_[z].readBegin + k; }
    const std::string& Template(int z) const { return zmws_[z].tpl; }
    std::string TemplateRev(int z) const { return reverse_complement(zmws_[z].tpl); }
    double ReadScore(int r) const { return reads_[r].baseline; }
    bool ReadActive(int r) const { return reads_[r].active; }
    int ReadTs(int r) const { return reads_[r].ts; }
    int ReadTe(int r) const { return reads_[r].te; }
    int ReadStrand(int r) const { return reads_[r].strand; }
    int ReadFlips(int r) const { return reads_[r].flips; }
    double BaselineScore(int z) const;
    void ZScores(int z, double* zg, double* za, std::vector<double>* zs) const;
    const ArrowOptions& Options(int z) const { return zmws_[z].opt; }
    // work counters + the band pool's current footprint (Counters::band*Bytes)
    const Counters& counters();
    void ResetCounters() { counters_ = Counters(); }
    hipStream_t stream() const { return stream_; }
    // Upload the reads and reserve the largest round's buffers (so a timed polish does no H2D of read bases).
    // The per-ZMW setup of Consensus.h:437-453 -- the ArrowConfig's transition tables and expectations, the
    // reverse-complement template, the descriptor arena -- runs at the first device operation (DeriveZmws, from
    // UploadDescriptors), i.e. inside the polish.
    void Prepare();
    void SetProfiling(bool on);
    // Resolve pending events and in-kernel counters into `out` (added), then clear.
    void CollectProfile(KernelStat out[kKernelKinds]);

private:
    struct HZmw {
        std::string tpl;
        double snr[4];
        bool derived = false;   // trans / ctx / ctxMeanVar / the template pool's copies computed (DeriveZmws)
        double ctx[45];
        TransParams trans[8];
        double ctxMeanVar[9][2];
        ArrowOptions opt;
        int readBegin = 0, nReads = 0;
        long long tplOff = 0;   // fwd at tplOff, rev at tplOff + tplCap
        int tplCap = 0;
    };
    struct HRead {
        std::string seq;
        int strand = 0, ts = 0, te = 0;
        int zmw = 0;
        bool active = false;
        bool filled = false;
        bool retired = false;   // bands no longer read (Retire): the reclaiming layout may drop them
        double baseline = 0.0;
        int flips = 0;
        int status = 0;
        int fillPath = 1;   // 0: (unused), 1: k_fill_coop<16>, 2: k_fill_coop<64> (LDS), 3: hybrid, 4: lane-serial
        long long seqOff = 0;
        long long colBase = 0;
        int colCap = 0;
        long long valA = 0, valB = 0, valCap = 0;
        long long usedA = 0, usedB = 0;   // band values the last fill kept (its region need)
        int maxH = 0;                       // the last cooperative fill's tallest column (rows)
        int ckpt = 0;   // checkpoint interval of the bands (0: every column's values kept)
        double dev = 0.0;     // bound on |LL - the reference's| of the last fill (0: exact path)
        bool exact = false;   // the certified fast path may not fill this read (an uncertain decision was met)
    };

    void EnsureZmwUploaded();
    void DeriveZmws();
    void UploadReads();
    void UploadDescriptors();
    void UploadTemplate(int z);
    void EnsureCapacity(int r);
    bool Relayout(const std::vector<int>& reads);
    DevBatch View() const;
    void TraceSummary(size_t n, int H, long long capSlots);
    void MeanVar(const HZmw& z, int strand, int ts, int te, double* mean, double* var) const;
    template <class F>
    void Timed(KernelKind k, F&& launch, hipStream_t st = nullptr);
    void ResolveEvents();
    // one scoring round on the device; codes==nullptr => device enumeration of all mutations
    void RunRound(const std::vector<int>& zmws, const std::vector<std::vector<int>>* codes, double fastThr,
                  bool needPositions, bool phased = false);

    int device_ = 0;
    std::unique_ptr<Workspace> ownWs_;
    Workspace* ws_;
    hipStream_t stream_ = nullptr;       // the workspace's streams (ws_->stream / stream2)
    bool ownStreams_ = false;            // this batch's own streams and events (the constructor's ownStreams)
    hipStream_t stream2_ = nullptr;      // second stream for the tall-band fill path
    hipEvent_t evFork_ = nullptr, evJoin_ = nullptr;
    DevVec<long long>& dSelBase_;         // phased scoring: per-item ranges of the surviving mutations
    DevVec<int>& dNSel_;
    DevVec<double>& dColScratch_;         // the hybrid fill path's column rows past its LDS buffers
    DevVec<long long> dCoopTrace_[4];     // PBCCS_FILL_PATHS=2 diagnostics: per-read fill timing, per path
    DevVec<unsigned long long> dFillWork_;   // PBCCS_FILL_WORK=1 diagnostics: CoopFill::work
    DevVec<unsigned long long>& dBump_;  // in-kernel band growth: the value pool's free top
    std::vector<HZmw> zmws_;
    std::vector<HRead> reads_;
    long long tplTop_ = 0, seqTop_ = 0, colTop_ = 0, valTop_ = 0;
    int initialBandHeight_ = 16;   // compact band values per column, first estimate
    bool descDirty_ = true;
    bool reclaim_ = false;
    size_t seqUploaded_ = 0;

    // host mirrors of pools
    std::vector<char> hTpl_, hSeq_;
    std::vector<unsigned char> hXStage_;   // host side of the packed transfers
    // device state owned by the batch (inputs + descriptors).  The per-ZMW and per-read descriptors and the
    // template pool live in one device arena, filled by one copy from a page-locked staging buffer per
    // UploadDescriptors (UploadDescriptors sets the typed views below).
    DevVec<char> ownDesc_, ownSeq_;
    DevVec<char>& dDesc_;
    DevVec<char>& dSeq_;
    PinnedBuf& hDesc_;
    int *pZFwd_ = nullptr, *pZRev_ = nullptr, *pZLen_ = nullptr, *pZReadBegin_ = nullptr, *pZNReads_ = nullptr;
    double* pZCtx_ = nullptr;
    char* pTpl_ = nullptr;
    long long *pRSeqOff_ = nullptr, *pRColBase_ = nullptr, *pRValA_ = nullptr, *pRValB_ = nullptr, *pRValCap_ = nullptr;
    int *pRLen_ = nullptr, *pRStrand_ = nullptr, *pRTs_ = nullptr, *pRTe_ = nullptr, *pRActive_ = nullptr,
        *pRZmw_ = nullptr, *pRCkpt_ = nullptr;
    DevVec<int2>& dCkPairs_;       // k_score_ckpt task list of a scoring phase
    DevVec<long long>& dCkStart_;
    // checkpointed bands: interval K for tall-path reads of windows >= ckptMinLen_; ckptAll_ (test hook
    // PBCCS_CKPT_ALL) puts every cooperative fill on checkpoints
    int ckptK_ = 0, ckptMinLen_ = 0, ckptAll_ = 0;
    long long ckSlotCap_ = 0;
    DevVec<double>& dRBaseline_;
    DevVec<double>& dRDev_;
    bool scan_ = false;
    DevVec<int>& dRFlips_, &dRStatus_, &dUsedA_, &dUsedB_, &dMaxH_;
    DevVec<int>& dWZmw_, &dWNMut_;
    DevVec<long long>& dWMutBase_, &dWDeltaBase_, &dWWaveStart_, &dWMutStart_, &dWPosStart_, &dWPosBase_,
        &dWQvBase_;
    // workspace pools (aliases into *ws_)
    DevVec<int2>& dARange_;
    DevVec<int2>& dBRange_;
    DevVec<int>& dAOff_;
    DevVec<int>& dBOff_;
    DevVec<double>& dALs_;
    DevVec<double>& dBLs_;
    DevVec<double>& dAPre_;
    DevVec<double>& dBSuf_;
    VmPool& dVal_;
    DevVec<int>& dCodes_;
    DevVec<int>& dPosOff_;
    DevVec<int>& dQv_;
    DevVec<int>& dList_;
    DevVec<int>& dEdge_;
    DevVec<int>& dEdgeCount_;
    DevVec<double>& dDelta_;
    DevVec<double>& dScore_;
    DevVec<unsigned char>& dFav_;
    DevVec<double>& dScratch_;
    DevVec<unsigned long long>& dScratchTop_;
    DevVec<int>& dScratchOverflow_;
    // last round bookkeeping (host)
    std::vector<long long> rMutStart_, rPosStart_, rDeltaBase_;
    std::vector<int> rNMut_;
    std::vector<double> rDevItem_;   // the last round's per-item score bounds (certified fast path; 0: exact)
    bool rAmbOn_ = false;            // the last round's k_reduce flagged uncertain items into ws_->wAmb
    long long rTotalMut_ = 0, rTotalPos_ = 0, rTotalDelta_ = 0;
    Counters counters_;
    // profiling
    bool profiling_ = false;
    DevVec<unsigned long long>& dStats_;
    DevVec<long long> dTrace_;   // PBCCS_FILL_TRACE diagnostics
    struct Pending {
        int kind;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending_;
    std::vector<hipEvent_t>& eventPool_;
    KernelStat stats_[kKernelKinds];
};

}  // namespace pbccs
