// pbccs_amd/csrc/engine.hip -- ArrowBatch: HBM residency + orchestration of the polishing rounds.
#include "engine.hpp"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <mutex>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <stdexcept>
#include <chrono>
#include <unordered_set>

namespace pbccs {

#define PBCCS_HIP(x)                                                         \
    do {                                                                     \
        hipError_t e_ = (x);                                                 \
        if (e_ != hipSuccess) throw DeviceError(hipGetErrorString(e_));      \
    } while (0)

const char* const kKernelNames[kKernelKinds] = {"k_fill",       "k_suffix",      "k_enumerate", "k_score",
                                                 "k_reduce",     "k_qv",          "k_best_subset", "k_compact",
                                                 "k_fill_tall",  "k_qfill_grp",   "k_qfill_coop", "k_qfill",
                                                 "k_qscore_mid"};

namespace {

constexpr int kFillBandHeight = 28;            // fill scratch values per column (doubled on overflow)
constexpr double kFillScratchBudget = 24.0 * (1ull << 30);
constexpr int kCoopNarrowRows = 64;           // LDS column rows of the 16-lane fill path
constexpr int kCoopTallRows = 1024;           // LDS column rows of the first 64-lane fill path
constexpr size_t kCoopLdsBytes = 60 * 1024;    // LDS planning budget of a fill block
// LDS column rows of the hybrid path (the rest of a column in global memory).  A tall 10 kb band is at most
// ~1500 rows; every LDS byte a wave holds beyond that only keeps other tall waves off the CU (at the 60 KB
// budget two fit a CU, at ~35 KB four).
constexpr int kHybridRows = 1536;
constexpr size_t kHeadroomMargin = 24ull << 30;   // device bytes band-growth headroom leaves free
// First region of a read that moves to the tall paths, as a fraction 1 / kTallFirstDiv of its (I+1)(J+1)
// matrix.  Exploded bands at 2 kb hold 0.8-21% of it per matrix (oracle, mean 9.9%); a read that outgrows
// its region re-runs that pass into an exact one (fill_coop.hip regrow_bands), so the first region only
// trades the memory left behind (all of it, for the reads that outgrow it) against one extra pass.
constexpr long long kTallFirstDiv = 25;
// Checkpointed bands: tall bands of long windows keep every K-th column's values only;
// the scorer replays the rest.  At 10 kb a tall read's two bands are ~0.2 GB in full.
constexpr int kCkptDefaultK = 8;
constexpr int kCkptDefaultMinLen = 4000;
constexpr int kCkptSlotsMax = 2048;   // k_score_ckpt persistent waves (2 per SIMD at its register budget)
// the replay slots' memory per scoring launch: fewer persistent waves once the slots outgrow it (a 20 kb read's
// exploded band asked 2048 slots x 2.9 MB = 5.8 GB beside full band pools: an OOM retry in configs[3])
constexpr long long kCkptSlotBytes = 1ll << 30;
int env_int(const char* name, int dflt)
{
    const char* e = std::getenv(name);
    return e ? std::atoi(e) : dflt;
}
constexpr long long kPhasedMinTasks = 1 << 21;   // (mutation, read) tasks from which a round scores in phases
constexpr size_t kInitialScratch = 1 << 20;    // doubles for whole-window refills of tiny windows
constexpr int kMaxCopySegs = 8;                // arrays per k_copy_segs launch

template <class T>
void upload(DevVec<T>& d, const std::vector<T>& h, hipStream_t s)
{
    d.reserve(std::max<size_t>(h.size(), 1), false);
    if (!h.empty()) PBCCS_HIP(hipMemcpyAsync(d.ptr, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, s));
}

// Device-to-host copy into pageable memory.  The runtime stages a pageable copy through a pinned buffer it shares
// between all streams of the device and holds that buffer until the copy has run -- i.e. until every kernel queued
// before it on its stream has finished.  Queued behind a multi-second tall fill, one slot's download stalled every
// other slot's pageable copies for seconds (configs[3]: 451 s of hipMemcpyAsync blocking over a 90 s run, 32% of
// the slots' time with none of their kernels on the device; profiles/r9b_api_gaps.json, r9a_slot_gaps.json).  So
// the stream is drained first (the caller waits for the result anyway) and the copy runs at once.
// PBCCS_D2H_DRAIN=0 (A/B): the copy queued behind the stream's work as before.
void d2h(void* dst, const void* src, size_t bytes, hipStream_t s)
{
    static const bool drain = env_int("PBCCS_D2H_DRAIN", 1) != 0;
    if (!bytes) return;
    if (drain) PBCCS_HIP(hipStreamSynchronize(s));
    PBCCS_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
}

template <class T>
void download(std::vector<T>& h, const DevVec<T>& d, size_t n, hipStream_t s)
{
    h.resize(n);
    d2h(h.data(), d.ptr, n * sizeof(T), s);
}

// Several device arrays moved in one host transfer (the runtime's pageable copies are one blit
// kernel each -- 12,401 of them in a profiled headline run -- and each device-to-host one drains the stream): the
// arrays are packed into / unpacked from a staging buffer by one k_copy_segs launch beside the single copy.
struct CopySeg {
    const unsigned int* src;
    unsigned int* dst;
    unsigned long long words;   // 4-byte words
};
struct CopySegs {
    CopySeg s[kMaxCopySegs];
};
__global__ void __launch_bounds__(256) k_copy_segs(CopySegs g)
{
    const CopySeg q = g.s[blockIdx.y];
    for (unsigned long long k = (unsigned long long)blockIdx.x * 256 + threadIdx.x; k < q.words;
         k += (unsigned long long)gridDim.x * 256)
        q.dst[k] = q.src[k];
}

// one item of a packed transfer: a device array and its host side (bytes a multiple of 4)
struct Xfer {
    void* dev;
    void* host;
    size_t bytes;
};

size_t stage_layout(const std::vector<Xfer>& items, std::vector<size_t>* off)
{
    size_t top = 0;
    off->clear();
    for (const Xfer& x : items) {
        if (x.bytes % 4) throw DeviceError("packed transfer of a size not a multiple of 4 bytes");
        off->push_back(top);
        top += (x.bytes + 15) & ~(size_t)15;
    }
    return top;
}

void launch_copy_segs(const std::vector<CopySeg>& segs, hipStream_t s)
{
    for (size_t b = 0; b < segs.size(); b += kMaxCopySegs) {
        CopySegs g{};
        const int n = (int)std::min(segs.size() - b, (size_t)kMaxCopySegs);
        unsigned long long most = 0;
        for (int k = 0; k < n; ++k) {
            g.s[k] = segs[b + k];
            most = std::max(most, segs[b + k].words);
        }
        if (!most) continue;
        const unsigned gx = (unsigned)std::min<unsigned long long>((most + 255) / 256, 1024);
        hipLaunchKernelGGL(k_copy_segs, dim3(gx, n), dim3(256), 0, s, g);
        PBCCS_HIP(hipGetLastError());
    }
}

// device arrays -> host: packed on the device, one copy, unpacked on the host (synchronises the stream)
void download_packed(const std::vector<Xfer>& items, DevVec<unsigned char>& stage, std::vector<unsigned char>& host,
                     hipStream_t s)
{
    std::vector<size_t> off;
    const size_t top = stage_layout(items, &off);
    if (!top) return;
    stage.reserve(top, false);
    std::vector<CopySeg> segs;
    for (size_t k = 0; k < items.size(); ++k)
        if (items[k].bytes)
            segs.push_back({static_cast<const unsigned int*>(items[k].dev),
                            reinterpret_cast<unsigned int*>(stage.ptr + off[k]), items[k].bytes / 4});
    launch_copy_segs(segs, s);
    host.resize(top);
    d2h(host.data(), stage.ptr, top, s);
    PBCCS_HIP(hipStreamSynchronize(s));
    for (size_t k = 0; k < items.size(); ++k)
        if (items[k].bytes) std::memcpy(items[k].host, host.data() + off[k], items[k].bytes);
}

// host arrays -> device arrays (already reserved): packed on the host, one copy, unpacked on the device
void upload_packed(const std::vector<Xfer>& items, DevVec<unsigned char>& stage, std::vector<unsigned char>& host,
                   hipStream_t s)
{
    std::vector<size_t> off;
    const size_t top = stage_layout(items, &off);
    if (!top) return;
    stage.reserve(top, false);
    host.resize(top);
    std::vector<CopySeg> segs;
    for (size_t k = 0; k < items.size(); ++k) {
        if (!items[k].bytes) continue;
        std::memcpy(host.data() + off[k], items[k].host, items[k].bytes);
        segs.push_back({reinterpret_cast<const unsigned int*>(stage.ptr + off[k]),
                        static_cast<unsigned int*>(items[k].dev), items[k].bytes / 4});
    }
    PBCCS_HIP(hipMemcpyAsync(stage.ptr, host.data(), top, hipMemcpyHostToDevice, s));
    launch_copy_segs(segs, s);
}

template <class T>
Xfer xfer_dl(std::vector<T>& h, const DevVec<T>& d, size_t n)   // n elements of d into h (resized)
{
    h.resize(n);
    return Xfer{d.ptr, h.data(), n * sizeof(T)};
}

template <class T>
Xfer xfer_ul(DevVec<T>& d, const std::vector<T>& h)   // h into d (reserved here)
{
    d.reserve(std::max<size_t>(h.size(), 1), false);
    return Xfer{d.ptr, const_cast<T*>(h.data()), h.size() * sizeof(T)};
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// VmPool
// ------------------------------------------------------------------------------------------------
// Every address range any band pool of the process has reserved for mapping: a range is never mapped twice, by
// the same pool or another (the same-VA remap, unmap_all).  Returns whether `va` is one; records it if not.
static bool va_used_before(void* va)
{
    static std::mutex mu;
    static std::vector<void*> used;
    std::lock_guard<std::mutex> lk(mu);
    if (std::find(used.begin(), used.end(), va) != used.end()) return true;
    used.push_back(va);
    return false;
}

void VmPool::try_reserve(size_t n)
{
    if (!vmm_ || n <= cap) return;
    map_to(n, true);
}

void VmPool::reserve(size_t n, bool keep)
{
    if (n <= cap) return;
    if (!tried_ && allowVmm) {
        tried_ = true;
        void* va = nullptr;
        static const bool dbgVa = env_int("PBCCS_DBG_VA", 0) != 0;   // debug: every reservation and unmap
        // a range this pool mapped before must never be mapped by it again (same-VA remap, unmap_all): a reservation
        // that returns one is parked (kept reserved, never mapped: address space only) and the next one taken
        for (int attempt = 0;; ++attempt) {
            vmm_ = hipMemAddressReserve(&va, kVaBytes, 0, nullptr, 0) == hipSuccess && va != nullptr;
            if (!vmm_) {
                (void)hipGetLastError();
                break;
            }
            if (dbgVa) std::fprintf(stderr, "[vmpool %p] reserve va=%p (%zu parked)\n", (void*)this, va, parkedVas_.size());
            if (!va_used_before(va)) break;
            reusedVas_ += 1;
            parkedVas_.push_back(va);
            if (attempt == 64) throw DeviceError("band pool: no address range this pool has not mapped before");
        }
        if (vmm_) ptr = static_cast<double*>(va);   // (recorded as used by va_used_before)
    }
    if (!vmm_) {
        fallback_.reserve(n, keep);
        ptr = fallback_.ptr;
        cap = fallback_.cap;
        return;
    }
    map_to(n, false);
}

void VmPool::map_to(size_t n, bool soft)
{
    size_t want = n * sizeof(double);
    if (want > kVaBytes) {
        if (!soft) throw DeviceError("band pool exceeds its address reservation");
        want = kVaBytes;
    }
    // Test hook: PBCCS_POOL_CAP_MB caps what one pool may map, so a batch runs out of device memory on
    // purpose and the EOOM defer/rerun paths can be checked (read on every call: tests set it at run time).
    size_t capBytes = kVaBytes;
    if (const char* e = std::getenv("PBCCS_POOL_CAP_MB")) {
        const long long mb = std::atoll(e);
        if (mb > 0) capBytes = std::min(kVaBytes, (size_t)mb << 20);
    }
    if (want > capBytes) {
        if (!soft)
            throw DeviceOom("band pool capped at " + std::to_string(capBytes >> 20) + " MB (PBCCS_POOL_CAP_MB), needs " +
                            std::to_string(want >> 20) + " MB");
        want = capBytes;
    }
    int dev = 0;
    PBCCS_HIP(hipGetDevice(&dev));
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    hipMemAccessDesc desc = {};
    desc.location = prop.location;
    desc.flags = hipMemAccessFlagsProtReadWrite;
    while (mappedBytes_ < want) {
        const size_t bytes = std::min(std::min(kChunkBytes, capBytes), kVaBytes - mappedBytes_);
        if (mappedBytes_ + bytes > capBytes) break;
        hipMemGenericAllocationHandle_t h;
        if (hipMemCreate(&h, bytes, &prop, 0) != hipSuccess) {
            (void)hipGetLastError();
            if (soft) break;
            size_t fr = 0, tot = 0;
            (void)hipMemGetInfo(&fr, &tot);
            throw DeviceOom("hipMemCreate failed (device memory): band pool at " + std::to_string(mappedBytes_ >> 30) +
                              " GB, needs " + std::to_string(want >> 30) + " GB, " + std::to_string(fr >> 20) +
                              " MB free");
        }
        char* at = reinterpret_cast<char*>(ptr) + mappedBytes_;
        if (hipMemMap(at, bytes, 0, h, 0) != hipSuccess) {
            (void)hipMemRelease(h);
            throw DeviceError("hipMemMap failed");
        }
        if (hipMemSetAccess(at, bytes, &desc, 1) != hipSuccess) {
            (void)hipMemUnmap(at, bytes);
            (void)hipMemRelease(h);
            throw DeviceError("hipMemSetAccess failed");
        }
        handles_.push_back(h);
        sizes_.push_back(bytes);
        mappedBytes_ += bytes;
    }
    cap = mappedBytes_ / sizeof(double);
    if (!soft && mappedBytes_ < want)
        throw DeviceOom("band pool capped at " + std::to_string(capBytes >> 20) + " MB (PBCCS_POOL_CAP_MB), needs " +
                        std::to_string(want >> 20) + " MB");
}

void VmPool::unmap_all(hipStream_t s)
{
    if (!vmm_) {
        if (s) (void)hipStreamSynchronize(s);
        fallback_.release();
        ptr = nullptr;
        cap = 0;
        return;
    }
    if (s) (void)hipStreamSynchronize(s);
    else (void)hipDeviceSynchronize();
    static const bool dbgVa = env_int("PBCCS_DBG_VA", 0) != 0;
    if (dbgVa) std::fprintf(stderr, "[vmpool %p] unmap_all va=%p mapped=%zu MB\n", (void*)this, (void*)ptr, mappedBytes_ >> 20);
    size_t off = 0;
    for (size_t k = 0; k < handles_.size(); ++k) {
        (void)hipMemUnmap(reinterpret_cast<char*>(ptr) + off, sizes_[k]);
        (void)hipMemRelease(handles_[k]);
        off += sizes_[k];
    }
    handles_.clear();
    sizes_.clear();
    mappedBytes_ = 0;
    cap = 0;
    // Same-VA remap: new granules mapped at an address range this pool had mapped and unmapped, with
    // the streams that used the old mapping still alive, gave wrong results -- POA drafts after a pool release,
    // and an out-of-memory rerun on slot-shared streams (its range was the one unmapped two reservations before,
    // PBCCS_DBG_VA=1 logs in profiles/r9s_same_va_oom.txt; with per-batch streams the same reuse was harmless).
    // The range is freed now -- the device memory of the unmapped granules comes back only with the range (kept
    // reserved, 600 MB per repetition stayed taken, tests/test_schedule.py::test_device_memory_does_not_grow_across_calls)
    // -- and reserve parks a reservation that returns it (va_used_before), so it is never mapped again.
    (void)hipMemAddressFree(ptr, kVaBytes);
    ptr = nullptr;
    tried_ = false;
    vmm_ = false;
}

VmPool::~VmPool()
{
    for (void* va : parkedVas_) (void)hipMemAddressFree(va, kVaBytes);
    if (!vmm_) return;
    (void)hipDeviceSynchronize();
    size_t off = 0;
    for (size_t k = 0; k < handles_.size(); ++k) {
        (void)hipMemUnmap(reinterpret_cast<char*>(ptr) + off, sizes_[k]);
        (void)hipMemRelease(handles_[k]);
        off += sizes_[k];
    }
    (void)hipMemAddressFree(ptr, kVaBytes);
}

void ckpt_policy(int* K, int* minLen)   // read per batch: tests switch it at run time
{
    *K = std::min(kCkptMaxK, std::max(0, env_int("PBCCS_CKPT_K", kCkptDefaultK)));
    *minLen = std::max(0, env_int("PBCCS_CKPT_MIN_LEN", kCkptDefaultMinLen));
}

Workspace::~Workspace()
{
    if (stream) (void)hipStreamSynchronize(stream);
    if (stream2) (void)hipStreamSynchronize(stream2);
    for (hipEvent_t e : eventPool) (void)hipEventDestroy(e);
    if (evFork) (void)hipEventDestroy(evFork);
    if (evJoin) (void)hipEventDestroy(evJoin);
    if (stream2) (void)hipStreamDestroy(stream2);
    if (stream) (void)hipStreamDestroy(stream);
}

size_t Workspace::TrimRetired()
{
    size_t b = 0;
    auto t = [&](auto& v) { b += v.trim(); };
    t(hDesc);
    t(selBase); t(nSel); t(colScratch); t(bump); t(desc); t(seq); t(ckPairs); t(ckStart); t(rBaseline); t(rFlips);
    t(rDev); t(wDev); t(wAmb);
    t(rStatus); t(usedA); t(usedB); t(maxH); t(wZmw); t(wNMut); t(wMutBase); t(wDeltaBase); t(wWaveStart);
    t(wMutStart); t(wPosStart); t(wPosBase); t(wQvBase); t(stats); t(aRange); t(bRange); t(aOff); t(bOff); t(aLs);
    t(bLs); t(aPre); t(bSuf); t(fVal); t(fLs); t(fPre); t(fRange); t(fOff); t(codes); t(posOff); t(qv); t(list);
    t(edge); t(edgeCount); t(ckSlots); t(ckCounter); t(delta); t(score); t(fav); t(scratch); t(scratchTop);
    t(scratchOverflow); t(xStage); t(sel); t(selCount); t(selScore); t(selCode); t(selRank); t(selTmp);
    b += val.trim_fallback();
    return b;
}

void Workspace::EnsureStreams()
{
    if (stream) return;
    PBCCS_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    PBCCS_HIP(hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking));
    PBCCS_HIP(hipEventCreateWithFlags(&evFork, hipEventDisableTiming));
    PBCCS_HIP(hipEventCreateWithFlags(&evJoin, hipEventDisableTiming));
}

ArrowBatch::ArrowBatch(int device, Workspace* shared, bool ownStreams, bool wsBuffers)
    : device_(device),
      ownWs_(shared ? nullptr : new Workspace()),
      ws_(shared ? shared : ownWs_.get()),
      dSelBase_(ws_->selBase), dNSel_(ws_->nSel), dColScratch_(ws_->colScratch), dBump_(ws_->bump),
      hDesc_(ws_->hDesc), dCkPairs_(ws_->ckPairs), dCkStart_(ws_->ckStart), dRBaseline_(ws_->rBaseline),
      dRDev_(ws_->rDev),
      dRFlips_(ws_->rFlips), dRStatus_(ws_->rStatus), dUsedA_(ws_->usedA), dUsedB_(ws_->usedB), dMaxH_(ws_->maxH),
      dWZmw_(ws_->wZmw), dWNMut_(ws_->wNMut), dWMutBase_(ws_->wMutBase), dWDeltaBase_(ws_->wDeltaBase),
      dWWaveStart_(ws_->wWaveStart), dWMutStart_(ws_->wMutStart), dWPosStart_(ws_->wPosStart),
      dWPosBase_(ws_->wPosBase), dWQvBase_(ws_->wQvBase),
      dARange_(ws_->aRange), dBRange_(ws_->bRange), dAOff_(ws_->aOff), dBOff_(ws_->bOff), dALs_(ws_->aLs),
      dBLs_(ws_->bLs), dAPre_(ws_->aPre), dBSuf_(ws_->bSuf), dVal_(ws_->val), dCodes_(ws_->codes),
      dPosOff_(ws_->posOff), dQv_(ws_->qv), dList_(ws_->list), dEdge_(ws_->edge), dEdgeCount_(ws_->edgeCount),
      dDelta_(ws_->delta), dScore_(ws_->score), dFav_(ws_->fav), dScratch_(ws_->scratch),
      dScratchTop_(ws_->scratchTop), dScratchOverflow_(ws_->scratchOverflow), dStats_(ws_->stats),
      eventPool_(ws_->eventPool), dDesc_(wsBuffers && shared ? ws_->desc : ownDesc_),
      dSeq_(wsBuffers && shared ? ws_->seq : ownSeq_)
{
    PBCCS_HIP(hipSetDevice(device_));
    // first value-region estimate per read (PBCCS_INITIAL_BAND_HEIGHT overrides it: tests use a tiny one
    // to force in-kernel band growth on every read)
    if (const char* e = std::getenv("PBCCS_INITIAL_BAND_HEIGHT")) initialBandHeight_ = std::max(1, std::atoi(e));
    ckpt_policy(&ckptK_, &ckptMinLen_);
    ckptAll_ = std::min(kCkptMaxK, std::max(0, env_int("PBCCS_CKPT_ALL", 0)));
    if (ownStreams) {
        ownStreams_ = true;
        PBCCS_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
        // PBCCS_ONE_STREAM=1 (A/B): the tall fills queue behind the 16-lane fill on the batch's one stream, so twice
        // the slots fit the hardware queues
        static const bool oneStream = env_int("PBCCS_ONE_STREAM", 0) != 0;
        if (oneStream) stream2_ = stream_;
        else PBCCS_HIP(hipStreamCreateWithFlags(&stream2_, hipStreamNonBlocking));
        PBCCS_HIP(hipEventCreateWithFlags(&evFork_, hipEventDisableTiming));
        PBCCS_HIP(hipEventCreateWithFlags(&evJoin_, hipEventDisableTiming));
    } else {
        ws_->EnsureStreams();
        stream_ = ws_->stream;
        stream2_ = ws_->stream2;
        evFork_ = ws_->evFork;
        evJoin_ = ws_->evJoin;
    }
    const StreamScope bound(stream_);   // stream-ordered DevVec growth for this batch's calls (engine.hpp)
    // PBCCS_DBG_CLEAR=1 (debug): the workspace's per-round scratch zeroed at every batch's start (does a batch
    // depend on what the slot's previous batch left there?)
    if (shared && std::getenv("PBCCS_DBG_CLEAR") && std::getenv("PBCCS_DBG_CLEAR")[0] == '1') {
        PBCCS_HIP(hipDeviceSynchronize());
        auto z = [](auto& v) {
            if (v.ptr) PBCCS_HIP(hipMemset(v.ptr, 0, v.cap * sizeof(*v.ptr)));
        };
        Workspace& w = *ws_;
        z(w.selBase); z(w.nSel); z(w.colScratch); z(w.bump); z(w.ckPairs); z(w.ckStart); z(w.rBaseline);
        z(w.rFlips); z(w.rStatus); z(w.usedA); z(w.usedB); z(w.maxH); z(w.wZmw); z(w.wNMut); z(w.wMutBase);
        z(w.wDeltaBase); z(w.wWaveStart); z(w.wMutStart); z(w.wPosStart); z(w.wPosBase); z(w.wQvBase); z(w.stats);
        if (w.hDesc.ptr) std::memset(w.hDesc.ptr, 0, w.hDesc.cap);
        PBCCS_HIP(hipDeviceSynchronize());
    }
    dScratch_.reserve(kInitialScratch, false);
    dScratchTop_.reserve(1, false);
    // the read pool starts with 16 bytes of padding (see UploadDescriptors: word loads of read bases)
    hSeq_.assign(16, '\0');
    seqTop_ = 16;
    dScratchOverflow_.reserve(1, false);
}

ArrowBatch::~ArrowBatch()
{
    // the streams and events belong to the workspace (the slot's next batch reuses them): wait, do not destroy
    if (stream_) {
        (void)hipStreamSynchronize(stream_);
        (void)hipStreamSynchronize(stream2_);
        for (const Pending& p : pending_) {
            eventPool_.push_back(p.a);
            eventPool_.push_back(p.b);
        }
        if (ownStreams_) {
            (void)hipEventDestroy(evFork_);
            (void)hipEventDestroy(evJoin_);
            if (stream2_ != stream_) (void)hipStreamDestroy(stream2_);
            (void)hipStreamDestroy(stream_);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// profiling: HIP events around every launch on the engine stream + in-kernel algorithmic counters
// ------------------------------------------------------------------------------------------------
void ArrowBatch::SetProfiling(bool on)
{
    const StreamScope bound(stream_);
    profiling_ = on;
    if (on) {
        dStats_.reserve(16, false);
        PBCCS_HIP(hipMemsetAsync(dStats_.ptr, 0, 16 * sizeof(unsigned long long), stream_));
    }
}

template <class F>
void ArrowBatch::Timed(KernelKind k, F&& launch, hipStream_t st)
{
    if (!st) st = stream_;
    // PBCCS_DBG_SYNC=1 (debug): every launch waits for both of the batch's streams to drain (no two device
    // operations of a batch overlap, and nothing is left queued when the host goes on)
    static const bool dbgSync = std::getenv("PBCCS_DBG_SYNC") && std::getenv("PBCCS_DBG_SYNC")[0] == '1';
    if (!profiling_) {
        launch();
        if (dbgSync) {
            PBCCS_HIP(hipStreamSynchronize(stream_));
            PBCCS_HIP(hipStreamSynchronize(stream2_));
        }
        return;
    }
    hipEvent_t ev[2];
    for (int i = 0; i < 2; ++i) {
        if (!eventPool_.empty()) {
            ev[i] = eventPool_.back();
            eventPool_.pop_back();
        } else {
            PBCCS_HIP(hipEventCreate(&ev[i]));
        }
    }
    PBCCS_HIP(hipEventRecord(ev[0], st));
    launch();
    PBCCS_HIP(hipEventRecord(ev[1], st));
    pending_.push_back({(int)k, ev[0], ev[1]});
    stats_[k].launches += 1;
}

void ArrowBatch::ResolveEvents()
{
    if (pending_.empty()) return;
    // events sit on both streams (the tall fills run on stream2_); a batch that failed after
    // the fork may not have joined them back into stream_, so wait for each
    PBCCS_HIP(hipStreamSynchronize(stream_));
    PBCCS_HIP(hipStreamSynchronize(stream2_));
    for (const Pending& p : pending_) {
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) stats_[p.kind].ms += ms;
        else (void)hipGetLastError();   // a launch that never ran (failed batch): no time to add
        eventPool_.push_back(p.a);
        eventPool_.push_back(p.b);
    }
    pending_.clear();
}

const Counters& ArrowBatch::counters()
{
    const StreamScope bound(stream_);
    if (dFillWork_.ptr) {   // PBCCS_FILL_WORK diagnostics: fold the device counters in and clear them
        unsigned long long h[16];
        d2h(h, dFillWork_.ptr, sizeof(h), stream_);
        PBCCS_HIP(hipMemsetAsync(dFillWork_.ptr, 0, sizeof(h), stream_));
        PBCCS_HIP(hipStreamSynchronize(stream_));
        for (int k = 0; k < 16; ++k) counters_.fillWork[k] += (long long)h[k];
    }
    long long region = 0, used = 0;
    for (const HRead& r : reads_) {
        region += 2 * r.valCap;
        used += r.usedA + r.usedB;
    }
    counters_.bandTopBytes = std::max(counters_.bandTopBytes, valTop_ * (long long)sizeof(double));
    counters_.bandRegionBytes = std::max(counters_.bandRegionBytes, region * (long long)sizeof(double));
    counters_.bandUsedBytes = std::max(counters_.bandUsedBytes, used * (long long)sizeof(double));
    return counters_;
}

void ArrowBatch::CollectProfile(KernelStat out[kKernelKinds])
{
    const StreamScope bound(stream_);
    ResolveEvents();
    if (profiling_) {
        unsigned long long h[16];
        d2h(h, dStats_.ptr, sizeof(h), stream_);
        PBCCS_HIP(hipStreamSynchronize(stream_));
        stats_[kKFill].cells += (double)h[2 * kStatFill];
        stats_[kKFill].bytes += (double)h[2 * kStatFill + 1];
        stats_[kKFillTall].cells += (double)h[2 * kStatFillTall];
        stats_[kKFillTall].bytes += (double)h[2 * kStatFillTall + 1];
        stats_[kKScore].cells += (double)h[2 * kStatScore];
        stats_[kKScore].bytes += (double)h[2 * kStatScore + 1];
        stats_[kKFill].waveTicks += (double)h[kWaveFill];
        stats_[kKFillTall].waveTicks += (double)h[kWaveFillTall];
        stats_[kKScore].waveTicks += (double)h[kWaveScore];   // k_score (its edge / checkpoint kernels do not stamp)
        stats_[kKSuffix].waveTicks += (double)h[kWaveSuffix];
        stats_[kKReduce].waveTicks += (double)h[kWaveReduce];
        static const bool trace = std::getenv("PBCCS_ROUND_TRACE") != nullptr;
        if (trace) std::fprintf(stderr, "[fillcells] g16=%llu g64=%llu\n", h[8], h[9]);
        PBCCS_HIP(hipMemsetAsync(dStats_.ptr, 0, sizeof(h), stream_));
    }
    for (int k = 0; k < kKernelKinds; ++k) {
        out[k].launches += stats_[k].launches;
        out[k].ms += stats_[k].ms;
        out[k].cells += stats_[k].cells;
        out[k].bytes += stats_[k].bytes;
        out[k].waveTicks += stats_[k].waveTicks;
        stats_[k] = KernelStat();
    }
}

void ArrowBatch::Prepare()
{
    const StreamScope bound(stream_);
    // the workspace may hold another (finished) batch's bands: size it without preserving them
    const size_t cols = std::max<long long>(colTop_, 1);
    dARange_.reserve(cols, false);
    dBRange_.reserve(cols, false);
    dAOff_.reserve(cols, false);
    dBOff_.reserve(cols, false);
    dALs_.reserve(cols, false);
    dBLs_.reserve(cols, false);
    dAPre_.reserve(cols, false);
    dBSuf_.reserve(cols, false);
    dVal_.reserve(std::max<long long>(valTop_, 1), false);
    UploadReads();
    long long mut = 0, delta = 0, pos = 0;
    for (const HZmw& z : zmws_) {
        const long long M = unique_mutation_count(z.tpl) + 64;
        mut += M;
        delta += M * z.nReads;
        pos += (long long)z.tpl.size() + 65;
    }
    dCodes_.reserve(std::max<long long>(mut, 1), false);
    dScore_.reserve(std::max<long long>(mut, 1), false);
    dFav_.reserve(std::max<long long>(mut, 1), false);
    dDelta_.reserve(std::max<long long>(delta, 1), false);
    dPosOff_.reserve(std::max<long long>(pos, 1), false);
    dQv_.reserve(std::max<long long>(pos, 1), false);
    ws_->sel.reserve(std::max<long long>(mut, 1), false);
    ws_->selScore.reserve(std::max<long long>(mut, 1), false);
    ws_->selCode.reserve(std::max<long long>(mut, 1), false);
    ws_->selRank.reserve(std::max<long long>(mut, 1), false);
    ws_->selCount.reserve(2, false);
    {   // hipCUB temp storage of the refine rounds' selections (a later growth would synchronise the device)
        size_t a = 0, b = 0, c = 0;
        const int nm = (int)std::min<long long>(std::max<long long>(mut, 1), INT_MAX);
        hipcub::CountingInputIterator<long long> it(0);
        PBCCS_HIP(hipcub::DeviceSelect::Flagged(nullptr, a, it, dFav_.ptr, ws_->sel.ptr, ws_->selCount.ptr, nm, stream_));
        PBCCS_HIP(hipcub::DeviceSelect::Flagged(nullptr, b, dScore_.ptr, dFav_.ptr, ws_->selScore.ptr,
                                                ws_->selCount.ptr + 1, nm, stream_));
        PBCCS_HIP(hipcub::DeviceSelect::Flagged(nullptr, c, dCodes_.ptr, dFav_.ptr, ws_->selCode.ptr,
                                                ws_->selCount.ptr + 1, nm, stream_));
        ws_->selTmp.reserve(std::max<size_t>(std::max(a, std::max(b, c)), 1), false);
    }
    PBCCS_HIP(hipStreamSynchronize(stream_));
}

// ------------------------------------------------------------------------------------------------
// host description
// ------------------------------------------------------------------------------------------------
int ArrowBatch::AddZmw(const std::string& tpl, const double snr[4], const ArrowOptions& opt)
{
    if (tpl.empty() || !is_acgt(tpl)) throw std::invalid_argument("template must be a non-empty ACGT string");
    if (!(opt.scoreDiff >= 0.0)) throw std::invalid_argument("ScoreDiff must be positive!");   // ArrowConfig.hpp:72-77
    HZmw z;
    z.tpl = tpl;
    for (int k = 0; k < 4; ++k) z.snr[k] = snr[k];
    z.opt = opt;
    z.readBegin = (int)reads_.size();
    z.nReads = 0;
    const int L = (int)tpl.size();
    z.tplCap = L + L / 4 + 64;
    z.tplOff = tplTop_;
    tplTop_ += 2LL * z.tplCap;
    zmws_.push_back(z);
    descDirty_ = true;
    return (int)zmws_.size() - 1;
}

// Consensus.h:437-453 per ZMW: ArrowConfig(ContextParameters(snr)) -- the transition table of every context, its
// device form and the context expectations of the z-score gate -- and the scorer's forward / reverse-complement
// template pair.  Runs once per ZMW, at the first device operation after AddZmw.
void ArrowBatch::DeriveZmws()
{
    const auto t0 = std::chrono::steady_clock::now();
    bool any = false;
    for (size_t zi = 0; zi < zmws_.size(); ++zi) {
        HZmw& z = zmws_[zi];
        if (z.derived) continue;
        transition_table(z.snr, z.trans);
        device_context_table(z.trans, z.ctx);
        for (int k = 0; k < 9; ++k) {
            const std::pair<double, double> mv = expected_context_ll(k < 8 ? z.trans[k] : TransParams(), kMismatchProbability);
            z.ctxMeanVar[k][0] = mv.first;
            z.ctxMeanVar[k][1] = mv.second;
        }
        z.derived = true;
        UploadTemplate((int)zi);
        any = true;
    }
    if (any)
        counters_.deriveNs += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
}

int ArrowBatch::AppendRead(int z, const std::string& seq, int strand, int ts, int te)
{
    if (z != (int)zmws_.size() - 1) throw std::invalid_argument("reads must be appended to the latest ZMW");
    const int L = (int)zmws_[z].tpl.size();
    if (ts < 0 || te > L || ts > te) throw std::invalid_argument("read window outside the template");
    HRead r;
    r.seq = seq;
    r.strand = strand;
    r.ts = ts;
    r.te = te;
    r.zmw = z;
    r.seqOff = seqTop_;
    seqTop_ += (long long)seq.size() + 1;
    hSeq_.insert(hSeq_.end(), seq.begin(), seq.end());
    hSeq_.push_back('\0');
    const int J = te - ts;
    r.colCap = J + J / 4 + 66;
    r.colBase = colTop_;
    colTop_ += r.colCap;
    r.valCap = (long long)(J + 66) * initialBandHeight_;   // regrown exactly by the fill if outgrown
    r.valA = valTop_;
    r.valB = valTop_ + r.valCap;
    valTop_ += 2 * r.valCap;
    reads_.push_back(r);
    zmws_[z].nReads += 1;
    descDirty_ = true;
    return (int)reads_.size() - 1;
}

void ArrowBatch::UploadTemplate(int zi)
{
    HZmw& z = zmws_[zi];
    const int L = (int)z.tpl.size();
    if (L > z.tplCap) {
        z.tplCap = L + L / 4 + 64;
        z.tplOff = tplTop_;
        tplTop_ += 2LL * z.tplCap;
        descDirty_ = true;
    }
    if ((long long)hTpl_.size() < tplTop_) hTpl_.resize(tplTop_);
    std::memcpy(&hTpl_[z.tplOff], z.tpl.data(), L);
    const std::string rc = reverse_complement(z.tpl);
    std::memcpy(&hTpl_[z.tplOff + z.tplCap], rc.data(), L);
    descDirty_ = true;
}

void ArrowBatch::EnsureCapacity(int ri)
{
    HRead& r = reads_[ri];
    const int J = r.te - r.ts;
    if (J + 2 > r.colCap) {
        r.colCap = J + J / 4 + 66;
        r.colBase = colTop_;
        colTop_ += r.colCap;
        if ((long long)r.colCap * initialBandHeight_ > r.valCap) {
            r.valCap = (long long)r.colCap * initialBandHeight_;
            r.valA = valTop_;
            r.valB = valTop_ + r.valCap;
            valTop_ += 2 * r.valCap;
        }
        descDirty_ = true;
    }
    if (r.valCap == 0) {   // its region was dropped by a reclaiming layout (Relayout)
        r.valCap = (long long)r.colCap * initialBandHeight_;
        r.valA = valTop_;
        r.valB = valTop_ + r.valCap;
        valTop_ += 2 * r.valCap;
        descDirty_ = true;
    }
}

void ArrowBatch::Retire(const std::vector<int>& zl)
{
    for (int zi : zl) {
        const HZmw& z = zmws_[zi];
        for (int k = 0; k < z.nReads; ++k) reads_[z.readBegin + k].retired = true;
    }
}

// Reclaiming layout (reclaim_ only): when every read whose bands are still live is about to be refilled,
// nothing in the value pool is needed any more, so the regions are handed out afresh from offset 0 in list
// order instead of bumping the pool's top.  A region is sized from the read's last fill (its larger matrix
// + 1/8 + 64: refills follow a template that moved by a few bases); a read never filled keeps the first
// estimate of its path.  Regions of reads outside the list are dropped (valCap 0; EnsureCapacity gives
// one back if such a read is ever filled again).  Without this the pool's top only grows: regions abandoned
// by growth and by moves to the tall paths were never reused (43.6 GB top against 18.2 GB of bands in use
// for a 2000-ZMW batch, profiles/r2h1_bench.json).
bool ArrowBatch::Relayout(const std::vector<int>& list)
{
    if (!reclaim_ || !ws_->val.allowVmm) return false;
    std::vector<char> in(reads_.size(), 0);
    for (int r : list) in[r] = 1;
    for (size_t r = 0; r < reads_.size(); ++r) {
        const HRead& h = reads_[r];
        if (h.filled && h.active && !h.retired && !in[r]) return false;   // live bands outside the list
    }
    for (HRead& h : reads_) {
        h.valCap = 0;
        h.valA = h.valB = 0;
    }
    valTop_ = 0;
    for (int r : list) {
        HRead& h = reads_[r];
        const long long m = std::max(h.usedA, h.usedB);
        long long cap;
        if (h.filled && m > 0) cap = m + m / 8 + 64;
        else if (h.fillPath == 2 || h.fillPath == 3)
            cap = ((long long)h.seq.size() + 1) * (h.te - h.ts + 1) / kTallFirstDiv / std::max(1, h.ckpt) + 64;
        else cap = (long long)h.colCap * initialBandHeight_;
        h.valCap = cap;
        h.valA = valTop_;
        h.valB = valTop_ + cap;
        valTop_ += 2 * cap;
    }
    for (size_t r = 0; r < reads_.size(); ++r)
        if (!in[r]) reads_[r].usedA = reads_[r].usedB = 0;   // dropped: no bands held
    descDirty_ = true;
    counters_.relayouts += 1;
    return true;
}

void ArrowBatch::UploadReads()
{
    // 32 bytes of slack at the end: the lane fill loads read bases 8 at a time (two aligned words), and
    // its prefetch of the rows past a band may reach 24 bytes beyond a read
    dSeq_.reserve(hSeq_.size() + 32, true);
    if (hSeq_.size() > seqUploaded_) {
        PBCCS_HIP(hipMemcpyAsync(dSeq_.ptr + seqUploaded_, hSeq_.data() + seqUploaded_, hSeq_.size() - seqUploaded_,
                                 hipMemcpyHostToDevice, stream_));
        seqUploaded_ = hSeq_.size();
    }
}

void ArrowBatch::UploadDescriptors()
{
    const StreamScope bound(stream_);
    DeriveZmws();
    if (!descDirty_) return;
    const int Z = (int)zmws_.size(), R = (int)reads_.size();
    std::vector<int> zf(Z), zr(Z), zl(Z), zb(Z), zn(Z);
    std::vector<double> zc((size_t)Z * 45);
    for (int i = 0; i < Z; ++i) {
        const HZmw& z = zmws_[i];
        zf[i] = (int)z.tplOff;
        zr[i] = (int)(z.tplOff + z.tplCap);
        zl[i] = (int)z.tpl.size();
        zb[i] = z.readBegin;
        zn[i] = z.nReads;
        std::memcpy(&zc[(size_t)i * 45], z.ctx, sizeof(z.ctx));
    }
    std::vector<long long> so(R), cb(R), va(R), vb(R), vc(R);
    std::vector<int> rl(R), rs(R), rts(R), rte(R), ra(R), rz(R), rck(R);
    for (int i = 0; i < R; ++i) {
        const HRead& r = reads_[i];
        so[i] = r.seqOff;
        cb[i] = r.colBase;
        va[i] = r.valA;
        vb[i] = r.valB;
        vc[i] = r.valCap;
        rl[i] = (int)r.seq.size();
        rs[i] = r.strand;
        rts[i] = r.ts;
        rte[i] = r.te;
        ra[i] = r.active ? 1 : 0;
        rz[i] = r.zmw;
        rck[i] = r.ckpt;
    }
    // one arena: every array at a 256-byte aligned offset, packed into page-locked staging, one copy
    size_t top = 0;
    auto place = [&](size_t bytes) {
        const size_t at = top;
        top += (bytes + 255) & ~(size_t)255;
        return at;
    };
    const size_t oZf = place(Z * sizeof(int)), oZr = place(Z * sizeof(int)), oZl = place(Z * sizeof(int)),
                 oZb = place(Z * sizeof(int)), oZn = place(Z * sizeof(int)), oZc = place(zc.size() * sizeof(double));
    const size_t oSo = place(R * sizeof(long long)), oCb = place(R * sizeof(long long)),
                 oVa = place(R * sizeof(long long)), oVb = place(R * sizeof(long long)),
                 oVc = place(R * sizeof(long long));
    const size_t oRl = place(R * sizeof(int)), oRs = place(R * sizeof(int)), oRts = place(R * sizeof(int)),
                 oRte = place(R * sizeof(int)), oRa = place(R * sizeof(int)), oRz = place(R * sizeof(int)),
                 oRck = place(R * sizeof(int));
    const size_t oTpl = place(hTpl_.size() + 32);   // (32 bytes of slack past the last template)
    hDesc_.reserve(std::max<size_t>(top, 1));
    auto put = [&](size_t at, const void* src, size_t bytes) {
        if (bytes) std::memcpy(hDesc_.ptr + at, src, bytes);
    };
    put(oZf, zf.data(), Z * sizeof(int));
    put(oZr, zr.data(), Z * sizeof(int));
    put(oZl, zl.data(), Z * sizeof(int));
    put(oZb, zb.data(), Z * sizeof(int));
    put(oZn, zn.data(), Z * sizeof(int));
    put(oZc, zc.data(), zc.size() * sizeof(double));
    put(oSo, so.data(), R * sizeof(long long));
    put(oCb, cb.data(), R * sizeof(long long));
    put(oVa, va.data(), R * sizeof(long long));
    put(oVb, vb.data(), R * sizeof(long long));
    put(oVc, vc.data(), R * sizeof(long long));
    put(oRl, rl.data(), R * sizeof(int));
    put(oRs, rs.data(), R * sizeof(int));
    put(oRts, rts.data(), R * sizeof(int));
    put(oRte, rte.data(), R * sizeof(int));
    put(oRa, ra.data(), R * sizeof(int));
    put(oRz, rz.data(), R * sizeof(int));
    put(oRck, rck.data(), R * sizeof(int));
    put(oTpl, hTpl_.data(), hTpl_.size());
    dDesc_.reserve(std::max<size_t>(top, 1), false);
    PBCCS_HIP(hipMemcpyAsync(dDesc_.ptr, hDesc_.ptr, top, hipMemcpyHostToDevice, stream_));
    char* base = dDesc_.ptr;
    pZFwd_ = reinterpret_cast<int*>(base + oZf);
    pZRev_ = reinterpret_cast<int*>(base + oZr);
    pZLen_ = reinterpret_cast<int*>(base + oZl);
    pZReadBegin_ = reinterpret_cast<int*>(base + oZb);
    pZNReads_ = reinterpret_cast<int*>(base + oZn);
    pZCtx_ = reinterpret_cast<double*>(base + oZc);
    pRSeqOff_ = reinterpret_cast<long long*>(base + oSo);
    pRColBase_ = reinterpret_cast<long long*>(base + oCb);
    pRValA_ = reinterpret_cast<long long*>(base + oVa);
    pRValB_ = reinterpret_cast<long long*>(base + oVb);
    pRValCap_ = reinterpret_cast<long long*>(base + oVc);
    pRLen_ = reinterpret_cast<int*>(base + oRl);
    pRStrand_ = reinterpret_cast<int*>(base + oRs);
    pRTs_ = reinterpret_cast<int*>(base + oRts);
    pRTe_ = reinterpret_cast<int*>(base + oRte);
    pRActive_ = reinterpret_cast<int*>(base + oRa);
    pRZmw_ = reinterpret_cast<int*>(base + oRz);
    pRCkpt_ = reinterpret_cast<int*>(base + oRck);
    pTpl_ = base + oTpl;
    UploadReads();
    const size_t cols = std::max<long long>(colTop_, 1);
    dARange_.reserve(cols, true);
    dBRange_.reserve(cols, true);
    dAOff_.reserve(cols, true);
    dBOff_.reserve(cols, true);
    dALs_.reserve(cols, true);
    dBLs_.reserve(cols, true);
    dAPre_.reserve(cols, true);
    dBSuf_.reserve(cols, true);
    dVal_.reserve(std::max<long long>(valTop_, 1), true);
    dRBaseline_.reserve(std::max(R, 1), true);
    dRDev_.reserve(std::max(R, 1), true);
    dRFlips_.reserve(std::max(R, 1), true);
    dRStatus_.reserve(std::max(R, 1), true);
    PBCCS_HIP(hipStreamSynchronize(stream_));   // host vectors above are temporaries
    descDirty_ = false;
}

DevBatch ArrowBatch::View() const
{
    DevBatch b;
    b.zFwdOff = pZFwd_;
    b.zRevOff = pZRev_;
    b.zLen = pZLen_;
    b.zCtx = pZCtx_;
    b.zReadBegin = pZReadBegin_;
    b.zNReads = pZNReads_;
    b.tplPool = pTpl_;
    b.rSeqOff = pRSeqOff_;
    b.rLen = pRLen_;
    b.rStrand = pRStrand_;
    b.rTs = pRTs_;
    b.rTe = pRTe_;
    b.rActive = pRActive_;
    b.rZmw = pRZmw_;
    b.rColBase = pRColBase_;
    b.rValA = pRValA_;
    b.rValB = pRValB_;
    b.rValCap = pRValCap_;
    b.rCkpt = pRCkpt_;
    b.seqPool = dSeq_.ptr;
    b.aRange = dARange_.ptr;
    b.aOff = dAOff_.ptr;
    b.aLs = dALs_.ptr;
    b.aPre = dAPre_.ptr;
    b.bRange = dBRange_.ptr;
    b.bOff = dBOff_.ptr;
    b.bLs = dBLs_.ptr;
    b.bSuf = dBSuf_.ptr;
    b.valPool = dVal_.ptr;
    b.rBaseline = dRBaseline_.ptr;
    b.rDev = dRDev_.ptr;
    b.rFlips = dRFlips_.ptr;
    b.rStatus = dRStatus_.ptr;
    b.prNot = 1.0 - kMismatchProbability;
    b.prThird = kMismatchProbability / 3.0;
    b.sdn = zmws_.empty() ? std::exp(12.5) : std::exp(zmws_[0].opt.scoreDiff);
    b.stats = profiling_ ? dStats_.ptr : nullptr;
    return b;
}

// ------------------------------------------------------------------------------------------------
// fills
// ------------------------------------------------------------------------------------------------
// Cooperative fills (fill_coop.hip): reads start on the 16-lane path; a read whose band outgrows the
// LDS column buffer moves to the 64-lane path, then to the lane-serial fallback (the path is
// remembered for its refills).  Value-capacity overflow moves the read to a region of the exact size
// the kernel reported.  Bands land directly in the compact layout; k_suffix adds the log-scale sums.
void ArrowBatch::FillReads(const std::vector<int>& readsIn)
{
    const StreamScope bound(stream_);
    // Cooperative paths (fill_coop.hip): 1: 16 lanes / 64 rows; 2: 64 lanes / 1024 rows, LDS only; 3: 64 lanes,
    // as many rows as LDS holds and the rest of a column in global memory (the hybrid path: never too tall, so a
    // fill re-routes a read at most twice).  Reads whose bases do not fit LDS beside 64 rows go to the
    // lane-serial k_fill (FillReadsSerial).  Path 0 was a one-lane-per-read fill with an LDS ring per lane
    // (fill_lane.hip, removed in round 3): ~2x fewer VALU instructions, but a single lane's serial loop per read
    // -- measured 2937 / 3006 ZMWs/s against 3403 / 3465 without it under the round-3 wave sorting
    // (profiles/r3m_*; round 2: profiles/r2_lane_fill_ab.txt).
    constexpr int kPaths = 4;
    for (int r : readsIn) EnsureCapacity(r);
    // a read moves from path p to the tall paths: long windows skip the 1024-row LDS path (their tall bands
    // mostly outgrow it -- 10 kb: 662 of 786 reads went on to the hybrid path -- and each step is one more
    // launch on the round's critical path); it gets a first tall region now (kTallFirstDiv): growing from the
    // typical 16-row region inside the kernel would copy and abandon two or three.  Returns the new path.
    auto promote = [&](int r, int p) {
        HRead& h = reads_[r];
        int q = p + 1;
        if (q == 2 && (long long)h.seq.size() + 1 > 4LL * kCoopTallRows) q = 3;
        h.fillPath = q;
        if (q >= 2 && q < kPaths) {
            const long long I = (long long)h.seq.size(), J = h.te - h.ts;
            // checkpointed: every K-th column plus the kept tails (the next launch sets h.ckpt)
            const bool ck = ckptAll_ > 0 || (ckptK_ > 0 && J >= ckptMinLen_);
            const long long K = ck ? std::max(ckptAll_, ckptK_) : 1;
            const long long want = (I + 1) * (J + 1) / kTallFirstDiv / K + (ck ? 2 * (kCkptTail + 1) * (I + 1) : 0) + 64;
            if (want > h.valCap) {
                h.valCap = want;
                h.valA = valTop_;
                h.valB = valTop_ + h.valCap;
                valTop_ += 2 * h.valCap;
                descDirty_ = true;
            }
        }
        return q;
    };
    Relayout(readsIn);
    std::vector<int> todo[kPaths], serial, done;
    for (int r : readsIn) {
        const int p = reads_[r].fillPath;
        if (p >= kPaths) serial.push_back(r);
        else todo[p].push_back(r);
    }
    auto words = [&](int r) {
        return (int)(reads_[r].seq.size() + 7) / 8 + (reads_[r].te - reads_[r].ts + 8) / 8;
    };
    // rows a column buffer of path p gets for reads with these sizes (0: does not fit in LDS)
    // Tall bands run on 64 lanes (one read per wavefront).  16-lane groups for them (4x fewer VALU issue
    // slots per chain step) measured 1290 against 2480 ZMWs/s and were removed: the tall reads are each
    // round's critical path and 16-row chunks pay the per-chunk band logic 4x as often.
    // Tall paths: one read per wavefront, rows per lane PBCCS_TALL_ROWS (1 / 2, A/B; 4 measured slowest in every
    // A/B, profiles/r4c_tall_rows_ab.txt, and was removed); a column buffer holds whole chunks of 64 x rows rows.
    constexpr int tallG = 64;
    static const int tallRows = env_int("PBCCS_TALL_ROWS", kTallRowsPerLane) == 1 ? 1 : 2;
    const long long chunk = (long long)tallG * tallRows;
    const long long tallGroupLds = (long long)kCoopLdsBytes;
    auto full_rows = [&](int maxI) { return ((long long)maxI + chunk) / chunk * chunk; };   // >= I + 1 rows
    // Narrow path: 16 lanes per read (four reads per wavefront), one row per lane.  Two rows per lane and sixteen
    // reads per wavefront (4 lanes x 4 rows, bases from global memory) measured slower and were removed
    // (profiles/r4i_narrow_rows_ab.txt, r4g_narrow_ab.txt).
    constexpr int narrowG = kNarrowGroupLanes;
    constexpr int narrowRows = 1;
    auto rows_for = [&](int p, int maxI, int w) -> int {
        if (p == 0) return 0;
        if (p == 1)
            return (64 / narrowG) * coop_group_bytes(kCoopNarrowRows, w, 0) <= kCoopLdsBytes
                       ? kCoopNarrowRows : 0;
        const long long room = (tallGroupLds - (long long)coop_group_bytes(0, w, 0)) / 16 / 64 * 64;
        const long long full = full_rows(maxI);   // a column never exceeds I + 1 rows
        if (p == 2) {   // LDS only
            const long long want = std::min<long long>(kCoopTallRows, full);
            return room >= want ? (int)want : 0;
        }
        // hybrid: as many LDS rows as fit, up to kHybridRows (the rest of a column goes to global memory)
        // PBCCS_HYBRID_LDS_KB / PBCCS_HYBRID_ROWS (A/B): the hybrid path's LDS budget per read and its row cap
        static const long long hybLds = (long long)env_int("PBCCS_HYBRID_LDS_KB", (int)(kCoopLdsBytes >> 10)) << 10;
        static const long long hybRows = env_int("PBCCS_HYBRID_ROWS", kHybridRows);
        const long long hroom = (std::min<long long>(hybLds, 160 << 10) - (long long)coop_group_bytes(0, w, 0)) / 16 / 64 * 64;
        const long long want = std::min(std::min(full, hroom), hybRows);
        return want >= 64 ? (int)want : 0;
    };
    // PBCCS_FILL_PATHS=1: one stderr line per launch set (reads per path, wall ms, reads re-routed / regrown)
    static const bool pathTrace = std::getenv("PBCCS_FILL_PATHS") != nullptr;
    // PBCCS_FILL_PATHS=2: also per launch the slowest read (its wall ms, cycles per cell, cells, passes)
    static const bool pathTrace2 = pathTrace && std::getenv("PBCCS_FILL_PATHS")[0] == '2';
    // PBCCS_FILL_WORK=1: where the fills' computed cells go (CoopFill::work; counters().fillWork)
    static const bool fillWork = std::getenv("PBCCS_FILL_WORK") != nullptr;
    for (int attempt = 0;; ++attempt) {
        // route reads whose buffers do not fit this path's LDS budget to the next path
        for (int p = 0; p < kPaths; ++p) {
            std::vector<int> keep;
            for (int r : todo[p]) {
                if (rows_for(p, (int)reads_[r].seq.size(), words(r)) > 0) keep.push_back(r);
                else if (p + 1 < kPaths) todo[p + 1].push_back(r);
                else {
                    reads_[r].fillPath = kPaths;
                    serial.push_back(r);
                }
            }
            todo[p].swap(keep);
        }
        if (std::all_of(todo, todo + kPaths, [](const std::vector<int>& v) { return v.empty(); })) break;
        if (attempt > 8) throw DeviceError("band storage keeps overflowing");
        // Wave composition: a 16-lane wavefront fills four consecutive reads of the list in lock-step and runs
        // until its slowest read's passes end.  A refill's pass count follows the read's last fill -- about half
        // of the typical reads at 2 kb end after alpha + beta (0 flip-flops), the rest run the flip-flop loop
        // (oracle: 101 / 110 of 211) -- so reads with flip-flops last time come first, then the others, each
        // group by window length (similar lengths share a wave; LDS is sized by the launch's longest).
        auto quick = [&](int x) { return reads_[x].filled && reads_[x].flips == 0 ? 1 : 0; };
        // Within a flip group, reads whose last band averaged more than 16 rows per column (two 16-row chunks in
        // many columns) come first (+1.4%).  The tall paths' reads go by their last band size, largest first:
        // the longest fills start first (+2.0%; profiles/r2h10_sort_ab/).
        auto high = [&](int x) {
            const HRead& h = reads_[x];
            return h.filled && std::max(h.usedA, h.usedB) > 16LL * (h.te - h.ts + 1) ? 0 : 1;
        };
        for (int p = 0; p < kPaths; ++p) {
            auto& v = todo[p];
            if (p >= 2) {
                std::stable_sort(v.begin(), v.end(), [&](int x, int y) {
                    return std::max(reads_[x].usedA, reads_[x].usedB) > std::max(reads_[y].usedA, reads_[y].usedB);
                });
                continue;
            }
            std::stable_sort(v.begin(), v.end(), [&](int x, int y) {
                const int qx = quick(x), qy = quick(y);
                if (qx != qy) return qx < qy;
                const int hx = high(x), hy = high(y);
                if (hx != hy) return hx < hy;
                return reads_[x].te - reads_[x].ts > reads_[y].te - reads_[y].ts;
            });
        }
        // checkpointed bands for the tall paths' long windows (and every cooperative fill under the test hook)
        for (int p = 0; p < kPaths; ++p)
            for (int r : todo[p]) {
                HRead& h = reads_[r];
                int k = 0;
                if (ckptAll_ > 0 && p >= 1) k = ckptAll_;
                else if (ckptK_ > 0 && p >= 2 && h.te - h.ts >= ckptMinLen_) k = ckptK_;
                if (h.ckpt != k) {
                    h.ckpt = k;
                    descDirty_ = true;
                }
            }
        // the certified fast path (scan_): the LDS-only tall path's reads (checkpointed or not) fill with the
        // reassociated chain, listed first; a read whose last certified fill met an uncertain decision runs exactly.
        // PBCCS_SCAN_PATHS (read per batch): bit 0 the LDS-only path, bit 1 the hybrid one -- certified and tested
        // too, but off by default: its fills ran no faster per cell and its longer reads' wider bounds sent 16 ZMW
        // rounds to the exact re-run instead of 3 (configs[3] 12.2 vs 13.6 ZMWs/s, profiles/r9o_hybrid_scan_ab.txt).
        const int scanPaths = env_int("PBCCS_SCAN_PATHS", 1);
        auto scannable = [&](int r) { return scan_ && !reads_[r].exact; };
        int nScan[kPaths] = {};
        for (int p = 2; p < kPaths; ++p) {
            if (!((scanPaths >> (p - 2)) & 1)) continue;
            std::stable_partition(todo[p].begin(), todo[p].end(), scannable);
            nScan[p] = (int)std::count_if(todo[p].begin(), todo[p].end(), scannable);
        }
        const bool anyScan = nScan[2] + nScan[3] > 0;
        UploadDescriptors();
        const size_t R = reads_.size();
        dUsedA_.reserve(std::max<size_t>(R, 1), true);
        dUsedB_.reserve(std::max<size_t>(R, 1), true);
        dMaxH_.reserve(std::max<size_t>(R, 1), true);
        std::vector<int> list;
        for (auto& v : todo) list.insert(list.end(), v.begin(), v.end());
        upload(dList_, list, stream_);
        const DevBatch B = View();
        size_t off = 0;
        // the 64-lane (tall) launches run on a second stream beside the 16-lane one: a round's latency
        // is then the slower of the two, not their sum.  Fork before the first launch (after the list
        // upload), so the tall fills do not wait for the 16-lane fill.
        const bool forked = !todo[2].empty() || !todo[3].empty();
        const auto tLaunch = std::chrono::steady_clock::now();
        // Headroom for in-kernel band growth (CoopFill::valBump): reads on the tall paths grow to a few
        // percent of their full (I+1)(J+1) matrix; budgeted against the device's free memory.  Growth
        // beyond the mapped headroom falls back to count-only + relaunch below.
        const bool grow = ws_->val.allowVmm;
        long long headroom = 0;
        if (grow) {
            long long want = 1ll << 24;   // 128 MB for the occasional 16-lane overflow
            for (int p = 2; p < kPaths; ++p)
                for (int r : todo[p]) {   // tall bands use ~2-22% of the full matrix (mean ~11%)
                    const long long I = (long long)reads_[r].seq.size(), J = reads_[r].te - reads_[r].ts;
                    const long long K = std::max(1, reads_[r].ckpt);
                    want += 2 * std::max<long long>(0, (I + 1) * (J + 1) / 7 / K - reads_[r].valCap);
                }
            size_t freeB = 0, totalB = 0;
            PBCCS_HIP(hipMemGetInfo(&freeB, &totalB));
            // a quarter of what is free beyond a margin kept for the score buffers and the other slots'
            // hipMalloc growth: speculative headroom must never be what runs the device out of memory
            // PBCCS_HEADROOM_MARGIN_GB (A/B): the free memory the speculative headroom leaves alone
            static const long long margin = (long long)env_int("PBCCS_HEADROOM_MARGIN_GB", (int)(kHeadroomMargin >> 30)) << 30;
            const long long spare = std::max<long long>(0, (long long)freeB - margin);
            headroom = std::min<long long>(want, spare / 4 / (long long)sizeof(double));
            // the reads' own regions must be mapped; the growth headroom only as far as device memory
            // allows (several batches grow at once): the kernel's limit is what actually got mapped
            dVal_.reserve((size_t)std::max<long long>(valTop_, 1), true);
            dVal_.try_reserve((size_t)std::max<long long>(valTop_ + headroom, 1));
            dBump_.reserve(1, false);
            const unsigned long long top = (unsigned long long)valTop_;
            PBCCS_HIP(hipMemcpyAsync(dBump_.ptr, &top, sizeof(top), hipMemcpyHostToDevice, stream_));
        }
        const long long valLimit = grow ? (long long)dVal_.cap : 0;
        if (forked) {
            PBCCS_HIP(hipEventRecord(evFork_, stream_));
            PBCCS_HIP(hipStreamWaitEvent(stream2_, evFork_, 0));
        }
        for (int p = 0; p < kPaths; ++p) {
            const int n = (int)todo[p].size();
            if (n == 0) continue;
            int maxI = 1, maxJ = 1;
            for (int r : todo[p]) {
                maxI = std::max(maxI, (int)reads_[r].seq.size());
                maxJ = std::max(maxJ, reads_[r].te - reads_[r].ts);
            }
            CoopFill F;
            F.usedA = dUsedA_.ptr;
            F.usedB = dUsedB_.ptr;
            F.maxH = dMaxH_.ptr;
            F.readWords = (maxI + 7) / 8;
            F.tplWords = (maxJ + 8) / 8;
            F.hcap = rows_for(p, maxI, F.readWords + F.tplWords);
            const int G = p == 1 ? narrowG : tallG;
            F.rows = p == 1 ? narrowRows : tallRows;
            F.prio = p >= 2;   // (neutral in an A/B against no priority, profiles/r4k_tall_prio_slots.txt)
            if (const char* e = std::getenv("PBCCS_FILL_THR_MARGIN"))   // test hook, read per launch
                F.thrMargin = std::max(0x1p-50, std::atof(e));
            F.groupBytes = coop_group_bytes(F.hcap, F.readWords, F.tplWords);
            const int full = (int)full_rows(maxI);
            if (p == 3 && full > F.hcap) {   // hybrid: column rows past the LDS buffer, two buffers per read
                F.gRows = full - F.hcap;
                dColScratch_.reserve((size_t)n * 2 * F.gRows, false);
                F.colScratch = dColScratch_.ptr;
            }
            if (grow) {
                F.valBump = dBump_.ptr;
                F.valLimit = valLimit;
                F.rValA = pRValA_;
                F.rValB = pRValB_;
                F.rValCap = pRValCap_;
            }
            const int* lp = dList_.ptr + off;
            const hipStream_t st = p <= 1 ? stream_ : stream2_;
            if (fillWork) {
                if (!dFillWork_.ptr) {
                    dFillWork_.reserve(16, false);
                    PBCCS_HIP(hipMemsetAsync(dFillWork_.ptr, 0, 16 * sizeof(unsigned long long), stream_));
                }
                F.work = dFillWork_.ptr;
            }
            if (pathTrace2) {   // on the launch's own stream (the tall ones run beside stream_)
                dCoopTrace_[p].reserve((size_t)6 * n, false);
                PBCCS_HIP(hipMemsetAsync(dCoopTrace_[p].ptr, 0, sizeof(long long) * 6 * n, st));
                F.trace = dCoopTrace_[p].ptr;
            }
            const int nScan2 = nScan[p];
            if (nScan2 > 0) {   // certified scan launch over the first nScan2 reads, the exact rest after it
                CoopFill FS = F;
                FS.scan = true;
                if (const char* e = std::getenv("PBCCS_SCAN_DEV_SCALE")) FS.devScale = std::max(1.0, std::atof(e));
                Timed(p == 1 ? kKFill : kKFillTall, [&] { launch_fill_coop(G, B, FS, lp, nScan2, st); }, st);
                PBCCS_HIP(hipGetLastError());
                counters_.fillLaunches += 1;
                counters_.scanReads += nScan2;
                if (n > nScan2) {
                    Timed(p == 1 ? kKFill : kKFillTall, [&] { launch_fill_coop(G, B, F, lp + nScan2, n - nScan2, st); },
                          st);
                    PBCCS_HIP(hipGetLastError());
                    counters_.fillLaunches += 1;
                }
            } else {
                Timed(p == 1 ? kKFill : kKFillTall, [&] { launch_fill_coop(G, B, F, lp, n, st); }, st);
                PBCCS_HIP(hipGetLastError());
                counters_.fillLaunches += 1;
            }
            off += n;
        }
        if (forked) {
            PBCCS_HIP(hipEventRecord(evJoin_, stream2_));
            PBCCS_HIP(hipStreamWaitEvent(stream_, evJoin_, 0));
            // PBCCS_DBG_JOINSYNC=1 (debug): the host also waits for the tall stream itself before the downloads
            static const bool joinSync = std::getenv("PBCCS_DBG_JOINSYNC") && std::getenv("PBCCS_DBG_JOINSYNC")[0] == '1';
            if (joinSync) PBCCS_HIP(hipStreamSynchronize(stream2_));
        }
        std::vector<int> st, fl, ua, ub, mh;
        std::vector<double> bl, dv;
        unsigned long long bump = (unsigned long long)valTop_;
        {   // the per-read results in one transfer
            std::vector<Xfer> xs{xfer_dl(mh, dMaxH_, R), xfer_dl(st, dRStatus_, R), xfer_dl(fl, dRFlips_, R),
                                 xfer_dl(bl, dRBaseline_, R), xfer_dl(ua, dUsedA_, R), xfer_dl(ub, dUsedB_, R)};
            if (anyScan) xs.push_back(xfer_dl(dv, dRDev_, R));
            if (grow) xs.push_back(Xfer{dBump_.ptr, &bump, sizeof(bump)});
            download_packed(xs, ws_->xStage, hXStage_, stream_);
        }
        if (grow && bump != (unsigned long long)valTop_) {
            // some reads moved to larger regions: adopt the device's descriptors (host mirrors stay exact)
            std::vector<long long> va, vb, vc;
            va.resize(R);
            vb.resize(R);
            vc.resize(R);
            d2h(va.data(), pRValA_, R * sizeof(long long), stream_);
            d2h(vb.data(), pRValB_, R * sizeof(long long), stream_);
            d2h(vc.data(), pRValCap_, R * sizeof(long long), stream_);
            PBCCS_HIP(hipStreamSynchronize(stream_));
            for (auto& v : todo)
                for (int r : v) {
                    reads_[r].valA = va[r];
                    reads_[r].valB = vb[r];
                    reads_[r].valCap = vc[r];
                }
            valTop_ = (long long)std::min<unsigned long long>(bump, (unsigned long long)valLimit);
            counters_.bandGrowths += 1;
        }
        if (pathTrace) {
            int nt = 0, no = 0;
            for (int p = 0; p < kPaths; ++p)
                for (int r : todo[p]) {
                    nt += st[r] == kFillTall;
                    no += st[r] == kFillOverflow;
                }
            std::fprintf(stderr, "[fillpaths] batch=%p attempt=%d n=%zu/%zu/%zu/%zu wall=%.1fms tall=%d ovf=%d\n",
                         (void*)this, attempt, todo[0].size(), todo[1].size(), todo[2].size(), todo[3].size(),
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tLaunch).count(),
                         nt, no);
            for (int p = 1; pathTrace2 && p < kPaths; ++p) {
                const size_t n = todo[p].size();
                if (n == 0) continue;
                std::vector<long long> tr;
                download(tr, dCoopTrace_[p], 6 * n, stream_);
                PBCCS_HIP(hipStreamSynchronize(stream_));
                long long t0 = LLONG_MAX, t1 = 0;
                size_t slow = 0;
                double sumCells = 0, sumCyc = 0;
                for (size_t t = 0; t < n; ++t) {
                    if (tr[6 * t + 1] <= 0) continue;
                    t0 = std::min(t0, tr[6 * t]);
                    t1 = std::max(t1, tr[6 * t + 1]);
                    if (tr[6 * t + 1] - tr[6 * t] > tr[6 * slow + 1] - tr[6 * slow]) slow = t;
                    sumCells += (double)tr[6 * t + 3];
                    sumCyc += (double)tr[6 * t + 2];
                }
                const long long* s = &tr[6 * slow];
                std::fprintf(stderr, "[fillread] path=%d n=%zu span=%.1fms slowest: %.1fms %.1f cyc/cell cells=%lld "
                             "passes=%lld cols=%lld; all: %.1f cyc/cell\n", p, n, (t1 - t0) / 1e5, (s[1] - s[0]) / 1e5,
                             s[3] ? (double)s[2] / (double)s[3] : 0.0, s[3], s[4], s[5],
                             sumCells > 0 ? sumCyc / sumCells : 0.0);
            }
        }
        std::vector<int> next[kPaths];
        for (int p = 0; p < kPaths; ++p) {
            for (int r : todo[p]) {
                HRead& h = reads_[r];
                if (st[r] == kFillTall) {   // never from the hybrid path (3)
                    const int q = promote(r, p);
                    if (q >= kPaths) serial.push_back(r);
                    else next[q].push_back(r);
                    continue;
                }
                if (st[r] == kFillUncertain) {   // re-run on the exact path (same path, the exact launch)
                    h.exact = true;
                    counters_.uncertainReads += 1;
                    for (int bit = 0; bit < 4; ++bit) counters_.uncertainWhy[bit] += (fl[r] >> bit) & 1;
                    next[p].push_back(r);
                    continue;
                }
                if (st[r] == kFillOverflow) {
                    const long long need = std::max(ua[r], ub[r]);
                    h.valCap = std::max(need + need / 16 + 64, h.valCap + 1);
                    h.valA = valTop_;
                    h.valB = valTop_ + h.valCap;
                    valTop_ += 2 * h.valCap;
                    descDirty_ = true;
                    next[p].push_back(r);
                    continue;
                }
                h.status = st[r];
                h.flips = fl[r];
                h.baseline = bl[r];
                h.dev = !dv.empty() ? dv[r] : 0.0;   // every cooperative fill writes it (0 when exact)
                h.filled = true;
                h.usedA = ua[r];
                h.usedB = ub[r];
                if (p >= 1) h.maxH = mh[r];
                if (st[r] == kFillOk || st[r] == kFillMismatch) done.push_back(r);
            }
        }
        for (int p = 0; p < kPaths; ++p) todo[p].swap(next[p]);
    }
    if (!done.empty()) {
        upload(dList_, done, stream_);
        const DevBatch B = View();
        Timed(kKSuffix, [&] { launch_suffix(B, dList_.ptr, (int)done.size(), stream_, true); });
        PBCCS_HIP(hipGetLastError());
        PBCCS_HIP(hipStreamSynchronize(stream_));   // the list buffer is reused by the next step
    }
    if (!serial.empty()) FillReadsSerial(serial);
    (void)counters();   // band footprint high-water marks
}

void ArrowBatch::FillReadsSerial(const std::vector<int>& readsIn)
{
    const StreamScope bound(stream_);
    std::vector<int> todo(readsIn);
    for (int r : todo)   // the lane-serial fill keeps full bands
        if (reads_[r].ckpt != 0) {
            reads_[r].ckpt = 0;
            descDirty_ = true;
        }
    for (int r : todo) EnsureCapacity(r);
    int H = kFillBandHeight;
    for (int attempt = 0; !todo.empty(); ++attempt) {
        if (attempt > 8) throw DeviceError("band storage keeps overflowing");
        // a 64-read fill group should hold windows of similar length (lanes run in lock-step)
        std::stable_sort(todo.begin(), todo.end(), [&](int x, int y) {
            return reads_[x].te - reads_[x].ts > reads_[y].te - reads_[y].ts;
        });
        UploadDescriptors();
        const size_t R = reads_.size();
        dUsedA_.reserve(std::max<size_t>(R, 1), true);
        dUsedB_.reserve(std::max<size_t>(R, 1), true);
        std::vector<int> again;
        size_t pos = 0;
        while (pos < todo.size()) {
            const int capCols = reads_[todo[pos]].te - reads_[todo[pos]].ts + 2;
            const long long capSlots = (long long)capCols * H + 64;
            const double perGroup = 2.0 * capSlots * 64 * 8 + 2.0 * capCols * 64 * 20 + (capCols + 1.0) * 64 * 8;
            const long long maxGroups = std::max<long long>(1, (long long)(kFillScratchBudget / perGroup));
            const size_t n = std::min<size_t>(todo.size() - pos, (size_t)maxGroups * 64);
            std::vector<int> chunk(todo.begin() + pos, todo.begin() + pos + n);
            const long long groups = (long long)(n + 63) / 64;
            ws_->fVal.reserve((size_t)(2 * groups * capSlots * 64), false);
            ws_->fRange.reserve((size_t)(2 * groups * capCols * 64), false);
            ws_->fOff.reserve((size_t)(2 * groups * capCols * 64), false);
            ws_->fLs.reserve((size_t)(2 * groups * capCols * 64), false);
            ws_->fPre.reserve((size_t)(groups * (capCols + 1) * 64), false);
            FillScratch F;
            F.val = ws_->fVal.ptr;
            F.range = ws_->fRange.ptr;
            F.off = ws_->fOff.ptr;
            F.ls = ws_->fLs.ptr;
            F.pre = ws_->fPre.ptr;
            F.usedA = dUsedA_.ptr;
            F.usedB = dUsedB_.ptr;
            F.capSlots = capSlots;
            F.capCols = capCols;
            static const bool trace = std::getenv("PBCCS_FILL_TRACE") != nullptr;
            if (trace) {
                dTrace_.reserve(8 * n, false);
                F.trace = dTrace_.ptr;
            }
            upload(dList_, chunk, stream_);
            const DevBatch B = View();
            Timed(kKFillTall, [&] { launch_fill(B, F, dList_.ptr, (int)n, stream_); });
            PBCCS_HIP(hipGetLastError());
            counters_.fillLaunches += 1;
            std::vector<int> st, fl, ua, ub;
            std::vector<double> bl;
            download_packed({xfer_dl(st, dRStatus_, R), xfer_dl(fl, dRFlips_, R), xfer_dl(bl, dRBaseline_, R),
                             xfer_dl(ua, dUsedA_, R), xfer_dl(ub, dUsedB_, R)},
                            ws_->xStage, hXStage_, stream_);
            if (trace) TraceSummary(n, H, capSlots);
            for (int r : chunk) {
                HRead& h = reads_[r];
                if (st[r] == kFillOverflow) {
                    again.push_back(r);
                    continue;
                }
                h.status = st[r];
                h.flips = fl[r];
                h.baseline = bl[r];
                h.dev = 0.0;   // the lane-serial fill is exact
                h.filled = true;
                h.usedA = ua[r];
                h.usedB = ub[r];
                if (st[r] == kFillOk || st[r] == kFillMismatch) {
                    const long long need = std::max(ua[r], ub[r]);
                    if (need > h.valCap) {   // move to a larger compact region
                        h.valCap = need + need / 4 + 64;
                        h.valA = valTop_;
                        h.valB = valTop_ + h.valCap;
                        valTop_ += 2 * h.valCap;
                        descDirty_ = true;
                    }
                }
            }
            UploadDescriptors();
            const DevBatch B2 = View();
            Timed(kKCompact, [&] { launch_compact(B2, F, dList_.ptr, (int)n, stream_); });
            Timed(kKSuffix, [&] { launch_suffix(B2, dList_.ptr, (int)n, stream_); });
            PBCCS_HIP(hipGetLastError());
            PBCCS_HIP(hipStreamSynchronize(stream_));   // the next chunk reuses the scratch and the list
            pos += n;
        }
        todo.swap(again);
        H *= 2;
    }
}

// Per-lane timing of the last fill launch (wall clock, 100 MHz), summarised to stderr.
void ArrowBatch::TraceSummary(size_t n, int H, long long capSlots)
{
    std::vector<long long> tr;
    download(tr, dTrace_, 8 * n, stream_);
    PBCCS_HIP(hipStreamSynchronize(stream_));
    long long t0 = LLONG_MAX, t1 = 0, maxDur = 0, maxCells = 0, sumCells = 0, sumPass = 0, maxPass = 0;
    double sumDur = 0;
    long long done = 0;
    for (size_t t = 0; t < n; ++t) {
        const long long* e = &tr[8 * t];
        if (e[1] <= 0) continue;
        ++done;
        t0 = std::min(t0, e[0]);
        t1 = std::max(t1, e[1]);
        maxDur = std::max(maxDur, e[1] - e[0]);
        sumDur += double(e[1] - e[0]);
        maxCells = std::max(maxCells, e[2]);
        sumCells += e[2];
        sumPass += e[3];
        maxPass = std::max(maxPass, e[3]);
    }
    std::fprintf(stderr,
                 "[fill-trace] lanes=%zu done=%lld H=%d capSlots=%lld span_ms=%.3f maxlane_ms=%.3f avglane_ms=%.3f "
                 "cells avg=%.0f max=%lld passes avg=%.2f max=%lld\n",
                 n, done, H, capSlots, (t1 - t0) / 1e5, maxDur / 1e5, done ? sumDur / done / 1e5 : 0.0,
                 done ? double(sumCells) / done : 0.0, maxCells, done ? double(sumPass) / done : 0.0, maxPass);
}

void ArrowBatch::MeanVar(const HZmw& z, int strand, int ts, int te, double* mean, double* var) const
{
    const std::string t = strand == kFwd ? z.tpl : reverse_complement(z.tpl);
    const int L = (int)t.size();
    double m = 0.0, v = 0.0;
    for (int i = ts; i < te - 1; ++i) {
        const int c = (i + 1 < L) ? context_index(t[i], t[i + 1]) : kCtxZero;
        m += z.ctxMeanVar[c][0];
        v += z.ctxMeanVar[c][1];
    }
    *mean = m;
    *var = v;
}

void ArrowBatch::CertifyAddReads(const std::vector<int>& readsIn, double threshold)
{
    if (std::isnan(threshold)) return;
    std::vector<int> redo;
    for (int ri : readsIn) {
        HRead& r = reads_[ri];
        if (r.dev <= 0.0 || r.status != kFillOk || !std::isfinite(r.baseline)) continue;
        double mean = 0.0, var = 0.0;
        MeanVar(zmws_[r.zmw], r.strand, r.ts, r.te, &mean, &var);
        const double sd = std::sqrt(var);
        const double z = (r.baseline - mean) / sd;
        // the reference's z lies within (dev + the rounding of (ll - mean) / sd) / sd of this one
        if (!std::isfinite(z) || std::fabs(z - threshold) <= (r.dev + 4.0 * kUnitRoundoff * (std::fabs(r.baseline) +
                                                                                          std::fabs(mean))) / sd +
                                                                  8.0 * kUnitRoundoff * std::fabs(z)) {
            r.exact = true;
            redo.push_back(ri);
        }
    }
    if (redo.empty()) return;
    counters_.uncertainReads += (long long)redo.size();
    FillReads(redo);
}

int ArrowBatch::FinishAddRead(int ri, double threshold)
{
    // MultiReadMutationScorer::AddRead (MultiReadMutationScorer.cpp:275-325)
    HRead& r = reads_[ri];
    int res = kSuccess;
    if (r.status == kFillBadInput) res = kOther;
    else if (r.status == kFillMismatch || std::isinf(r.baseline)) res = kAlphaBetaMismatch;   // MutationScorer.cpp:68-69
    if (res == kSuccess && !std::isnan(threshold)) {
        double mean = 0.0, var = 0.0;
        MeanVar(zmws_[r.zmw], r.strand, r.ts, r.te, &mean, &var);
        const double ll = r.baseline;
        const double z = (ll - mean) / std::sqrt(var);
        if (!std::isfinite(ll) || !std::isfinite(z) || z < threshold) res = kPoorZScore;
    }
    r.active = res == kSuccess;
    descDirty_ = true;
    return res;
}

double ArrowBatch::BaselineScore(int zi) const
{
    const HZmw& z = zmws_[zi];
    double s = 0.0;
    for (int k = 0; k < z.nReads; ++k) {
        const HRead& r = reads_[z.readBegin + k];
        if (r.active) s += r.baseline;
    }
    return s;
}

void ArrowBatch::ZScores(int zi, double* zg, double* za, std::vector<double>* zs) const
{
    // MultiReadMutationScorer::ZScores (MultiReadMutationScorer.hpp:208-263)
    const HZmw& z = zmws_[zi];
    const double nan = std::numeric_limits<double>::quiet_NaN();
    zs->clear();
    double gmean = 0.0, gvar = 0.0;
    size_t n = 0;
    for (int k = 0; k < z.nReads; ++k) {
        const HRead& r = reads_[z.readBegin + k];
        if (!r.active) { zs->push_back(nan); continue; }
        n += 1;
        const int s = r.ts, e = r.te - 1;
        if (e - s < 1) { zs->push_back(nan); continue; }
        double mu = 0.0, var = 0.0;
        MeanVar(z, r.strand, r.ts, r.te, &mu, &var);
        gmean += mu;
        gvar += var;
        zs->push_back((r.baseline - mu) / std::sqrt(var));
    }
    const double gs = BaselineScore(zi);
    *zg = (gvar == 0.0) ? nan : (gs - gmean) / std::sqrt(gvar);
    *za = (n == 0 || gvar == 0.0) ? nan : (gs / n - gmean / n) / std::sqrt(gvar / n);
}

// ------------------------------------------------------------------------------------------------
// scoring rounds
// ------------------------------------------------------------------------------------------------
void ArrowBatch::RunRound(const std::vector<int>& zl, const std::vector<std::vector<int>>* codes, double fastThr,
                          bool needPositions, bool phased)
{
    const StreamScope bound(stream_);
    UploadDescriptors();
    const int n = (int)zl.size();
    rNMut_.assign(n, 0);
    rMutStart_.assign(n + 1, 0);
    rPosStart_.assign(n + 1, 0);
    rDeltaBase_.assign(n, 0);
    std::vector<long long> waveStart(n + 1, 0), posBase(n, 0);
    long long delta = 0, posOffTotal = 0;
    for (int k = 0; k < n; ++k) {
        const HZmw& z = zmws_[zl[k]];
        const long long M = codes ? (long long)(*codes)[k].size() : unique_mutation_count(z.tpl);
        rNMut_[k] = (int)M;
        rMutStart_[k + 1] = rMutStart_[k] + M;
        rDeltaBase_[k] = delta;
        delta += M * z.nReads;
        waveStart[k + 1] = waveStart[k] + (long long)z.nReads * ((M + 63) / 64);
        rPosStart_[k + 1] = rPosStart_[k] + (long long)z.tpl.size();
        posBase[k] = posOffTotal;
        posOffTotal += (long long)z.tpl.size() + 1;
    }
    rTotalMut_ = rMutStart_[n];
    rTotalPos_ = rPosStart_[n];
    rTotalDelta_ = delta;
    std::vector<long long> mutBase(rMutStart_.begin(), rMutStart_.begin() + n);
    upload_packed({xfer_ul(dWZmw_, zl), xfer_ul(dWNMut_, rNMut_), xfer_ul(dWMutBase_, mutBase),
                   xfer_ul(dWDeltaBase_, rDeltaBase_), xfer_ul(dWWaveStart_, waveStart), xfer_ul(dWMutStart_, rMutStart_),
                   xfer_ul(dWPosStart_, rPosStart_), xfer_ul(dWPosBase_, posBase)},
                  ws_->xStage, hXStage_, stream_);
    dCodes_.reserve(std::max<long long>(rTotalMut_, 1), false);
    dScore_.reserve(std::max<long long>(rTotalMut_, 1), false);
    dFav_.reserve(std::max<long long>(rTotalMut_, 1), false);
    dDelta_.reserve(std::max<long long>(rTotalDelta_, 1), false);
    const DevBatch B = View();
    if (codes) {
        std::vector<int> flat;
        flat.reserve(rTotalMut_);
        for (const std::vector<int>& c : *codes) flat.insert(flat.end(), c.begin(), c.end());
        upload(dCodes_, flat, stream_);
        PBCCS_HIP(hipStreamSynchronize(stream_));
    } else {
        dPosOff_.reserve(std::max<long long>(posOffTotal, 1), false);
        Timed(kKEnumerate, [&] {
            launch_enumerate(B, dWZmw_.ptr, n, dWMutBase_.ptr, dWPosBase_.ptr, dCodes_.ptr, dPosOff_.ptr, stream_);
        });
    }
    (void)needPositions;
    ScoreWork W;
    W.nWork = n;
    W.zmw = dWZmw_.ptr;
    W.nMut = dWNMut_.ptr;
    W.mutBase = dWMutBase_.ptr;
    W.deltaBase = dWDeltaBase_.ptr;
    W.waveStart = dWWaveStart_.ptr;
    W.mutStart = dWMutStart_.ptr;
    W.posStart = dWPosStart_.ptr;
    W.codes = dCodes_.ptr;
    W.delta = dDelta_.ptr;
    // certified fast path: per item the bound of its summed scores -- each active read contributes 3x its LL bound
    // (the mutated read's LL, its baseline, and the prefix / suffix log-scale sums of its bands)
    {
        std::vector<double> dev(n, 0.0);
        bool any = false;
        for (int k = 0; k < n; ++k) {
            const HZmw& z = zmws_[zl[k]];
            for (int q = 0; q < z.nReads; ++q) {
                const HRead& h = reads_[z.readBegin + q];
                if (h.active && h.dev > 0.0) dev[k] += 3.0 * h.dev;
            }
            any = any || dev[k] > 0.0;
        }
        rDevItem_ = dev;
        if (any) {
            upload(ws_->wDev, dev, stream_);
            ws_->wAmb.reserve(std::max(n, 1), false);
            PBCCS_HIP(hipMemsetAsync(ws_->wAmb.ptr, 0, std::max(n, 1) * sizeof(int), stream_));
            W.dev = ws_->wDev.ptr;
            W.amb = ws_->wAmb.ptr;
        }
        rAmbOn_ = any;
    }
    // k_score_edge list: tasks within 3 columns of a window end; bound = 80 per (work item, read)
    long long edgeCap = 0;
    for (int k = 0; k < n; ++k) edgeCap += 80LL * zmws_[zl[k]].nReads;
    edgeCap = std::min<long long>(std::max<long long>(edgeCap, 64), rTotalDelta_ + 64);
    dEdge_.reserve(3 * edgeCap, false);
    dEdgeCount_.reserve(1, false);
    W.edgeList = dEdge_.ptr;
    W.edgeCount = dEdgeCount_.ptr;
    W.edgeCap = (int)edgeCap;
    // Checkpointed reads are scored by k_score_ckpt from a task list of (work item, read)
    // pairs: the phase's reads [lo, hi) of each item whose read keeps checkpoint columns only, with the chunks
    // of the phase's mutations (all of them, or the item's survivors nSel).
    bool anyCkpt = false;
    for (int k = 0; k < n && !anyCkpt; ++k) {
        const HZmw& z = zmws_[zl[k]];
        for (int q = 0; q < z.nReads; ++q) anyCkpt = anyCkpt || reads_[z.readBegin + q].ckpt != 0;
    }
    CkptWork ck;
    auto ckpt_tasks = [&](int lo, int hi, const std::vector<int>* nSelH) {
        ck = CkptWork();
        if (!anyCkpt) return;
        std::vector<int2> pairs;
        std::vector<long long> start{0};
        long long maxI = 1;
        int maxK = 1;
        for (int k = 0; k < n; ++k) {
            const HZmw& z = zmws_[zl[k]];
            const long long mc = nSelH ? (*nSelH)[k] : rNMut_[k];
            if (mc <= 0) continue;
            for (int q = std::max(0, lo); q < std::min(hi, z.nReads); ++q) {
                const HRead& h = reads_[z.readBegin + q];
                if (h.ckpt == 0) continue;
                pairs.push_back(make_int2(k, q));
                start.push_back(start.back() + (mc + 63) / 64);
                maxI = std::max<long long>(maxI, (long long)h.seq.size() + 1);
                maxK = std::max(maxK, h.ckpt);
            }
        }
        if (pairs.empty()) return;
        upload(dCkPairs_, pairs, stream_);
        upload(dCkStart_, start, stream_);
        ws_->ckCounter.reserve(2, false);
        // a block replays <= 3K + 4 columns, each at most I + 1 rows; start from 1024-row columns
        const long long first = (3LL * maxK + 4) * std::min<long long>(maxI, 1024);
        ckSlotCap_ = std::max(ckSlotCap_, first);
        ck.pairs = dCkPairs_.ptr;
        ck.taskStart = dCkStart_.ptr;
        ck.nPairs = (int)pairs.size();
        ck.nTasks = start.back();
        ck.counter = ws_->ckCounter.ptr;
        ck.need = ws_->ckCounter.ptr + 1;
        ck.nSlots = (int)std::min<long long>(ck.nTasks, kCkptSlotsMax);
    };
    ckpt_tasks(0, 1 << 30, nullptr);
    // one scoring launch (k_score + k_score_ckpt + k_score_edge) over W's current phase; re-run on scratch
    // overflow or when a checkpoint replay outgrew its slot
    auto score_launch = [&](long long nWaves) {
        for (int attempt = 0;; ++attempt) {
            PBCCS_HIP(hipMemsetAsync(dEdgeCount_.ptr, 0, sizeof(int), stream_));
            PBCCS_HIP(hipMemsetAsync(dScratchTop_.ptr, 0, sizeof(unsigned long long), stream_));
            PBCCS_HIP(hipMemsetAsync(dScratchOverflow_.ptr, 0, sizeof(int), stream_));
            ScoreScratch sc;
            sc.pool = dScratch_.ptr;
            sc.top = dScratchTop_.ptr;
            sc.cap = dScratch_.cap;
            sc.overflow = dScratchOverflow_.ptr;
            if (ck.nTasks > 0) {
                // replay slots: as many as fit kCkptSlotBytes, but at least 64 waves' worth -- a soft bound: for very
                // tall reads (slots over 16 MB each) the 64-slot floor takes more than 1 GB
                const long long fit = kCkptSlotBytes / std::max<long long>(1, ckSlotCap_ * (long long)sizeof(double));
                ck.nSlots = (int)std::max<long long>(
                    1, std::min<long long>(std::min<long long>(ck.nTasks, kCkptSlotsMax), std::max<long long>(64, fit)));
                ws_->ckSlots.reserve((size_t)ck.nSlots * ckSlotCap_, false);
                ck.slots = ws_->ckSlots.ptr;
                ck.slotCap = ckSlotCap_;
                PBCCS_HIP(hipMemsetAsync(ws_->ckCounter.ptr, 0, 2 * sizeof(unsigned long long), stream_));
            }
            Timed(kKScore, [&] { launch_score(B, W, nWaves, sc, stream_, ck.nTasks > 0 ? &ck : nullptr); });
            PBCCS_HIP(hipGetLastError());
            int ovf = 0;
            unsigned long long ckNeed = 0;
            d2h(&ovf, dScratchOverflow_.ptr, sizeof(int), stream_);
            if (ck.nTasks > 0)
                d2h(&ckNeed, ck.need, sizeof(ckNeed), stream_);
            PBCCS_HIP(hipStreamSynchronize(stream_));
            if (ckNeed >= kCkptBadGeometry) throw DeviceError("checkpoint replay: block outgrew its column tables");
            if (ckNeed > 0) {
                if (attempt > 8) throw DeviceError("checkpoint replay slots keep overflowing");
                ckSlotCap_ = (long long)ckNeed + (long long)ckNeed / 4 + 64;
                continue;
            }
            if (!ovf) break;
            if (attempt > 8) throw DeviceError("scratch overflow");
            if (ovf & 1) dScratch_.reserve(dScratch_.cap * 4, false);
            if (ovf & 2) {
                edgeCap *= 4;
                dEdge_.reserve(3 * edgeCap, false);
                W.edgeList = dEdge_.ptr;
                W.edgeCap = (int)std::min<long long>(edgeCap, INT_MAX / 4);
            }
        }
    };
    // Phased scoring (refine rounds only; fast-score threshold set, no per-read output wanted;
    // PBCCS_PHASED_MIN_TASKS=-1 turns it off).  The
    // reduction sums a mutation's reads in order and stops as soon as the sum falls below the fast-score
    // threshold (MultiReadMutationScorer.cpp:352-362), so the deltas of the reads after that break are never
    // read.  At configs[1] the break comes after 4.5 of 10 reads on average.  Phase 0 scores reads [0, 3)
    // of every mutation; each later phase first evaluates the ordered prefix over the reads scored so far
    // (k_alive: the same sums and break as k_reduce), keeps the mutations that have not broken (hipCUB
    // select, kept in list order), and scores the next reads of those only.  k_reduce then runs unchanged
    // over all reads: it breaks exactly where k_alive did and never touches an unscored delta.
    // PBCCS_PHASED_MIN_TASKS overrides the size from which a round is phased (tests: 0 = every round)
    const char* minEnv = std::getenv("PBCCS_PHASED_MIN_TASKS");
    const long long minTasks = minEnv ? std::atoll(minEnv) : kPhasedMinTasks;
    long long tasks = rTotalDelta_;
    if (phased && minTasks >= 0 && rTotalDelta_ >= minTasks && rTotalMut_ <= INT_MAX) {
        // phase boundaries (read indices); PBCCS_PHASE_BOUNDS="3,5" is the default, e.g. "3,4,5" adds a phase
        static const std::vector<int> bounds = [] {
            std::vector<int> b{0};
            const char* e = std::getenv("PBCCS_PHASE_BOUNDS");
            std::string spec = e ? e : "3,5";
            size_t pos = 0;
            while (pos < spec.size()) {
                const size_t c = spec.find(',', pos);
                const int v = std::atoi(spec.substr(pos, c == std::string::npos ? std::string::npos : c - pos).c_str());
                if (v > b.back()) b.push_back(v);
                if (c == std::string::npos) break;
                pos = c + 1;
            }
            b.push_back(1 << 30);
            return b;
        }();
        const int nPhases = (int)bounds.size() - 1;
        std::vector<std::vector<long long>> ws(nPhases);
        std::vector<int> nSel;
        ws_->sel.reserve(std::max<long long>(rTotalMut_, 1), false);
        ws_->selCount.reserve(2, false);
        dSelBase_.reserve(std::max(n, 1), false);
        dNSel_.reserve(std::max(n, 1), false);
        tasks = 0;
        for (int ph = 0; ph < nPhases; ++ph) {
            const int lo = bounds[ph], hi = bounds[ph + 1];
            if (ph > 0) {
                Timed(kKReduce, [&] { launch_alive(B, W, rTotalMut_, fastThr, lo, dFav_.ptr, stream_); });
                size_t tb = 0;
                hipcub::CountingInputIterator<long long> it(0);
                PBCCS_HIP(hipcub::DeviceSelect::Flagged(nullptr, tb, it, dFav_.ptr, ws_->sel.ptr, ws_->selCount.ptr,
                                                        (int)rTotalMut_, stream_));
                ws_->selTmp.reserve(std::max<size_t>(tb, 1), false);
                PBCCS_HIP(hipcub::DeviceSelect::Flagged(ws_->selTmp.ptr, tb, it, dFav_.ptr, ws_->sel.ptr,
                                                        ws_->selCount.ptr, (int)rTotalMut_, stream_));
                launch_sel_ranges(W, ws_->sel.ptr, ws_->selCount.ptr, dSelBase_.ptr, dNSel_.ptr, stream_);
                PBCCS_HIP(hipGetLastError());
                download(nSel, dNSel_, n, stream_);
                PBCCS_HIP(hipStreamSynchronize(stream_));
                W.sel = ws_->sel.ptr;
                W.selBase = dSelBase_.ptr;
                W.nSel = dNSel_.ptr;
            }
            std::vector<long long>& wsv = ws[ph];
            wsv.assign(n + 1, 0);
            for (int k = 0; k < n; ++k) {
                const int nr = zmws_[zl[k]].nReads;
                const long long reads = std::max(0, std::min(hi, nr) - lo);
                const long long mc = ph == 0 ? rNMut_[k] : nSel[k];
                wsv[k + 1] = wsv[k] + reads * ((mc + 63) / 64);
                tasks += reads * mc;
            }
            if (wsv[n] == 0) break;
            W.readLo = lo;
            W.readHi = hi;
            upload(dWWaveStart_, wsv, stream_);
            W.waveStart = dWWaveStart_.ptr;
            ckpt_tasks(lo, hi, ph == 0 ? nullptr : &nSel);
            score_launch(wsv[n]);
        }
        W.sel = nullptr;
        W.selBase = nullptr;
        W.nSel = nullptr;
        W.readLo = 0;
        W.readHi = 1 << 30;
    } else {
        score_launch(waveStart[n]);
    }
    Timed(kKReduce, [&] { launch_reduce(B, W, rTotalMut_, fastThr, dScore_.ptr, dFav_.ptr, stream_); });
    PBCCS_HIP(hipGetLastError());
    counters_.scoreLaunches += 1;
    counters_.scoreTasks += tasks;
    counters_.mutations += rTotalMut_;
}

void ArrowBatch::ScoreLists(const std::vector<int>& zl, const std::vector<std::vector<int>>& codes, double fastThr,
                            std::vector<std::vector<double>>* scores, std::vector<std::vector<double>>* perRead)
{
    const StreamScope bound(stream_);
    RunRound(zl, &codes, fastThr, false);
    std::vector<double> s, d;
    download(s, dScore_, rTotalMut_, stream_);
    if (perRead) download(d, dDelta_, rTotalDelta_, stream_);
    PBCCS_HIP(hipStreamSynchronize(stream_));
    scores->assign(zl.size(), {});
    if (perRead) perRead->assign(zl.size(), {});
    for (size_t k = 0; k < zl.size(); ++k) {
        (*scores)[k].assign(s.begin() + rMutStart_[k], s.begin() + rMutStart_[k + 1]);
        if (perRead) {
            const int nr = zmws_[zl[k]].nReads;
            (*perRead)[k].assign(d.begin() + rDeltaBase_[k], d.begin() + rDeltaBase_[k] + (long long)nr * rNMut_[k]);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// ApplyMutations (MultiReadMutationScorer.cpp:235-267): template edit + window remap; refill is
// done by the caller (batched across ZMWs).
// ------------------------------------------------------------------------------------------------
static bool apply_host(std::string* tpl, const std::vector<Mutation>& muts, std::vector<int>* mtp)
{
    std::string next;
    if (!apply_mutations(*tpl, muts, &next, mtp)) return false;
    *tpl = next;
    return true;
}

bool ArrowBatch::ApplyMutations(int zi, const std::vector<Mutation>& muts)
{
    const StreamScope bound(stream_);
    HZmw& z = zmws_[zi];
    std::vector<int> mtp;
    if (!apply_host(&z.tpl, muts, &mtp)) return false;
    UploadTemplate(zi);
    std::vector<int> refill;
    for (int k = 0; k < z.nReads; ++k) {
        HRead& r = reads_[z.readBegin + k];
        r.ts = mtp[r.ts];
        r.te = mtp[r.te];
        if (r.active) refill.push_back(z.readBegin + k);
    }
    descDirty_ = true;
    FillReads(refill);
    for (int r : refill)
        if (reads_[r].status != kFillOk) reads_[r].active = false;   // AlphaBetaMismatchException -> inactive
    descDirty_ = true;
    return true;
}

// ------------------------------------------------------------------------------------------------
// RefineConsensus (Consensus-inl.hpp:159-251), all listed ZMWs in lock-step rounds
// ------------------------------------------------------------------------------------------------
namespace {

struct Scored {
    int code;
    float score;
};

std::vector<Scored> best_subset(std::vector<Scored> in, int sep)   // Consensus-inl.hpp:98-118
{
    if (sep == 0) return in;
    std::vector<Scored> out;
    while (!in.empty()) {
        size_t best = 0;
        for (size_t k = 1; k < in.size(); ++k)
            if (in[best].score < in[k].score) best = k;
        const Scored b = in[best];
        out.push_back(b);
        const int lo = mut_pos(b.code) - sep, hi = mut_pos(b.code) + sep;
        std::vector<Scored> keep;
        keep.reserve(in.size());
        for (const Scored& s : in)
            if (!(lo <= mut_pos(s.code) && mut_pos(s.code) <= hi)) keep.push_back(s);
        in.swap(keep);
    }
    return out;
}

// Certified fast path: does BestSubset (Consensus-inl.hpp:98-118, first maximum of the float-cast
// scores) pick the same entries for every set of double scores within e of `sc`?  The casts of a score within e lie
// in [(float)(s - e), (float)(s + e)] (round to nearest is monotone).  Each pick is certain when the nominal winner's
// lowest cast beats every remaining entry's highest, or both casts are fixed and equal with the winner first.
bool best_subset_certain(const std::vector<Scored>& in, const std::vector<double>& sc, double e, int sep)
{
    const size_t n = in.size();
    if (n == 0 || e <= 0.0) return true;
    std::vector<float> lo(n), hi(n);
    for (size_t i = 0; i < n; ++i) {
        const double w = e + 4.0 * kUnitRoundoff * std::fabs(sc[i]);
        lo[i] = (float)(sc[i] - w);
        hi[i] = (float)(sc[i] + w);
    }
    std::vector<char> alive(n, 1);
    for (;;) {
        size_t best = n;
        for (size_t k = 0; k < n; ++k)
            if (alive[k] && (best == n || in[best].score < in[k].score)) best = k;
        if (best == n) return true;
        for (size_t k = 0; k < n; ++k) {
            if (!alive[k] || k == best) continue;
            if (hi[k] < lo[best]) continue;
            const bool fixedTie = lo[k] == hi[k] && lo[best] == hi[best] && lo[k] == lo[best] && k > best;
            if (!fixedTie) return false;
        }
        const int bp = mut_pos(in[best].code);
        if (sep == 0) {
            alive[best] = 0;
            continue;
        }
        for (size_t k = 0; k < n; ++k)
            if (alive[k] && bp - sep <= mut_pos(in[k].code) && mut_pos(in[k].code) <= bp + sep) alive[k] = 0;
    }
}

}  // namespace

void ArrowBatch::Refine(const std::vector<int>& zl, const RefineOptions& ro, std::vector<int>* converged,
                        std::vector<long long>* nTested, std::vector<long long>* nApplied, bool needFinalState,
                        std::vector<std::vector<int>>* qvsOnConverge)
{
    const StreamScope bound(stream_);
    const int n = (int)zl.size();
    converged->assign(n, 0);
    if (qvsOnConverge) qvsOnConverge->assign(n, {});
    // ZMWs whose bands nobody reads again once they are done (needFinalState = false: the batch polish reads
    // only converged ZMWs, through their QVs): retired so the reclaiming layout can drop them
    const bool retireDone = reclaim_ && !needFinalState;
    nTested->assign(n, 0);
    nApplied->assign(n, 0);
    std::vector<char> done(n, 0);
    std::vector<std::unordered_set<std::string>> history(n);
    std::vector<std::vector<int>> centers(n);
    std::vector<int> zit(n, 0);   // per-ZMW iteration of AbstractRefineConsensus
    // Iteration memo (replay of the reference's non-converging tails).
    //   An iteration's scoring outcome (the favourable list with its float scores) is a function of the
    //   loop state entering it, *relative* to the leftmost read window start a: the template from a - 1
    //   on (window bases plus the context base before a, which the reverse strand reads), the windows and
    //   active flags relative to a, and the previous favourable positions relative to a.  Template bases
    //   left of a - 1 are never read by a fill or scored by a read.  When the state entering iteration i
    //   equals (relative) the state entering iteration i - p, iteration i repeats iteration i - p's
    //   favourable list shifted by the change of a: the host then replays the iteration exactly -- nTested
    //   from the enumeration of the real template, BestSubset, the cycle check against the real history,
    //   ApplyMutations and the window remap -- with no fills and no scoring, and keeps going while the
    //   states keep matching.  This covers the two NonConvergent shapes seen at 2 kb: period-2
    //   oscillations and period-1 "crawls" that insert one base before the windows per iteration.
    struct Memo {
        int anchor = 0;
        std::string rtpl;
        std::vector<int> rwin;   // per read: ts - a, te - a, active
        std::vector<int> rcen;
        std::vector<Scored> fav;
        bool same(const Memo& o) const { return rtpl == o.rtpl && rwin == o.rwin && rcen == o.rcen; }
    };
    std::vector<std::vector<Memo>> memo(n);
    static const bool noReplay = std::getenv("PBCCS_NO_CYCLE_REPLAY") != nullptr;
    constexpr int kMaxPeriod = 4;
    auto make_memo = [&](int k) {
        const HZmw& z = zmws_[zl[k]];
        Memo m;
        int a = (int)z.tpl.size();
        for (int q = 0; q < z.nReads; ++q) a = std::min(a, reads_[z.readBegin + q].ts);
        m.anchor = a;
        m.rtpl = z.tpl.substr(std::max(0, a - 1));
        for (int q = 0; q < z.nReads; ++q) {
            const HRead& r = reads_[z.readBegin + q];
            m.rwin.push_back(r.ts - a);
            m.rwin.push_back(r.te - a);
            m.rwin.push_back(r.active ? 1 : 0);
        }
        for (int c : centers[k]) m.rcen.push_back(c - a);
        return m;
    };
    auto match = [&](int k, const Memo& cur) -> int {   // period p of a matching earlier state, or 0
        const int i = zit[k];
        for (int p = 1; p <= kMaxPeriod && p <= i; ++p)
            if (cur.same(memo[k][i - p])) return p;
        return 0;
    };
    const double fastThr = zl.empty() ? -12.5 : zmws_[zl[0]].opt.fastScoreThreshold;
    // PBCCS_ROUND_TRACE=1: one stderr line per round (active ZMWs, refilled reads, phase wall times)
    static const bool roundTrace = std::getenv("PBCCS_ROUND_TRACE") != nullptr;
    if (roundTrace)
        std::fprintf(stderr, "[round] batch=%p start zmws=%d bandtop=%.2fGB\n", (void*)this, n, valTop_ * 8.0 / 1e9);
    using Clock = std::chrono::steady_clock;
    auto ms = [](Clock::time_point a, Clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    std::vector<int> finalRefill;
    long long replayed = 0;
    for (int round = 0;; ++round) {
        const Clock::time_point t0 = Clock::now();
        // ---- memo: record the state entering each ZMW's iteration; replay matching iterations on the host
        std::vector<int> preRefill;
        for (int k = 0; k < n; ++k) {
            if (done[k]) continue;
            Memo cur = make_memo(k);
            int p = (noReplay || zit[k] == 0) ? 0 : match(k, cur);
            if (p == 0) {
                memo[k].push_back(std::move(cur));
                continue;
            }
            HZmw& z = zmws_[zl[k]];
            bool ended = false;
            while (p > 0) {
                const int i = zit[k];
                memo[k].push_back(std::move(cur));   // memo[k][i]: the state entering this iteration
                const int shift = memo[k][i].anchor - memo[k][i - p].anchor;
                std::vector<Scored> fav;
                for (const Scored& f : memo[k][i - p].fav)
                    fav.push_back({mut_code(mut_pos(f.code) + shift, mut_type(f.code), mut_base(f.code)), f.score});
                memo[k][i].fav = fav;
                // active flags after the refill = those the memoised transition's refill produced
                // (memo[k][i - p + 1] is memo[k][i] itself when p = 1)
                std::vector<char> succActive(z.nReads);
                for (int q = 0; q < z.nReads; ++q) succActive[q] = memo[k][i - p + 1].rwin[3 * q + 2] != 0;
                std::vector<int> tried;
                nearby_mutations(z.tpl, centers[k], ro.mutationNeighborhood, &tried);
                (*nTested)[k] += (long long)tried.size();
                std::vector<Scored> best = best_subset(fav, ro.mutationSeparation);
                std::vector<Mutation> muts;
                for (const Scored& b : best) muts.push_back(mutation_from_code(b.code));
                if (best.size() > 1) {
                    std::string next;
                    std::vector<int> mtp;
                    if (apply_mutations(z.tpl, muts, &next, &mtp) && history[k].count(next)) {
                        best.resize(1);
                        muts.resize(1);
                    }
                }
                (*nApplied)[k] += (long long)best.size();
                history[k].insert(z.tpl);
                centers[k].clear();
                for (const Scored& f : fav) centers[k].push_back(mut_pos(f.code));
                std::vector<int> mtp;
                if (!apply_host(&z.tpl, muts, &mtp)) {
                    done[k] = 1;
                    converged->at(k) = -1;
                    ended = true;
                    break;
                }
                for (int q = 0; q < z.nReads; ++q) {   // refill outcome = the memoised transition's
                    HRead& r = reads_[z.readBegin + q];
                    r.ts = mtp[r.ts];
                    r.te = mtp[r.te];
                    r.active = succActive[q] != 0;
                }
                ++replayed;
                if (++zit[k] >= ro.maxIterations) {
                    done[k] = 1;   // NonConvergent
                    ended = true;
                    break;
                }
                cur = make_memo(k);
                p = match(k, cur);
            }
            UploadTemplate(zl[k]);
            descDirty_ = true;
            if (!ended) memo[k].push_back(std::move(cur));   // a real iteration follows from this state
            std::vector<int>& dst = ended ? finalRefill : preRefill;
            if (ended && !needFinalState) {
                if (retireDone) Retire({zl[k]});
                continue;
            }
            for (int q = 0; q < z.nReads; ++q)
                if (reads_[z.readBegin + q].active) {
                    EnsureCapacity(z.readBegin + q);
                    dst.push_back(z.readBegin + q);
                }
        }
        if (!preRefill.empty()) {
            FillReads(preRefill);
            for (int r : preRefill)
                if (reads_[r].status != kFillOk) reads_[r].active = false;
            descDirty_ = true;
        }
        std::vector<int> act, idx;
        for (int k = 0; k < n; ++k)
            if (!done[k]) { act.push_back(zl[k]); idx.push_back(k); }
        if (act.empty()) break;
        std::vector<std::vector<int>> lists;
        if (round == 0) {
            RunRound(act, nullptr, fastThr, false, true);
        } else {
            lists.resize(act.size());
            for (size_t a = 0; a < act.size(); ++a)
                nearby_mutations(zmws_[act[a]].tpl, centers[idx[a]], ro.mutationNeighborhood, &lists[a]);
            RunRound(act, &lists, fastThr, false, true);
        }
        for (size_t a = 0; a < act.size(); ++a) (*nTested)[idx[a]] += rNMut_[a];
        const Clock::time_point t1 = Clock::now();

        // the favourable list of each listed ZMW of the last RunRound, compacted on the device in list order, with the
        // device BestSubset's picks (rank, entry) and the double scores (the certified path checks the float casts)
        auto select_round = [&](const std::vector<int>& actL, std::vector<std::vector<Scored>>& favL,
                                std::vector<std::vector<std::pair<int, Scored>>>& pickedL,
                                std::vector<std::vector<double>>& favD) {
            // favourable mutations, compacted on the device in list order
            DevVec<long long>& dSel = ws_->sel;
            DevVec<double>& dSelScore = ws_->selScore;
            DevVec<long long>& dCount = ws_->selCount;
            dSel.reserve(std::max<long long>(rTotalMut_, 1), false);
            dSelScore.reserve(std::max<long long>(rTotalMut_, 1), false);
            dCount.reserve(2, false);
            size_t tmpBytes = 0, tmpBytes2 = 0;
            hipcub::CountingInputIterator<long long> it(0);
            PBCCS_HIP(hipcub::DeviceSelect::Flagged(nullptr, tmpBytes, it, dFav_.ptr, dSel.ptr, dCount.ptr,
                                                    (int)rTotalMut_, stream_));
            PBCCS_HIP(hipcub::DeviceSelect::Flagged(nullptr, tmpBytes2, dScore_.ptr, dFav_.ptr, dSelScore.ptr,
                                                    dCount.ptr + 1, (int)rTotalMut_, stream_));
            DevVec<unsigned char>& tmp = ws_->selTmp;
            tmp.reserve(std::max<size_t>(std::max(tmpBytes, tmpBytes2), 1), false);
            PBCCS_HIP(hipcub::DeviceSelect::Flagged(tmp.ptr, tmpBytes, it, dFav_.ptr, dSel.ptr, dCount.ptr,
                                                    (int)rTotalMut_, stream_));
            PBCCS_HIP(hipcub::DeviceSelect::Flagged(tmp.ptr, tmpBytes2, dScore_.ptr, dFav_.ptr, dSelScore.ptr,
                                                    dCount.ptr + 1, (int)rTotalMut_, stream_));
            // the codes of the favourable entries (round 0's exist only on the device; later rounds' were uploaded)
            DevVec<int>& dSelCode = ws_->selCode;
            dSelCode.reserve(std::max<long long>(rTotalMut_, 1), false);
            size_t tb = 0;
            PBCCS_HIP(hipcub::DeviceSelect::Flagged(nullptr, tb, dCodes_.ptr, dFav_.ptr, dSelCode.ptr, dCount.ptr + 1,
                                                    (int)rTotalMut_, stream_));
            tmp.reserve(std::max<size_t>(tb, 1), false);
            PBCCS_HIP(hipcub::DeviceSelect::Flagged(tmp.ptr, tb, dCodes_.ptr, dFav_.ptr, dSelCode.ptr, dCount.ptr + 1,
                                                    (int)rTotalMut_, stream_));
            // BestSubset on the device: per ZMW its range of the compacted list, then one wavefront per ZMW
            const int nAct = (int)actL.size();
            dSelBase_.reserve(std::max(nAct, 1), false);
            dNSel_.reserve(std::max(nAct, 1), false);
            DevVec<int>& dSelRank = ws_->selRank;
            dSelRank.reserve(std::max<long long>(rTotalMut_, 1), false);
            ScoreWork SW;
            SW.nWork = nAct;
            SW.mutStart = dWMutStart_.ptr;
            launch_sel_ranges(SW, dSel.ptr, dCount.ptr, dSelBase_.ptr, dNSel_.ptr, stream_);
            const char* capEnv = std::getenv("PBCCS_BEST_LDS");   // tests: force the HBM path of long lists
            Timed(kKSelect, [&] {
                launch_best_subset(nAct, dSelBase_.ptr, dNSel_.ptr, dSelCode.ptr, dSelScore.ptr, ro.mutationSeparation,
                                   capEnv ? std::atoi(capEnv) : -1, dSelRank.ptr, stream_);
            });
            PBCCS_HIP(hipGetLastError());
            long long cnt[2] = {0, 0};
            d2h(cnt, dCount.ptr, 2 * sizeof(long long), stream_);
            PBCCS_HIP(hipStreamSynchronize(stream_));
            std::vector<long long> sel;
            std::vector<double> selScore;
            std::vector<int> selCode, selRank;
            download_packed({xfer_dl(sel, dSel, cnt[0]), xfer_dl(selScore, dSelScore, cnt[0]),
                             xfer_dl(selCode, dSelCode, cnt[0]), xfer_dl(selRank, dSelRank, cnt[0])},
                            ws_->xStage, hXStage_, stream_);

            favL.assign(actL.size(), {});
            pickedL.assign(actL.size(), {});
            favD.assign(actL.size(), {});
            for (size_t q = 0; q < sel.size(); ++q) {
                const long long g = sel[q];
                const size_t a = std::upper_bound(rMutStart_.begin(), rMutStart_.end(), g) - rMutStart_.begin() - 1;
                const Scored e{selCode[q], (float)selScore[q]};
                favL[a].push_back(e);
                favD[a].push_back(selScore[q]);
                if (selRank[q] > 0) pickedL[a].emplace_back(selRank[q], e);
            }
        };
        std::vector<std::vector<Scored>> fav;
        std::vector<std::vector<std::pair<int, Scored>>> picked;   // (rank, entry)
        std::vector<std::vector<double>> favD;
        select_round(act, fav, picked, favD);
        // Certified fast path: a ZMW whose round took a decision within its score bound -- k_reduce's
        // favourable test or fast-score break, or a BestSubset pick among float casts that the bound could reorder --
        // has its reads re-filled exactly and its round scored again on exact bands (its later rounds stay exact).
        if (rAmbOn_) {
            std::vector<int> ambFlag;
            download(ambFlag, ws_->wAmb, act.size(), stream_);
            PBCCS_HIP(hipStreamSynchronize(stream_));
            std::vector<int> redo;   // positions in act
            for (size_t a = 0; a < act.size(); ++a) {
                const double e = rDevItem_[a];
                if (e <= 0.0) continue;
                if (ambFlag[a] || !best_subset_certain(fav[a], favD[a], e, ro.mutationSeparation)) redo.push_back((int)a);
            }
            if (!redo.empty()) {
                std::vector<int> actR, readsR;
                std::vector<std::vector<int>> listsR;
                for (int a : redo) {
                    actR.push_back(act[a]);
                    if (round > 0) listsR.push_back(lists[a]);
                    const HZmw& z = zmws_[act[a]];
                    for (int q = 0; q < z.nReads; ++q) {
                        HRead& h = reads_[z.readBegin + q];
                        h.exact = true;
                        if (h.active) readsR.push_back(z.readBegin + q);
                    }
                }
                counters_.exactRounds += (long long)redo.size();
                FillReads(readsR);   // the same template and windows, now on the exact paths: the reference's bands
                for (int r : readsR)
                    if (reads_[r].status != kFillOk) reads_[r].active = false;
                descDirty_ = true;
                RunRound(actR, round == 0 ? nullptr : &listsR, fastThr, false, true);
                std::vector<std::vector<Scored>> favR;
                std::vector<std::vector<std::pair<int, Scored>>> pickedR;
                std::vector<std::vector<double>> favDR;
                select_round(actR, favR, pickedR, favDR);
                for (size_t i = 0; i < redo.size(); ++i) {
                    fav[redo[i]] = std::move(favR[i]);
                    picked[redo[i]] = std::move(pickedR[i]);
                }
            }
        }
        // PBCCS_CHECK_BEST_SUBSET=1: the host restatement beside the device select, any difference fatal
        const bool checkBest = std::getenv("PBCCS_CHECK_BEST_SUBSET") != nullptr;
        std::vector<int> changed, qvNow, qvIdx;
        for (size_t a = 0; a < act.size(); ++a) {
            const int k = idx[a];
            const int zi = act[a];
            memo[k].back().fav = fav[a];
            if (fav[a].empty()) {
                converged->at(k) = 1;
                done[k] = 1;
                if (qvsOnConverge) {
                    qvNow.push_back(zi);
                    qvIdx.push_back(k);
                }
                continue;
            }
            std::sort(picked[a].begin(), picked[a].end(),
                      [](const std::pair<int, Scored>& x, const std::pair<int, Scored>& y) { return x.first < y.first; });
            std::vector<Scored> best;
            for (const std::pair<int, Scored>& p : picked[a]) best.push_back(p.second);
            if (checkBest) {
                const std::vector<Scored> host = best_subset(fav[a], ro.mutationSeparation);
                bool same = host.size() == best.size();
                for (size_t i = 0; same && i < host.size(); ++i)
                    same = host[i].code == best[i].code && host[i].score == best[i].score;
                if (!same) throw DeviceError("k_best_subset differs from the host BestSubset");
            }
            std::vector<Mutation> muts;
            for (const Scored& s : best) muts.push_back(mutation_from_code(s.code));
            if (best.size() > 1) {
                std::string next;
                std::vector<int> mtp;
                if (apply_mutations(zmws_[zi].tpl, muts, &next, &mtp) && history[k].count(next)) {
                    best.resize(1);
                    muts.resize(1);
                }
            }
            (*nApplied)[k] += (long long)best.size();
            history[k].insert(zmws_[zi].tpl);
            centers[k].clear();
            for (const Scored& s : fav[a]) centers[k].push_back(mut_pos(s.code));
            // apply on the host; refills are batched below
            HZmw& z = zmws_[zi];
            std::vector<int> mtp;
            if (!apply_host(&z.tpl, muts, &mtp)) {
                done[k] = 1;   // the reference throws out of RefineConsensus here (ZMW -> Other)
                converged->at(k) = -1;
                if (retireDone) Retire({zi});
                continue;
            }
            UploadTemplate(zi);
            // NonConvergent after this iteration: the refill only matters to a caller that reads the final state
            const bool last = zit[k] + 1 >= ro.maxIterations;
            const bool refill = !(last && retireDone);
            for (int q = 0; q < z.nReads; ++q) {
                HRead& r = reads_[z.readBegin + q];
                r.ts = mtp[r.ts];
                r.te = mtp[r.te];
                if (r.active && refill) {
                    EnsureCapacity(z.readBegin + q);
                    changed.push_back(z.readBegin + q);
                }
            }
            if (!refill) Retire({zi});
            if (++zit[k] >= ro.maxIterations) done[k] = 1;   // NonConvergent
        }
        descDirty_ = true;
        // ConsensusQVs of the ZMWs that converged this round, from their final bands; after that (reclaim) their
        // bands are dead, so the refill below holds every live read and can lay the value pool out afresh
        if (!qvNow.empty()) {
            std::vector<std::vector<int>> q;
            QVs(qvNow, &q);
            for (size_t i = 0; i < qvNow.size(); ++i) (*qvsOnConverge)[qvIdx[i]] = std::move(q[i]);
            if (reclaim_) Retire(qvNow);
        }
        const Clock::time_point t2 = Clock::now();
        if (!changed.empty()) {
            FillReads(changed);
            for (int r : changed)
                if (reads_[r].status != kFillOk) reads_[r].active = false;
            descDirty_ = true;
        }
        if (roundTrace) {
            const Clock::time_point t3 = Clock::now();
            std::fprintf(stderr, "[round] batch=%p round=%d zmws=%zu muts=%lld refill=%zu prerefill=%zu replayed=%lld "
                                 "score=%.1fms select=%.1fms fill=%.1fms bandtop=%.2fGB\n",
                         (void*)this, round, act.size(), rTotalMut_, changed.size(), preRefill.size(), replayed,
                         ms(t0, t1), ms(t1, t2), ms(t2, t3), valTop_ * 8.0 / 1e9);
        }
    }
    if (!finalRefill.empty()) {   // the scorer API observes the final state: give replayed ZMWs their bands
        FillReads(finalRefill);
        for (int r : finalRefill)
            if (reads_[r].status != kFillOk) reads_[r].active = false;
        descDirty_ = true;
    }
}

// ------------------------------------------------------------------------------------------------
// ConsensusQVs
// ------------------------------------------------------------------------------------------------
void ArrowBatch::QVs(const std::vector<int>& zl, std::vector<std::vector<int>>* qvs)
{
    const StreamScope bound(stream_);
    RunRound(zl, nullptr, -std::numeric_limits<double>::max(), true);
    std::vector<long long> qvBase(zl.size());
    for (size_t k = 0; k < zl.size(); ++k) qvBase[k] = rPosStart_[k];
    upload(dWQvBase_, qvBase, stream_);
    dQv_.reserve(std::max<long long>(rTotalPos_, 1), false);
    ScoreWork W;
    W.nWork = (int)zl.size();
    W.zmw = dWZmw_.ptr;
    W.nMut = dWNMut_.ptr;
    W.mutBase = dWMutBase_.ptr;
    W.deltaBase = dWDeltaBase_.ptr;
    W.waveStart = dWWaveStart_.ptr;
    W.mutStart = dWMutStart_.ptr;
    W.posStart = dWPosStart_.ptr;
    W.codes = dCodes_.ptr;
    W.delta = dDelta_.ptr;
    const DevBatch B = View();
    Timed(kKQv, [&] {
        launch_qv(B, W, rTotalPos_, dWPosBase_.ptr, dPosOff_.ptr, dScore_.ptr, dWQvBase_.ptr, dQv_.ptr, stream_);
    });
    PBCCS_HIP(hipGetLastError());
    std::vector<int> q;
    download(q, dQv_, rTotalPos_, stream_);
    PBCCS_HIP(hipStreamSynchronize(stream_));
    qvs->assign(zl.size(), {});
    for (size_t k = 0; k < zl.size(); ++k) (*qvs)[k].assign(q.begin() + rPosStart_[k], q.begin() + rPosStart_[k + 1]);
}

}  // namespace pbccs
