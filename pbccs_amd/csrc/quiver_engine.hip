// pbccs_amd/csrc/quiver_engine.hip -- QuiverBatch (quiver_engine.hpp).
#include "quiver_engine.hpp"

#include <chrono>
#include <cstdio>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <set>
#include <stdexcept>
#include <thread>
#include <unordered_set>

#include "arrow_kernels.hpp"

namespace pbccs {
namespace quiver {
namespace {

#define QHIP(x)                                                              \
    do {                                                                     \
        hipError_t e_ = (x);                                                 \
        if (e_ != hipSuccess) throw DeviceError(hipGetErrorString(e_));      \
    } while (0)

template <class T>
void put(DevVec<T>& d, const std::vector<T>& h, hipStream_t s)
{
    d.reserve(std::max<size_t>(h.size(), 1), false);
    if (!h.empty()) QHIP(hipMemcpyAsync(d.ptr, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, s));
}

template <class T>
void get(std::vector<T>& h, const DevVec<T>& d, size_t n, hipStream_t s)
{
    h.resize(n);
    if (n) QHIP(hipMemcpyAsync(h.data(), d.ptr, n * sizeof(T), hipMemcpyDeviceToHost, s));
}

constexpr int kInitialBand = 24;   // values per column per arena to start with

// f(k) for k in [0, n) on up to 16 host threads, contiguous index ranges (scorers' independent host work:
// mutation lists, list flattening, template edits); the first exception is rethrown
template <class F>
void par_for(int n, F&& f, int minPerThread = 32)
{
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    const int nt = std::max(1, std::min(std::min(16, hw), n / std::max(1, minPerThread)));
    if (nt <= 1) {
        for (int k = 0; k < n; ++k) f(k);
        return;
    }
    std::exception_ptr err;
    std::mutex mu;
    auto run = [&](int t) {
        const int a = (int)((long long)n * t / nt), b = (int)((long long)n * (t + 1) / nt);
        try {
            for (int k = a; k < b; ++k) f(k);
        } catch (...) {
            std::lock_guard<std::mutex> lk(mu);
            if (!err) err = std::current_exception();
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(run, t);
    run(0);
    for (std::thread& x : th) x.join();
    if (err) std::rethrow_exception(err);
}

struct ScoredMut {
    int code;
    float score;
};

std::vector<ScoredMut> best_subset(std::vector<ScoredMut> in, int sep)   // Consensus-inl.hpp:98-118
{
    if (sep == 0) return in;
    std::vector<ScoredMut> out;
    while (!in.empty()) {
        size_t best = 0;
        for (size_t k = 1; k < in.size(); ++k)
            if (in[best].score < in[k].score) best = k;
        const ScoredMut b = in[best];
        out.push_back(b);
        const int lo = mut_pos(b.code) - sep, hi = mut_pos(b.code) + sep;
        std::vector<ScoredMut> keep;
        for (const ScoredMut& s : in)
            if (!(lo <= mut_pos(s.code) && mut_pos(s.code) <= hi)) keep.push_back(s);
        in.swap(keep);
    }
    return out;
}

}  // namespace

QuiverBatch::QuiverBatch(int device) : device_(device)
{
    QHIP(hipSetDevice(device_));
    QHIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    QHIP(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
    QHIP(hipEventCreateWithFlags(&evFork_, hipEventDisableTiming));
    QHIP(hipEventCreateWithFlags(&evJoin_, hipEventDisableTiming));
    dScratchTop_.reserve(1, false);
    dOverflow_.reserve(1, false);
    dScratch_.reserve(1 << 20, false);
}

QuiverBatch::~QuiverBatch()
{
    if (side_) {
        (void)hipStreamSynchronize(side_);
        (void)hipStreamDestroy(side_);
    }
    if (stream_) {
        (void)hipStreamSynchronize(stream_);
        (void)hipStreamDestroy(stream_);
    }
    if (evFork_) (void)hipEventDestroy(evFork_);
    if (evJoin_) (void)hipEventDestroy(evJoin_);
    for (const Pending& p : pending_) {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    for (hipEvent_t e : eventPool_) (void)hipEventDestroy(e);
}

void QuiverBatch::SetProfiling(bool on)
{
    profiling_ = on;
    if (on && !dStats_.ptr) {
        dStats_.reserve(8, false);
        QHIP(hipMemsetAsync(dStats_.ptr, 0, 8 * sizeof(unsigned long long), stream_));
    }
}

template <class F>
void QuiverBatch::Timed(KernelKind k, F&& launch, hipStream_t st)
{
    if (!profiling_) {
        launch();
        return;
    }
    hipEvent_t ev[2];
    for (int i = 0; i < 2; ++i) {
        if (!eventPool_.empty()) {
            ev[i] = eventPool_.back();
            eventPool_.pop_back();
        } else {
            QHIP(hipEventCreate(&ev[i]));
        }
    }
    QHIP(hipEventRecord(ev[0], st));
    launch();
    QHIP(hipEventRecord(ev[1], st));
    pending_.push_back({(int)k, ev[0], ev[1]});
    stats_[k].launches += 1;
}

void QuiverBatch::CollectProfile(KernelStat out[kKernelKinds])
{
    if (!pending_.empty()) {
        QHIP(hipStreamSynchronize(stream_));
        QHIP(hipStreamSynchronize(side_));
        for (const Pending& p : pending_) {
            float ms = 0.0f;
            if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) stats_[p.kind].ms += ms;
            else (void)hipGetLastError();
            eventPool_.push_back(p.a);
            eventPool_.push_back(p.b);
        }
        pending_.clear();
    }
    if (profiling_ && dStats_.ptr) {
        unsigned long long h[8];
        QHIP(hipMemcpyAsync(h, dStats_.ptr, sizeof(h), hipMemcpyDeviceToHost, stream_));
        QHIP(hipStreamSynchronize(stream_));
        const KernelKind kinds[3] = {kKQFillGrp, kKQFillCoop, kKQFillLane};
        for (int k = 0; k < 3; ++k) {
            stats_[kinds[k]].cells += (double)h[2 * k];
            stats_[kinds[k]].bytes += (double)h[2 * k + 1];
        }
        QHIP(hipMemsetAsync(dStats_.ptr, 0, sizeof(h), stream_));
        QHIP(hipStreamSynchronize(stream_));
    }
    for (int k = 0; k < kKernelKinds; ++k) {
        out[k].launches += stats_[k].launches;
        out[k].ms += stats_[k].ms;
        out[k].cells += stats_[k].cells;
        out[k].bytes += stats_[k].bytes;
        stats_[k] = KernelStat();
    }
}

void QuiverBatch::grow_scratch(unsigned long long requested)
{
    size_t want = std::max<size_t>((size_t)dScratch_.cap * 2, (size_t)(requested + requested / 8));
    dScratch_.reserve(want, false);
}

void QuiverBatch::Reset()
{
    QHIP(hipSetDevice(device_));
    QHIP(hipStreamSynchronize(stream_));
    // a call that threw between the side stream's tall fills and the join may have left them running: they
    // read the read list and the arenas this call is about to overwrite
    if (side_) QHIP(hipStreamSynchronize(side_));
    configs_.clear();
    zmws_.clear();
    reads_.clear();
    hSeq_.n = 0;
    hFeat_.n = 0;
    colTop_ = valTop_ = 0;
    seqUp_ = featUp_ = 0;
    dirty_ = true;
}

int QuiverBatch::AddConfig(const QParams& p)
{
    if (!(p.scoreDiff >= 0.0f)) throw std::invalid_argument("ScoreDiff must be positive");
    configs_.push_back(p);
    dirty_ = true;
    return (int)configs_.size() - 1;
}

int QuiverBatch::AddZmw(const std::string& tpl, float fastScoreThreshold)
{
    if (tpl.empty() || !is_acgt(tpl)) throw std::invalid_argument("template must be a non-empty ACGT string");
    HZmw z;
    z.tpl = tpl;
    z.fastThreshold = fastScoreThreshold;
    zmws_.push_back(z);
    dirty_ = true;
    return (int)zmws_.size() - 1;
}

void QuiverBatch::EnsureCapacity(int ri)
{
    HRead& r = reads_[ri];
    const int J = r.te - r.ts;
    if (J + 1 > r.colCap) {
        r.colCap = J + J / 4 + 16;
        r.colBase = colTop_;
        colTop_ += 4LL * r.colCap;
        dirty_ = true;
    }
    const long long want = (long long)(J + 1) * kInitialBand;
    if (r.valCap < want) {
        r.valCap = want + want / 4;
        r.valBase = valTop_;
        valTop_ += 4 * r.valCap;
        dirty_ = true;
    }
}

bool QuiverBatch::AddRead(int zi, const QReadFeatures& f, int strand, int ts, int te, int config, float threshold)
{
    std::vector<ReadSpec> one(1);
    one[0].z = zi;
    one[0].strand = strand;
    one[0].ts = ts;
    one[0].te = te;
    one[0].config = config;
    one[0].threshold = threshold;
    const size_t I = f.seq.size();
    if (f.ins.size() != I || f.subs.size() != I || f.del.size() != I || f.tag.size() != I || f.merge.size() != I)
        throw std::invalid_argument("QV feature tracks must match the read length");
    one[0].seq = f.seq.data();
    one[0].len = (int)I;
    const float* const track[5] = {f.ins.data(), f.subs.data(), f.del.data(), f.tag.data(), f.merge.data()};
    for (int k = 0; k < 5; ++k) one[0].track[k] = track[k];
    return AddReads(&one)[0] != 0;
}

std::vector<char> QuiverBatch::AddReads(std::vector<ReadSpec>* specs)
{
    // the host pools grow once, then the reads' bases and QV tracks (~4 GB for a 10000-scorer batch) are copied in
    // on several host threads
    static const bool trace = std::getenv("PBCCS_QUIVER_TRACE") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    const size_t ns = specs->size();
    std::vector<long long> seqOff(ns);
    size_t bases = 0;
    for (size_t k = 0; k < ns; ++k) {   // every spec is checked before the pools grow
        const ReadSpec& sp = (*specs)[k];
        const int L = (int)zmws_.at(sp.z).tpl.size();
        if (sp.len < 1 || !sp.seq || sp.ts < 0 || sp.te > L || sp.ts > sp.te || sp.config < 0 ||
            sp.config >= (int)configs_.size())
            throw std::invalid_argument("read without bases, window outside the template or bad config");
        seqOff[k] = (long long)(hSeq_.size() + bases);
        bases += (size_t)sp.len;
    }
    const size_t s0 = hSeq_.grow(bases);
    hFeat_.grow(5 * bases);
    const auto tGrow = std::chrono::steady_clock::now();
    auto copy = [&](size_t k) {
        const ReadSpec& sp = (*specs)[k];
        const size_t I = (size_t)sp.len, so = (size_t)seqOff[k];
        std::memcpy(hSeq_.data() + so, sp.seq, I);
        for (int t = 0; t < 5; ++t) {   // track t of read k at 5 * seqOff + t * len (ReadView's layout)
            float* dst = hFeat_.data() + 5 * so + (size_t)t * I;
            if (sp.track[t]) std::memcpy(dst, sp.track[t], I * sizeof(float));
            else std::memset(dst, 0, I * sizeof(float));
        }
    };
    (void)s0;
    {
        const int nt = (int)std::max<size_t>(1, std::min<size_t>(16, std::min<size_t>(ns / 64 + 1, std::thread::hardware_concurrency())));
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t)
            th.emplace_back([&, t] { for (size_t k = t; k < ns; k += nt) copy(k); });
        for (size_t k = 0; k < ns; k += nt) copy(k);
        for (std::thread& x : th) x.join();
    }
    const auto tCopy = std::chrono::steady_clock::now();
    std::vector<int> added;
    for (size_t k = 0; k < ns; ++k) {
        const ReadSpec& sp = (*specs)[k];
        added.push_back(RegisterRaw(sp.z, seqOff[k], sp.len, sp.strand, sp.ts, sp.te, sp.config));
    }
    const auto t1 = std::chrono::steady_clock::now();
    Upload();
    const auto t2 = std::chrono::steady_clock::now();
    Fill(added);
    if (trace)
        std::fprintf(stderr, "[quiver] addreads %zu register %.1f ms (grow %.1f copy %.1f) upload %.1f ms fill %.1f ms\n",
                     added.size(), std::chrono::duration<double, std::milli>(t1 - t0).count(),
                     std::chrono::duration<double, std::milli>(tGrow - t0).count(),
                     std::chrono::duration<double, std::milli>(tCopy - tGrow).count(),
                     std::chrono::duration<double, std::milli>(t2 - t1).count(),
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t2).count());
    std::vector<char> act(specs->size());
    for (size_t k = 0; k < specs->size(); ++k) {
        // AddRead: a scorer whose construction threw (alpha/beta mismatch) is dropped; so is one whose
        // matrices allocate more than `threshold` of the full matrix (:263-276)
        HRead& h = reads_[added[k]];
        const float threshold = (*specs)[k].threshold;
        h.hasScorer = h.active;
        if (h.active && threshold < 1.0f) {
            const int J = h.te - h.ts;
            // float threshold * int * int is float; 0.5 + float is double (:268)
            const int maxSize = static_cast<int>(0.5 + threshold * (float)(int)(h.len + 1) * (float)(J + 1));
            if (h.alloc[0] >= maxSize || h.alloc[1] >= maxSize) h.active = h.hasScorer = false;
        }
        act[k] = h.active ? 1 : 0;
    }
    return act;
}

int QuiverBatch::RegisterRaw(int zi, long long seqOff, int len, int strand, int ts, int te, int config)
{
    HZmw& z = zmws_.at(zi);
    const int L = (int)z.tpl.size();
    const size_t I = (size_t)std::max(0, len);
    if (ts < 0 || te > L || ts > te || len < 1 || config < 0 || config >= (int)configs_.size())
        throw std::invalid_argument("read window outside the template or bad config");
    HRead r;
    r.zmw = zi;
    r.config = config;
    r.strand = strand;
    r.ts = ts;
    r.te = te;
    r.len = (int)I;
    r.seqOff = seqOff;
    r.colBuf = -1;
    reads_.push_back(r);
    const int ri = (int)reads_.size() - 1;
    z.reads.push_back(ri);
    HRead& h = reads_[ri];
    h.colBuf = valTop_;
    valTop_ += (long long)I + 8;
    EnsureCapacity(ri);
    dirty_ = true;
    return ri;
}

void QuiverBatch::Upload()
{
    if (!dirty_) return;
    std::vector<long long> zf, zr;
    std::vector<int> zl;
    std::vector<char> tp;
    for (const HZmw& z : zmws_) {
        zf.push_back((long long)tp.size());
        tp.insert(tp.end(), z.tpl.begin(), z.tpl.end());
        tp.push_back('\0');
        const std::string rc = reverse_complement(z.tpl);
        zr.push_back((long long)tp.size());
        tp.insert(tp.end(), rc.begin(), rc.end());
        tp.push_back('\0');
        zl.push_back((int)z.tpl.size());
    }
    const size_t R = reads_.size();
    std::vector<int> rz(R), rp(R), rs(R), rts(R), rte(R), rl(R), rcc(R);
    std::vector<long long> rso(R), rcb(R), rvb(R), rvc(R), rcbuf(R);
    for (size_t i = 0; i < R; ++i) {
        const HRead& r = reads_[i];
        rz[i] = r.zmw;
        rp[i] = r.config;
        rs[i] = r.strand;
        rts[i] = r.ts;
        rte[i] = r.te;
        rso[i] = r.seqOff;
        rcb[i] = r.colBase;
        rcc[i] = r.colCap;
        rvb[i] = r.valBase;
        rvc[i] = r.valCap;
        rcbuf[i] = r.colBuf;
    }
    for (size_t i = 0; i < R; ++i) {
        const HRead& r = reads_[i];
        const size_t I = (i + 1 < R ? reads_[i + 1].seqOff : (long long)hSeq_.size()) - r.seqOff;
        rl[i] = (int)I;
    }
    put(dZFwd_, zf, stream_);
    put(dZRev_, zr, stream_);
    put(dZLen_, zl, stream_);
    put(dTpl_, tp, stream_);
    put(dParams_, configs_, stream_);
    put(dRZmw_, rz, stream_);
    put(dRParam_, rp, stream_);
    put(dRStrand_, rs, stream_);
    put(dRTs_, rts, stream_);
    put(dRTe_, rte, stream_);
    put(dRLen_, rl, stream_);
    put(dRSeq_, rso, stream_);
    put(dRColBase_, rcb, stream_);
    put(dRColCap_, rcc, stream_);
    put(dRValBase_, rvb, stream_);
    put(dRValCap_, rvc, stream_);
    put(dRColBuf_, rcbuf, stream_);
    // the read pools only ever grow (AddRead appends): upload the new tail, not every read's bases and five
    // feature tracks again on each refine round that edits a template
    auto tail = [&](auto& d, const auto& h, size_t& up) {
        if (h.size() < up) up = 0;   // never happens (append-only); re-upload if it did
        if (h.size() == up) return;
        d.reserve(std::max<size_t>(h.size(), 1), true);
        QHIP(hipMemcpyAsync(d.ptr + up, h.data() + up, (h.size() - up) * sizeof(*h.data()), hipMemcpyHostToDevice,
                            stream_));
        up = h.size();
    };
    tail(dSeq_, hSeq_, seqUp_);
    tail(dFeat_, hFeat_, featUp_);
    dRange_.reserve(std::max<long long>(colTop_, 1), true);
    dOff_.reserve(std::max<long long>(colTop_, 1), true);
    dAlloc_.reserve(std::max<long long>(colTop_ / 2, 1), true);
    dHint_.reserve(std::max<long long>(colTop_ / 4 + 1, 1), false);
    dVal_.reserve(std::max<long long>(valTop_, 1), true);
    dRCurA_.reserve(std::max<size_t>(R, 1), true);
    dRCurB_.reserve(std::max<size_t>(R, 1), true);
    dRScore_.reserve(std::max<size_t>(R, 1), true);
    dRFlips_.reserve(std::max<size_t>(R, 1), true);
    dRStatus_.reserve(std::max<size_t>(R, 1), true);
    dRUsed_.reserve(std::max<size_t>(2 * R, 1), true);
    dRAlloc_.reserve(std::max<size_t>(2 * R, 1), true);
    QHIP(hipStreamSynchronize(stream_));
    dirty_ = false;
}

QBatch QuiverBatch::View()
{
    QBatch b;
    b.zFwd = dZFwd_.ptr;
    b.zRev = dZRev_.ptr;
    b.zLen = dZLen_.ptr;
    b.tplPool = dTpl_.ptr;
    b.params = dParams_.ptr;
    b.rZmw = dRZmw_.ptr;
    b.rParam = dRParam_.ptr;
    b.rStrand = dRStrand_.ptr;
    b.rTs = dRTs_.ptr;
    b.rTe = dRTe_.ptr;
    b.rLen = dRLen_.ptr;
    b.rSeq = dRSeq_.ptr;
    b.seqPool = dSeq_.ptr;
    b.featPool = dFeat_.ptr;
    b.rColBase = dRColBase_.ptr;
    b.rColCap = dRColCap_.ptr;
    b.rValBase = dRValBase_.ptr;
    b.rValCap = dRValCap_.ptr;
    b.rColBuf = dRColBuf_.ptr;
    b.range = dRange_.ptr;
    b.off = dOff_.ptr;
    b.alloc = dAlloc_.ptr;
    b.hint = dHint_.ptr;
    b.valPool = dVal_.ptr;
    b.rCurA = dRCurA_.ptr;
    b.rCurB = dRCurB_.ptr;
    b.rScore = dRScore_.ptr;
    b.rFlips = dRFlips_.ptr;
    b.rStatus = dRStatus_.ptr;
    b.rUsed = dRUsed_.ptr;
    b.rAlloc = dRAlloc_.ptr;
    b.stats = profiling_ ? dStats_.ptr : nullptr;
    return b;
}

// MutationScorer ctor / Template(): FillAlphaBeta; grows a read's arenas and re-runs it on overflow.
void QuiverBatch::Fill(const std::vector<int>& readsIn)
{
    std::vector<int> todo(readsIn);
    for (int attempt = 0; !todo.empty(); ++attempt) {
        if (attempt > 8) throw DeviceError("quiver band storage keeps overflowing");
        Upload();
        // SparseSse configs with reads below kQCoopRows rows: one wavefront per read (k_qfill_coop); the
        // Simple / Dense recursors and longer reads: one lane per read (k_qfill).  PBCCS_QFILL_LANE=1 sends
        // every read to the lane kernel.
        // The coop kernel's LDS ring holds kQRingRows rows per column (band height, rows modulo the ring), so
        // many read waves share a CU; a read with a taller column comes back kQTall and from then on fills with
        // a ring of its full height (tallRing).
        // SparseSse reads go to k_qfill_grp first (four reads per wavefront, a 64-row band ring); a read that
        // comes back kQTall moves to k_qfill_coop's band-height ring, then to its full-height ring.
        std::vector<int> grp, coop, full, lane;
        int maxCols = 1, maxColsFull = 1, maxRowsFull = 1;
        for (int r : todo) {
            const QParams& p = configs_[reads_[r].config];
            const int cols = reads_[r].te - reads_[r].ts + 1;
            if (!p.simple && !p.dense && reads_[r].len + 1 <= kQCoopRows && cols <= kQCoopCols) {
                if (reads_[r].tallRing) {
                    full.push_back(r);
                    maxRowsFull = std::max(maxRowsFull, reads_[r].len + 1);
                    maxColsFull = std::max(maxColsFull, cols);
                } else if (reads_[r].grpTall) {
                    coop.push_back(r);
                    maxCols = std::max(maxCols, cols);
                } else {
                    grp.push_back(r);
                }
            } else {
                lane.push_back(r);
            }
        }
        // k_qfill_grp's list: each QuiverConfig's reads in whole waves of four (-1 pads), so a wave's parameters
        // are one config's
        std::vector<int> grpList;
        {
            std::stable_sort(grp.begin(), grp.end(),
                             [&](int a, int b) { return reads_[a].config < reads_[b].config; });
            for (size_t k = 0; k < grp.size(); ++k) {
                if (k > 0 && reads_[grp[k]].config != reads_[grp[k - 1]].config)
                    while (grpList.size() % 4) grpList.push_back(-1);
                grpList.push_back(grp[k]);
            }
            while (grpList.size() % 4) grpList.push_back(-1);
        }
        std::vector<int> both(grpList);
        both.insert(both.end(), coop.begin(), coop.end());
        both.insert(both.end(), full.begin(), full.end());
        both.insert(both.end(), lane.begin(), lane.end());
        put(dList_, both, stream_);
        const QBatch B = View();
        constexpr int ringRows = kQRingRows;   // a power of two (128 / 256 / 512 / 1024 measured, quiver_kernels.hpp)
        static_assert((kQRingRows & (kQRingRows - 1)) == 0, "the band ring is a power of two of rows");
        const size_t g0 = grpList.size();
        // the coop lists (reads that were tall for k_qfill_grp) on the side stream, concurrently with the grouped
        // launch; both streams join before the status download
        const bool sideRun = !coop.empty() || !full.empty();
        if (sideRun) {
            QHIP(hipEventRecord(evFork_, stream_));   // after the uploads above
            QHIP(hipStreamWaitEvent(side_, evFork_, 0));
            if (!coop.empty())
                Timed(kKQFillCoop, [&] { launch_qfill_coop(B, dList_.ptr + g0, (int)coop.size(), ringRows, maxCols, side_); },
                      side_);
            if (!full.empty())
                Timed(kKQFillCoop, [&] {
                    launch_qfill_coop(B, dList_.ptr + g0 + coop.size(), (int)full.size(), maxRowsFull, maxColsFull, side_);
                }, side_);
            QHIP(hipGetLastError());
            QHIP(hipEventRecord(evJoin_, side_));
        }
        if (!grpList.empty()) Timed(kKQFillGrp, [&] { launch_qfill_grp(B, dList_.ptr, (int)grpList.size(), stream_); }, stream_);
        if (!lane.empty())
            Timed(kKQFillLane, [&] { launch_qfill(B, dList_.ptr + g0 + coop.size() + full.size(), (int)lane.size(), stream_); },
                  stream_);
        if (sideRun) QHIP(hipStreamWaitEvent(stream_, evJoin_, 0));
        QHIP(hipGetLastError());
        const size_t R = reads_.size();
        std::vector<int> st, ca, cb, fl;
        std::vector<float> sc;
        std::vector<long long> used, al;
        get(st, dRStatus_, R, stream_);
        get(ca, dRCurA_, R, stream_);
        get(cb, dRCurB_, R, stream_);
        get(fl, dRFlips_, R, stream_);
        get(sc, dRScore_, R, stream_);
        get(used, dRUsed_, 2 * R, stream_);
        get(al, dRAlloc_, 2 * R, stream_);
        QHIP(hipStreamSynchronize(stream_));
        std::vector<int> next;
        static const bool trace = std::getenv("PBCCS_QFILL_TRACE") != nullptr;   // one stderr line per launch set
        int tallG = 0, tallR = 0;
        // a read too tall for the grouped kernel's 64-row ring goes straight to the full-height ring: most of
        // them outgrow the 128-row band ring as well (round 0 of the Quiver bench: 43 of 46), and each step down
        // the paths is one more serial launch on the round's critical path
        for (int r : grp)
            if (st[r] == kQTall) { reads_[r].grpTall = reads_[r].tallRing = true; tallG++; }
        for (int r : coop)
            if (st[r] == kQTall) { reads_[r].tallRing = true; tallR++; }
        if (trace)
            std::fprintf(stderr, "[qfill] attempt %d grp %zu ring %zu full %zu lane %zu -> tall %d / %d\n", attempt,
                         grp.size(), coop.size(), full.size(), lane.size(), tallG, tallR);
        for (int r : todo) {
            HRead& h = reads_[r];
            if (st[r] == kQTall) {
                next.push_back(r);
                continue;
            }
            if (st[r] == kQOverflow) {
                // the need covers the passes run before the overflow stopped the schedule; a tall read's later
                // flip-flop passes tend to need more, so it grows by 2x (each retry is a whole refill)
                const long long need = std::max(used[2 * r], used[2 * r + 1]);
                h.valCap = std::max(h.tallRing ? 2 * need + 64 : need + need / 4 + 64, h.valCap + 1);
                h.valBase = valTop_;
                valTop_ += 4 * h.valCap;
                dirty_ = true;
                next.push_back(r);
                continue;
            }
            h.active = st[r] == kQOk;   // AlphaBetaMismatchException -> no scorer / inactive
            h.curA = ca[r];
            h.curB = cb[r];
            h.flips = fl[r];
            h.score = sc[r];
            h.alloc[0] = al[2 * r];
            h.alloc[1] = al[2 * r + 1];
        }
        todo.swap(next);
    }
    // the device copies of curA / curB are what k_qscore reads: they were written by the kernel itself
}

void QuiverBatch::Deltas(int zi, const std::vector<int>& codes, std::vector<float>* out)
{
    // the batched scoring path (k_qscore_mid + the listed edge cases) over one item: NaN for inactive reads
    // and for reads that do not score a mutation, as MultiReadMutationScorer::Score skips them
    const HZmw& z = zmws_.at(zi);
    const long long nt = (long long)codes.size() * (long long)z.reads.size();
    out->assign((size_t)nt, std::numeric_limits<float>::quiet_NaN());
    if (nt == 0) return;
    std::vector<long long> taskStart, mutStart;
    ScoreDeltas({zi}, {codes}, &taskStart, &mutStart);
    get(*out, dDelta_, (size_t)nt, stream_);
    QHIP(hipStreamSynchronize(stream_));
}

void QuiverBatch::RunScore(const std::vector<int>& tr, const std::vector<int>& tm, const std::vector<int>& codes,
                           bool raw, std::vector<float>* out)
{
    Upload();
    put(dTaskRead_, tr, stream_);
    put(dTaskMut_, tm, stream_);
    put(dCodes_, codes, stream_);
    dDelta_.reserve(std::max<size_t>(tr.size(), 1), false);
    for (int attempt = 0;; ++attempt) {
        QHIP(hipMemsetAsync(dScratchTop_.ptr, 0, sizeof(unsigned long long), stream_));
        QHIP(hipMemsetAsync(dOverflow_.ptr, 0, sizeof(int), stream_));
        QScoreWork W;
        W.taskRead = dTaskRead_.ptr;
        W.taskMut = dTaskMut_.ptr;
        W.codes = dCodes_.ptr;
        W.delta = dDelta_.ptr;
        W.scratch = dScratch_.ptr;
        W.scratchTop = dScratchTop_.ptr;
        W.scratchCap = dScratch_.cap;
        W.overflow = dOverflow_.ptr;
        W.nTasks = (long long)tr.size();
        W.raw = raw ? 1 : 0;
        launch_qscore(View(), W, stream_);
        QHIP(hipGetLastError());
        int ovf = 0;
        unsigned long long top = 0;
        QHIP(hipMemcpyAsync(&ovf, dOverflow_.ptr, sizeof(int), hipMemcpyDeviceToHost, stream_));
        QHIP(hipMemcpyAsync(&top, dScratchTop_.ptr, sizeof(top), hipMemcpyDeviceToHost, stream_));
        QHIP(hipStreamSynchronize(stream_));
        if (!ovf) break;
        if ((ovf & 2) || attempt > 6) throw DeviceError("quiver extend buffer exceeds 8 columns / scratch");
        grow_scratch(top);
    }
    get(*out, dDelta_, tr.size(), stream_);
    QHIP(hipStreamSynchronize(stream_));
}

float QuiverBatch::ReadScoreMutation(int r, int code)
{
    if (!reads_.at(r).hasScorer) return 0.0f;
    std::vector<float> d;
    RunScore({r}, {0}, {code}, true, &d);
    return d[0];
}

// Score / FastScore (Quiver/MultiReadMutationScorer.cpp:312-353): float sum in read order; NaN = the read
// does not score the mutation (or is inactive).
float QuiverBatch::Score(int zi, const std::vector<float>& deltas, int m, bool fast) const
{
    const HZmw& z = zmws_[zi];
    const int nr = (int)z.reads.size();
    float sum = 0;
    for (int k = 0; k < nr; ++k) {
        const float d = deltas[(size_t)m * nr + k];
        if (std::isnan(d)) continue;
        sum += d;
        if (fast && sum < z.fastThreshold) return sum;
    }
    return sum;
}

bool QuiverBatch::FastIsFavorable(int zi, const std::vector<float>& deltas, int m) const   // :392-409
{
    const HZmw& z = zmws_[zi];
    const int nr = (int)z.reads.size();
    float sum = 0;
    for (int k = 0; k < nr; ++k) {
        const float d = deltas[(size_t)m * nr + k];
        if (std::isnan(d)) continue;
        sum += d;
        if (sum < z.fastThreshold) return false;
    }
    return (double)sum > 0.04;   // MIN_FAVORABLE_SCOREDIFF (:52), a double
}

float QuiverBatch::BaselineScore(int zi) const   // :467-476
{
    float sum = 0;
    for (int r : zmws_[zi].reads)
        if (reads_[r].active) sum += reads_[r].score;
    return sum;
}

bool QuiverBatch::ApplyMutations(int zi, const std::vector<Mutation>& muts)   // :205-239
{
    HZmw& z = zmws_.at(zi);
    std::string next;
    std::vector<int> mtp;
    if (!apply_mutations(z.tpl, muts, &next, &mtp)) return false;
    z.tpl = next;
    std::vector<int> refill;
    for (int r : z.reads) {
        HRead& h = reads_[r];
        h.ts = mtp[h.ts];
        h.te = mtp[h.te];
        if (h.active) {
            EnsureCapacity(r);
            refill.push_back(r);
        }
    }
    dirty_ = true;
    Fill(refill);   // a refill that mismatches marks the read inactive
    return true;
}

// AbstractRefineConsensus (Consensus-inl.hpp:159-251) with Quiver's float scores.
bool QuiverBatch::Refine(int zi, const RefineOptions& ro, long long* nTested, long long* nApplied, bool* converged)
{
    *nTested = 0;
    *nApplied = 0;
    *converged = false;
    std::set<std::string> history;
    std::vector<int> centers;
    for (int iter = 0; iter < ro.maxIterations; ++iter) {
        const std::string tpl = zmws_[zi].tpl;
        std::vector<int> codes;
        if (iter == 0) unique_mutations(tpl, 0, (int)tpl.size(), &codes);
        else nearby_mutations(tpl, centers, ro.mutationNeighborhood, &codes);
        *nTested += (long long)codes.size();
        std::vector<float> d;
        Deltas(zi, codes, &d);
        std::vector<ScoredMut> fav;
        for (int m = 0; m < (int)codes.size(); ++m)
            if (FastIsFavorable(zi, d, m)) fav.push_back({codes[m], Score(zi, d, m, false)});
        if (fav.empty()) {
            *converged = true;
            break;
        }
        std::vector<ScoredMut> best = best_subset(fav, ro.mutationSeparation);
        std::vector<Mutation> muts;
        for (const ScoredMut& s : best) muts.push_back(mutation_from_code(s.code));
        if (best.size() > 1) {
            std::string nx;
            std::vector<int> mtp;
            if (apply_mutations(tpl, muts, &nx, &mtp) && history.count(nx)) {
                best.resize(1);
                muts.resize(1);
            }
        }
        *nApplied += (long long)best.size();
        history.insert(tpl);
        centers.clear();
        for (const ScoredMut& s : fav) centers.push_back(mut_pos(s.code));
        if (!ApplyMutations(zi, muts)) return false;
    }
    return true;
}

bool QuiverBatch::Alignment(int r, std::string* target, std::string* query)
{
    const HRead& h = reads_.at(r);
    if (!h.hasScorer || configs_[h.config].sumProduct) return false;   // Viterbi only (ShouldNotReachHere)
    Upload();
    const int I = h.len, J = h.te - h.ts;
    put(dList_, std::vector<int>{r}, stream_);
    put(dMoveOff_, std::vector<long long>{0}, stream_);
    dMoves_.reserve((size_t)I + J + 1, false);
    // the move count has its own buffer: dOff_ is the bands' column offsets (QBatch::off), which the count once
    // overwrote (column 0 of the first arena), so a second Alignment of the read walked a damaged band
    dNMoves_.reserve(1, false);
    launch_qalign(View(), dList_.ptr, 1, dMoveOff_.ptr, dMoves_.ptr, dNMoves_.ptr, stream_);
    QHIP(hipGetLastError());
    int n = 0;
    QHIP(hipMemcpyAsync(&n, dNMoves_.ptr, sizeof(int), hipMemcpyDeviceToHost, stream_));
    QHIP(hipStreamSynchronize(stream_));
    if (n < 0) throw DeviceError("quiver alignment: no valid move (alpha not filled?)");
    std::vector<unsigned char> mv(n);
    if (n) QHIP(hipMemcpy(mv.data(), dMoves_.ptr, n, hipMemcpyDeviceToHost));
    // replay from the start (the moves are stored from the end) into the gapped strings (:228-262)
    const std::string& tpl0 = zmws_[h.zmw].tpl;
    const int L = (int)tpl0.size();
    const std::string tpl = h.strand == 0 ? tpl0.substr(h.ts, J) : reverse_complement(tpl0).substr(L - h.te, J);
    const char* seq = hSeq_.data() + h.seqOff;
    target->clear();
    query->clear();
    int i = 0, j = 0;
    for (int k = n - 1; k >= 0; --k) {
        switch (mv[k]) {
            case 1: *target += tpl[j]; *query += seq[i]; i++; j++; break;
            case 2: *target += '-'; *query += seq[i]; i++; break;
            case 4: *target += tpl[j]; *query += '-'; j++; break;
            default: *target += tpl[j]; *target += tpl[j + 1]; *query += '-'; *query += seq[i]; i++; j += 2; break;
        }
    }
    return true;
}

std::vector<int> QuiverBatch::QVs(int zi)   // ConsensusQVs (Consensus-inl.hpp:274-295), the batched device path
{
    return QVsMany({zi})[0];
}


// ---- batched rounds ---------------------------------------------------------------------------------------
// Tasks per scorer laid out [mutation][read] (the Deltas layout), scored in launches of at most kTaskChunk
// tasks so that the extend buffers' bump scratch stays bounded; then k_qreduce (Score / FastIsFavorable),
// hipCUB compaction of the favourable list and k_best_subset (BestSubset) on the device.
constexpr long long kTaskChunk = 1LL << 21;

// Every (mutation, read) delta of the listed scorers into dDelta_, laid out [item][mutation][read] from
// taskStart[w]; the item tables stay on the device for k_qreduce.
void QuiverBatch::ScoreDeltas(const std::vector<int>& zs, const std::vector<std::vector<int>>& codes,
                              std::vector<long long>* taskStartOut, std::vector<long long>* mutStartOut)
{
    static const bool trace = std::getenv("PBCCS_QUIVER_TRACE") != nullptr;
    using Clock = std::chrono::steady_clock;
    auto msSince = [](Clock::time_point a) { return std::chrono::duration<double, std::milli>(Clock::now() - a).count(); };
    const Clock::time_point ts0 = Clock::now();
    const int n = (int)zs.size();
    std::vector<long long>& taskStart = *taskStartOut;
    std::vector<long long>& mutStart = *mutStartOut;
    taskStart.assign(n + 1, 0);
    mutStart.assign(n + 1, 0);
    std::vector<int> readBase(n), nReads(n), readList;
    std::vector<float> fastThr(n);
    for (int w = 0; w < n; ++w) {
        const HZmw& z = zmws_[zs[w]];
        readBase[w] = (int)readList.size();
        nReads[w] = (int)z.reads.size();
        readList.insert(readList.end(), z.reads.begin(), z.reads.end());
        fastThr[w] = z.fastThreshold;
        mutStart[w + 1] = mutStart[w] + (long long)codes[w].size();
        taskStart[w + 1] = taskStart[w] + (long long)codes[w].size() * nReads[w];
    }
    hCodes_.n = 0;   // the scorers' lists back to back (the previous round's upload has completed)
    hCodes_.grow((size_t)mutStart[n]);
    par_for(n, [&](int w) {
        if (!codes[w].empty())
            std::memcpy(hCodes_.data() + mutStart[w], codes[w].data(), codes[w].size() * sizeof(int));
    });
    const long long nTask = taskStart[n];
    std::vector<int> active(reads_.size());
    for (size_t r = 0; r < reads_.size(); ++r) active[r] = reads_[r].active ? 1 : 0;
    Upload();
    put(dWTaskStart_, taskStart, stream_);
    std::vector<long long> mutBase(mutStart.begin(), mutStart.begin() + n);
    put(dWMutBase_, mutStart, stream_);
    put(dWReadBase_, readBase, stream_);
    put(dWNReads_, nReads, stream_);
    put(dReadList_, readList, stream_);
    put(dRActive_, active, stream_);
    put(dWFast_, fastThr, stream_);
    dCodes_.reserve(std::max<size_t>(hCodes_.size(), 1), false);
    if (hCodes_.size())
        QHIP(hipMemcpyAsync(dCodes_.ptr, hCodes_.data(), hCodes_.size() * sizeof(int), hipMemcpyHostToDevice, stream_));
    dDelta_.reserve(std::max<long long>(nTask, 1), false);
    const double msPrep = msSince(ts0);
    const Clock::time_point ts1 = Clock::now();
    // middle cases: k_qscore_mid, one wave per (item, read, 64-mutation chunk); it lists the edge cases
    std::vector<long long> waveStart(n + 1, 0), mutCount(n);
    long long edgeCap = 1024;
    for (int w = 0; w < n; ++w) {
        mutCount[w] = mutStart[w + 1] - mutStart[w];
        waveStart[w + 1] = waveStart[w] + (mutCount[w] > 0 ? (long long)nReads[w] * ((mutCount[w] + 63) / 64) : 0);
        edgeCap += (long long)nReads[w] * std::min<long long>(mutCount[w], 160);   // ~7 edge positions per read
    }
    put(dWaveStart_, waveStart, stream_);
    put(dWMutCount_, mutCount, stream_);
    dEdgeCount_.reserve(1, false);
    unsigned long long nEdge = 0;
    for (int attempt = 0;; ++attempt) {
        dEdge_.reserve(std::max<long long>(edgeCap, 1), false);
        QHIP(hipMemsetAsync(dEdgeCount_.ptr, 0, sizeof(unsigned long long), stream_));
        QMidWork MW;
        MW.nWork = n;
        MW.waveStart = dWaveStart_.ptr;
        MW.wTaskStart = dWTaskStart_.ptr;
        MW.wMutBase = dWMutBase_.ptr;
        MW.wMutCount = dWMutCount_.ptr;
        MW.wReadBase = dWReadBase_.ptr;
        MW.wNReads = dWNReads_.ptr;
        MW.readList = dReadList_.ptr;
        MW.rActive = dRActive_.ptr;
        MW.codes = dCodes_.ptr;
        MW.delta = dDelta_.ptr;
        MW.edgeList = dEdge_.ptr;
        MW.edgeCount = dEdgeCount_.ptr;
        MW.edgeCap = edgeCap;
        Timed(kKQScoreMid, [&] { launch_qscore_mid(View(), MW, waveStart[n], stream_); }, stream_);
        QHIP(hipGetLastError());
        QHIP(hipMemcpyAsync(&nEdge, dEdgeCount_.ptr, sizeof(nEdge), hipMemcpyDeviceToHost, stream_));
        QHIP(hipStreamSynchronize(stream_));
        if ((long long)nEdge <= edgeCap) break;
        if (attempt > 2) throw DeviceError("quiver edge-case list overflow");
        edgeCap = (long long)nEdge;   // the list was cut short: rerun with room for every edge case
    }
    const double msMid = msSince(ts1);
    const Clock::time_point ts2 = Clock::now();
    // edge cases (ExtendAlpha to the end, ExtendBeta, whole fills): k_qscore over the listed tasks
    for (long long t0 = 0; t0 < (long long)nEdge;) {
        const long long m = std::min(kTaskChunk, (long long)nEdge - t0);
        for (int attempt = 0;; ++attempt) {
            QHIP(hipMemsetAsync(dScratchTop_.ptr, 0, sizeof(unsigned long long), stream_));
            QHIP(hipMemsetAsync(dOverflow_.ptr, 0, sizeof(int), stream_));
            QScoreWork W;
            W.codes = dCodes_.ptr;
            W.delta = dDelta_.ptr;
            W.scratch = dScratch_.ptr;
            W.scratchTop = dScratchTop_.ptr;
            W.scratchCap = dScratch_.cap;
            W.overflow = dOverflow_.ptr;
            W.nTasks = m;
            W.raw = 0;
            W.nWork = n;
            W.taskBase = 0;
            W.taskList = dEdge_.ptr + t0;
            W.wTaskStart = dWTaskStart_.ptr;
            W.wMutBase = dWMutBase_.ptr;
            W.wReadBase = dWReadBase_.ptr;
            W.wNReads = dWNReads_.ptr;
            W.readList = dReadList_.ptr;
            W.rActive = dRActive_.ptr;
            launch_qscore(View(), W, stream_);
            QHIP(hipGetLastError());
            int ovf = 0;
            unsigned long long top = 0;
            QHIP(hipMemcpyAsync(&ovf, dOverflow_.ptr, sizeof(int), hipMemcpyDeviceToHost, stream_));
            QHIP(hipMemcpyAsync(&top, dScratchTop_.ptr, sizeof(top), hipMemcpyDeviceToHost, stream_));
            QHIP(hipStreamSynchronize(stream_));
            if (!ovf) break;
            if ((ovf & 2) || attempt > 6) throw DeviceError("quiver extend buffer exceeds 8 columns / scratch");
            grow_scratch(top);
        }
        t0 += m;
    }
    if (trace)
        std::fprintf(stderr, "[quiver] deltas items %d mutations %lld tasks %lld: prepare %.1f ms mid %.1f ms edges %lld %.1f ms\n",
                     n, mutStart[n], nTask, msPrep, msMid, (long long)nEdge, msSince(ts2));
}

void QuiverBatch::ScoreRound(const std::vector<int>& zs, const std::vector<std::vector<int>>& codes, int sep,
                             std::vector<std::vector<Scored>>* fav, std::vector<std::vector<Scored>>* picked)
{
    const int n = (int)zs.size();
    std::vector<long long> taskStart, mutStart;
    ScoreDeltas(zs, codes, &taskStart, &mutStart);
    const long long nMut = mutStart[n];
    dMScore_.reserve(std::max<long long>(nMut, 1), false);
    dFav_.reserve(std::max<long long>(nMut, 1), false);
    QReduceWork R;
    R.nWork = n;
    R.wMutStart = dWMutBase_.ptr;
    R.wTaskStart = dWTaskStart_.ptr;
    R.wNReads = dWNReads_.ptr;
    R.wFastThreshold = dWFast_.ptr;
    R.delta = dDelta_.ptr;
    R.score = dMScore_.ptr;
    R.fav = dFav_.ptr;
    R.nMut = nMut;
    launch_qreduce(R, stream_);
    QHIP(hipGetLastError());
    // favourable entries in list order, then BestSubset per scorer
    const int nm = (int)std::max<long long>(nMut, 1);
    dSel_.reserve(nm, false);
    dSelScore_.reserve(nm, false);
    dSelCode_.reserve(nm, false);
    dSelRank_.reserve(nm, false);
    dSelCount_.reserve(3, false);
    dSelBase_.reserve(std::max(n, 1), false);
    dNSel_.reserve(std::max(n, 1), false);
    hipcub::CountingInputIterator<long long> it(0);
    size_t a = 0, b = 0, c = 0;
    QHIP(hipcub::DeviceSelect::Flagged(nullptr, a, it, dFav_.ptr, dSel_.ptr, dSelCount_.ptr, nm, stream_));
    QHIP(hipcub::DeviceSelect::Flagged(nullptr, b, dMScore_.ptr, dFav_.ptr, dSelScore_.ptr, dSelCount_.ptr + 1, nm,
                                       stream_));
    QHIP(hipcub::DeviceSelect::Flagged(nullptr, c, dCodes_.ptr, dFav_.ptr, dSelCode_.ptr, dSelCount_.ptr + 2, nm,
                                       stream_));
    dSelTmp_.reserve(std::max<size_t>(std::max(a, std::max(b, c)), 1), false);
    if (nMut > 0) {
        QHIP(hipcub::DeviceSelect::Flagged(dSelTmp_.ptr, a, it, dFav_.ptr, dSel_.ptr, dSelCount_.ptr, nm, stream_));
        QHIP(hipcub::DeviceSelect::Flagged(dSelTmp_.ptr, b, dMScore_.ptr, dFav_.ptr, dSelScore_.ptr,
                                           dSelCount_.ptr + 1, nm, stream_));
        QHIP(hipcub::DeviceSelect::Flagged(dSelTmp_.ptr, c, dCodes_.ptr, dFav_.ptr, dSelCode_.ptr,
                                           dSelCount_.ptr + 2, nm, stream_));
    } else {
        QHIP(hipMemsetAsync(dSelCount_.ptr, 0, 3 * sizeof(long long), stream_));
    }
    pbccs::ScoreWork SW;
    SW.nWork = n;
    SW.mutStart = dWMutBase_.ptr;
    pbccs::launch_sel_ranges(SW, dSel_.ptr, dSelCount_.ptr, dSelBase_.ptr, dNSel_.ptr, stream_);
    pbccs::launch_best_subset(n, dSelBase_.ptr, dNSel_.ptr, dSelCode_.ptr, dSelScore_.ptr, std::max(sep, 0), -1,
                              dSelRank_.ptr, stream_);
    QHIP(hipGetLastError());
    long long cnt = 0;
    QHIP(hipMemcpyAsync(&cnt, dSelCount_.ptr, sizeof(long long), hipMemcpyDeviceToHost, stream_));
    QHIP(hipStreamSynchronize(stream_));
    std::vector<long long> sel;
    std::vector<double> selScore;
    std::vector<int> selCode, selRank;
    get(sel, dSel_, cnt, stream_);
    get(selScore, dSelScore_, cnt, stream_);
    get(selCode, dSelCode_, cnt, stream_);
    get(selRank, dSelRank_, cnt, stream_);
    QHIP(hipStreamSynchronize(stream_));
    fav->assign(n, {});
    picked->assign(n, {});
    std::vector<std::vector<std::pair<int, Scored>>> pk(n);
    for (long long q = 0; q < cnt; ++q) {
        const int w = (int)(std::upper_bound(mutStart.begin(), mutStart.end(), sel[q]) - mutStart.begin() - 1);
        const Scored e{selCode[q], (float)selScore[q]};
        (*fav)[w].push_back(e);
        if (selRank[q] > 0) pk[w].emplace_back(selRank[q], e);
    }
    for (int w = 0; w < n; ++w) {
        std::sort(pk[w].begin(), pk[w].end(),
                  [](const std::pair<int, Scored>& x, const std::pair<int, Scored>& y) { return x.first < y.first; });
        for (const std::pair<int, Scored>& p : pk[w]) (*picked)[w].push_back(p.second);
    }
}

void QuiverBatch::RefineMany(const std::vector<int>& zs, const RefineOptions& ro, std::vector<long long>* nTested,
                             std::vector<long long>* nApplied, std::vector<char>* converged, std::vector<char>* ok)
{
    const int n = (int)zs.size();
    nTested->assign(n, 0);
    nApplied->assign(n, 0);
    converged->assign(n, 0);
    ok->assign(n, 1);
    std::vector<char> done(n, 0);
    std::vector<int> iter(n, 0);
    std::vector<std::unordered_set<std::string>> history(n);
    std::vector<std::vector<int>> centers(n);
    if (ro.maxIterations <= 0) return;
    static const bool trace = std::getenv("PBCCS_QUIVER_TRACE") != nullptr;
    using Clock = std::chrono::steady_clock;
    auto msSince = [](Clock::time_point a) { return std::chrono::duration<double, std::milli>(Clock::now() - a).count(); };
    for (int round = 0;; ++round) {
        const Clock::time_point tr0 = Clock::now();
        std::vector<int> act, idx;
        for (int k = 0; k < n; ++k)
            if (!done[k]) { act.push_back(zs[k]); idx.push_back(k); }
        if (act.empty()) break;
        std::vector<std::vector<int>> codes(act.size());
        par_for((int)act.size(), [&](int a) {
            const std::string& tpl = zmws_[act[a]].tpl;
            const int k = idx[a];
            if (iter[k] == 0) unique_mutations(tpl, 0, (int)tpl.size(), &codes[a]);
            else nearby_mutations(tpl, centers[k], ro.mutationNeighborhood, &codes[a]);
            (*nTested)[k] += (long long)codes[a].size();
        });
        std::vector<std::vector<Scored>> fav, picked;
        const double msEnum = msSince(tr0);
        const Clock::time_point tr1 = Clock::now();
        ScoreRound(act, codes, ro.mutationSeparation, &fav, &picked);
        const double msScore = msSince(tr1);
        const Clock::time_point tr2 = Clock::now();
        // every scorer's edit on its own (host threads), then the refilled reads' capacity in list order
        std::vector<char> edited(act.size(), 0);
        par_for((int)act.size(), [&](int a) {
            const int k = idx[a];
            HZmw& z = zmws_[act[a]];
            if (fav[a].empty()) {
                (*converged)[k] = 1;
                done[k] = 1;
                return;
            }
            std::vector<Scored>& best = picked[a];
            std::vector<Mutation> muts;
            for (const Scored& b : best) muts.push_back(mutation_from_code(b.code));
            if (best.size() > 1) {
                std::string nx;
                std::vector<int> mtp;
                if (apply_mutations(z.tpl, muts, &nx, &mtp) && history[k].count(nx)) {
                    best.resize(1);
                    muts.resize(1);
                }
            }
            (*nApplied)[k] += (long long)best.size();
            history[k].insert(z.tpl);
            centers[k].clear();
            for (const Scored& f : fav[a]) centers[k].push_back(mut_pos(f.code));
            std::string next;
            std::vector<int> mtp;
            if (!apply_mutations(z.tpl, muts, &next, &mtp)) {   // ApplyMutations refused: Refine returns false
                (*ok)[k] = 0;
                done[k] = 1;
                return;
            }
            z.tpl = next;
            for (int r : z.reads) {
                HRead& h = reads_[r];
                h.ts = mtp[h.ts];
                h.te = mtp[h.te];
            }
            edited[a] = 1;
            if (++iter[k] >= ro.maxIterations) done[k] = 1;
        });
        std::vector<int> refill;
        for (size_t a = 0; a < act.size(); ++a) {
            if (!edited[a]) continue;
            for (int r : zmws_[act[a]].reads)
                if (reads_[r].active) {
                    EnsureCapacity(r);
                    refill.push_back(r);
                }
            dirty_ = true;
        }
        const double msApply = msSince(tr2);
        const Clock::time_point tr3 = Clock::now();
        if (!refill.empty()) Fill(refill);   // a refill that mismatches marks the read inactive
        if (trace)
            std::fprintf(stderr, "[quiver] round %d scorers %zu enumerate %.1f ms score %.1f ms apply %.1f ms fill %.1f ms\n",
                         round, act.size(), msEnum, msScore, msApply, msSince(tr3));
    }
}

std::vector<std::vector<int>> QuiverBatch::QVsMany(const std::vector<int>& zs)   // ConsensusQVs (:274-295)
{
    // every unique single-base mutation of every position, scored over all reads (Score, no fast break), then the
    // per-position sums and QVs on the device (k_qqv); only the QVs come back
    const int n = (int)zs.size();
    std::vector<std::vector<int>> codes(n);
    std::vector<int> posOff;
    std::vector<long long> posStart(n + 1, 0), posOffBase(n);
    for (int w = 0; w < n; ++w) {
        const long long L = (long long)zmws_[zs[w]].tpl.size();
        posOffBase[w] = posStart[w] + w;   // L + 1 offsets per scorer
        posStart[w + 1] = posStart[w] + L;
    }
    posOff.resize((size_t)(posStart[n] + n));
    par_for(n, [&](int w) {   // per position's mutation list, scorers on several threads
        const std::string& tpl = zmws_[zs[w]].tpl;
        int* po = posOff.data() + posOffBase[w];
        for (int p = 0; p < (int)tpl.size(); ++p) {
            po[p] = (int)codes[w].size();
            unique_mutations(tpl, p, p + 1, &codes[w]);
        }
        po[tpl.size()] = (int)codes[w].size();
    });
    std::vector<long long> taskStart, mutStart;
    ScoreDeltas(zs, codes, &taskStart, &mutStart);
    const long long nMut = mutStart[n], nPos = posStart[n];
    dMScore_.reserve(std::max<long long>(nMut, 1), false);
    dFav_.reserve(std::max<long long>(nMut, 1), false);
    QReduceWork R;
    R.nWork = n;
    R.wMutStart = dWMutBase_.ptr;
    R.wTaskStart = dWTaskStart_.ptr;
    R.wNReads = dWNReads_.ptr;
    R.wFastThreshold = dWFast_.ptr;
    R.delta = dDelta_.ptr;
    R.score = dMScore_.ptr;
    R.fav = dFav_.ptr;
    R.nMut = nMut;
    launch_qreduce(R, stream_);
    put(dPosStart_, posStart, stream_);
    put(dPosOffBase_, posOffBase, stream_);
    put(dPosOff_, posOff, stream_);
    dQv_.reserve(std::max<long long>(nPos, 1), false);
    QQvWork Q;
    Q.nWork = n;
    Q.posStart = dPosStart_.ptr;
    Q.wMutStart = dWMutBase_.ptr;
    Q.posOffBase = dPosOffBase_.ptr;
    Q.posOff = dPosOff_.ptr;
    Q.score = dMScore_.ptr;
    Q.qv = dQv_.ptr;
    Q.hostAll = std::getenv("PBCCS_QQV_HOST") != nullptr;   // test hook: the host path for every position
    launch_qqv(Q, nPos, stream_);
    QHIP(hipGetLastError());
    std::vector<int> all;
    get(all, dQv_, (size_t)nPos, stream_);
    QHIP(hipStreamSynchronize(stream_));
    // positions k_qqv left to the host (-1: the rounding of -10 log10(prob) could depend on the libm): their
    // mutation scores come back and the sum, ProbabilityToQV and the libm are the reference's
    std::vector<std::pair<int, int>> amb;   // (scorer, position)
    for (int w = 0; w < n; ++w)
        for (long long g = posStart[w]; g < posStart[w + 1]; ++g)
            if (all[(size_t)g] < 0) amb.emplace_back(w, (int)(g - posStart[w]));
    static const bool qtrace = std::getenv("PBCCS_QUIVER_TRACE") != nullptr;
    if (qtrace) std::fprintf(stderr, "[quiver] qvs positions %lld host-recomputed %zu\n", nPos, amb.size());
    if (!amb.empty()) {   // packed on the device (k_qgather), one download
        const int na = (int)amb.size();
        std::vector<long long> src(na), dst(na + 1, 0);
        for (int a = 0; a < na; ++a) {
            const int w = amb[a].first, p = amb[a].second;
            const int* po = posOff.data() + posOffBase[w];
            src[a] = mutStart[w] + po[p];
            dst[a + 1] = dst[a] + (po[p + 1] - po[p]);
        }
        put(dAmbSrc_, src, stream_);
        put(dAmbDst_, dst, stream_);
        dAmbScore_.reserve(std::max<long long>(dst[na], 1), false);
        launch_qgather(dMScore_.ptr, dAmbSrc_.ptr, dAmbDst_.ptr, na, dAmbScore_.ptr, stream_);
        QHIP(hipGetLastError());
        std::vector<double> sc;
        get(sc, dAmbScore_, (size_t)dst[na], stream_);
        QHIP(hipStreamSynchronize(stream_));
        par_for(na, [&](int a) {   // (a fifth of the positions at 10 passes: the high QVs sit near prob ~ eps)
            double sum = 0.0;
            for (long long m = dst[a]; m < dst[a + 1]; ++m) {
                const double f = (double)(float)sc[(size_t)m];   // Score() is a float sum
                if (f < 0.0) sum += std::exp(f);
            }
            all[(size_t)(posStart[amb[a].first] + amb[a].second)] = probability_to_qv(1.0 - 1.0 / (1.0 + sum));
        }, 4096);
    }
    std::vector<std::vector<int>> qv(n);
    for (int w = 0; w < n; ++w) qv[w].assign(all.begin() + posStart[w], all.begin() + posStart[w + 1]);
    return qv;
}

}  // namespace quiver
}  // namespace pbccs
