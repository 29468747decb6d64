// pbccs_amd/csrc/capi.hip -- the C ABI (include/pbccs_amd.h) over ArrowBatch.
#include "../../include/pbccs_amd.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "engine.hpp"
#include "driver.hpp"
#include "poa_engine.hpp"
#include "quiver_engine.hpp"

using namespace pbccs;

// ZMW work queue (pbccs_polish_batch): device memory left free beside the batches' band pools (score
// buffers, selection scratch, in-kernel growth headroom), and the largest batch (the best 2 kb batch
// shape measured).
constexpr double kQueueMargin = 24.0 * (1ull << 30);
constexpr int kCcsTailPiece = 250;   // smallest piece of the last ccs chunk's polish (pbccs_ccs_batch)
constexpr int kQueueMaxZmws = 2000;
// readOf entry of a read the caller did not add (NULL sequence): counted in the drop fraction's
// denominator only, as the reads Consensus.h:441-471 skips (POA rejected it, or ExtractMappedRead did)
constexpr int kSkippedRead = -2;

struct pbccs_engine {
    int device = 0;
    Counters counters;
    bool profiling = false;
    KernelStat stats[kKernelKinds];
    // Resident pools.  Batches are dealt round-robin onto `concurrency` workspace slots; batches that
    // share a slot never polish at the same time (pbccs_batch_polish_many runs one slot per thread).
    int concurrency = 4;
    int nextSlot = 0;
    std::mutex statsMu;        // counters / stats are merged from the slots' worker threads
    long long oomRetries = 0;   // device batches rerun after PBCCS_EOOM
    long long createHostNs = 0, createUploadNs = 0;   // pbccs_batch_create: host setup / reservations + upload
    std::vector<std::unique_ptr<Workspace>> slots;
    // the POA draft step's device state (made on first use): kPoaSlices runners, one per concurrent slice
    // PBCCS_POA_SLICES overrides the slice count (A/B): more slices overlap one slice's host graph work with
    // the others' device rounds, with fewer host threads each
    static constexpr int kPoaSlicesDefault = 3;   // 1 / 2 / 3 / 4 slices: 1400 / 1527 / 1575 / 1571 ccs ZMWs/s (profiles/r3y_ccs_slices_ab.txt)
    static int PoaSlices()
    {
        static const int n = std::max(1, std::min(8, std::getenv("PBCCS_POA_SLICES") ? std::atoi(std::getenv("PBCCS_POA_SLICES"))
                                                                                      : kPoaSlicesDefault));
        return n;
    }
    std::vector<std::unique_ptr<poa::PoaRunner>> poa;
    std::mutex poaMu;
    poa::PoaRunner& Poa(int k = 0)
    {
        if (poa.empty()) {
            const int hw = std::max(2, std::min(16, (int)std::thread::hardware_concurrency()));
            for (int i = 0; i < PoaSlices(); ++i)
                poa.emplace_back(new poa::PoaRunner(device, std::max(1, hw / PoaSlices())));
        }
        poa[k]->profiling = profiling;
        return *poa[k];
    }
    std::vector<poa::PoaRunner*> PoaRunners()
    {
        std::vector<poa::PoaRunner*> v;
        for (int k = 0; k < PoaSlices(); ++k) v.push_back(&Poa(k));
        return v;
    }
    // pbccs_quiver_polish_batch's scorer batch, kept between calls (Reset per call) so its device buffers and host
    // pools are allocated once; calls on one engine take turns on it
    std::unique_ptr<quiver::QuiverBatch> quiverBatch;
    std::mutex quiverMu;
    Workspace* Slot(int s)
    {
        while ((int)slots.size() <= s) slots.emplace_back(new Workspace(true));
        return slots[s].get();
    }
};

// Owned host copy of a batch's inputs: a batch that ran the device out of memory is rebuilt from it.
struct HostInputs {
    struct Zmw {
        std::string draft;
        std::vector<std::string> seqs;
        std::vector<const char*> seqPtr;
        std::vector<int> lens, strands, ts, te;
        std::vector<unsigned char> full;
    };
    std::vector<Zmw> z;
    std::vector<pbccs_zmw_input> in;   // views into z
    void assign(const pbccs_zmw_input* src, int n)
    {
        z.assign(n, Zmw());
        in.assign(n, pbccs_zmw_input());
        for (int i = 0; i < n; ++i) {
            const pbccs_zmw_input& s = src[i];
            Zmw& d = z[i];
            const int nr = std::max(0, s.n_reads);
            d.draft.assign(s.draft ? s.draft : "", s.draft ? std::max(0, s.draft_len) : 0);
            d.seqs.resize(nr);
            d.lens.assign(nr, 0);
            d.strands.assign(nr, 0);
            d.ts.assign(nr, 0);
            d.te.assign(nr, 0);
            d.full.assign(nr, 1);
            for (int k = 0; k < nr; ++k) {
                d.lens[k] = s.lens[k];
                if (s.seqs[k]) d.seqs[k].assign(s.seqs[k], std::max(0, s.lens[k]));
                d.strands[k] = s.strands[k];
                d.ts[k] = s.tstarts[k];
                d.te[k] = s.tends[k];
                if (s.full_pass) d.full[k] = s.full_pass[k];
            }
            d.seqPtr.resize(nr);
            for (int k = 0; k < nr; ++k) d.seqPtr[k] = s.seqs[k] ? d.seqs[k].c_str() : nullptr;
            pbccs_zmw_input& v = in[i];
            v = s;
            v.draft = d.draft.c_str();
            v.seqs = d.seqPtr.data();
            v.lens = d.lens.data();
            v.strands = d.strands.data();
            v.tstarts = d.ts.data();
            v.tends = d.te.data();
            v.full_pass = d.full.data();
        }
    }
};

struct pbccs_batch {
    HostInputs inputs;
    pbccs_engine* eng = nullptr;
    int slot = 0;
    std::unique_ptr<ArrowBatch> B;
    pbccs_polish_options o;
    int n = 0;
    std::vector<int> zOf;                       // -1: rejected before the device (status in preStatus)
    std::vector<int> preStatus;
    std::vector<int> nReads;
    std::vector<std::vector<int>> readOf;       // -1: read not added (invalid window)
    std::vector<std::vector<unsigned char>> fullPass;
    std::vector<int> allReads;
    bool polished = false;
};

struct pbccs_scorer {
    pbccs_engine* eng = nullptr;
    std::unique_ptr<ArrowBatch> batch;
    pbccs_arrow_config cfg;
    int z = 0;
};

namespace {

thread_local std::string g_lastError;

int fail(int code, const char* msg)
{
    g_lastError = msg ? msg : "";
    return code;
}

template <class F>
int guarded(F&& f)
{
    try {
        return f();
    } catch (const DeviceOom& e) {
        return fail(PBCCS_EOOM, e.what());
    } catch (const DeviceError& e) {
        return fail(PBCCS_EDEVICE, e.what());
    } catch (const std::bad_alloc&) {
        return fail(PBCCS_EOOM, "out of memory");
    } catch (const std::invalid_argument& e) {
        return fail(PBCCS_EINVAL, e.what());
    } catch (const std::out_of_range& e) {
        return fail(PBCCS_EINVAL, e.what());
    } catch (const std::exception& e) {
        return fail(PBCCS_EDEVICE, e.what());
    } catch (...) {
        return fail(PBCCS_EDEVICE, "unknown failure");
    }
}

ArrowOptions options_from(const pbccs_arrow_config* c)
{
    ArrowOptions o;
    if (c) {
        o.scoreDiff = c->score_diff;
        o.fastScoreThreshold = c->fast_score_threshold;
        o.addThreshold = c->add_threshold;
    }
    return o;
}

bool to_mutation(const pbccs_mutation& in, int L, Mutation* out)
{
    if (in.type < 0 || in.type > 2) return false;
    const int width = in.end - in.start;
    if (in.type == PBCCS_INSERTION ? width != 0 : width != 1) return false;   // single-base only
    if (in.start < 0) return false;
    if (in.type == PBCCS_INSERTION ? in.start > L : in.start >= L) return false;
    if (in.type != PBCCS_DELETION && !(in.new_base == 'A' || in.new_base == 'C' || in.new_base == 'G' || in.new_base == 'T'))
        return false;
    *out = Mutation::Make(in.type, in.start, in.new_base);
    return true;
}

bool read_scores(int ts, int te, const Mutation& m)   // MultiReadMutationScorer.cpp:70-80
{
    if (m.type == PBCCS_INSERTION) return ts <= m.end && m.start <= te;
    return ts < m.end && m.start < te;
}

}  // namespace

extern "C" {

const char* pbccs_last_error(void) { return g_lastError.c_str(); }

int pbccs_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int pbccs_engine_create(int device, pbccs_engine** out)
{
    if (!out) return fail(PBCCS_EINVAL, "null out");
    return guarded([&] {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
            return fail(PBCCS_EDEVICE, "no such HIP device");
        if (hipSetDevice(device) != hipSuccess) return fail(PBCCS_EDEVICE, "hipSetDevice failed");
        pbccs_engine* e = new pbccs_engine();
        e->device = device;
        *out = e;
        return PBCCS_OK;
    });
}

void pbccs_engine_destroy(pbccs_engine* eng) { delete eng; }

int pbccs_engine_counters(pbccs_engine* eng, pbccs_counters* out, int reset)
{
    if (!eng || !out) return fail(PBCCS_EINVAL, "null argument");
    out->fill_launches = eng->counters.fillLaunches;
    out->score_launches = eng->counters.scoreLaunches;
    out->score_tasks = eng->counters.scoreTasks;
    out->mutations = eng->counters.mutations;
    out->band_top_bytes = eng->counters.bandTopBytes;
    out->band_region_bytes = eng->counters.bandRegionBytes;
    out->band_used_bytes = eng->counters.bandUsedBytes;
    long long mapped = 0;
    for (const auto& s : eng->slots) mapped += (long long)s->val.mapped_bytes();
    out->pool_mapped_bytes = mapped;
    out->oom_retries = eng->oomRetries;
    out->create_host_ns = eng->createHostNs;
    out->create_upload_ns = eng->createUploadNs;
    out->derive_ns = eng->counters.deriveNs;
    for (int k = 0; k < 16; ++k) out->fill_work[k] = eng->counters.fillWork[k];
    out->scan_reads = eng->counters.scanReads;
    out->uncertain_reads = eng->counters.uncertainReads;
    out->exact_rounds = eng->counters.exactRounds;
    for (int k = 0; k < 4; ++k) out->uncertain_why[k] = eng->counters.uncertainWhy[k];
    if (reset) {
        eng->counters = Counters();
        eng->oomRetries = 0;
        eng->createHostNs = eng->createUploadNs = 0;
    }
    return PBCCS_OK;
}

// ---- scorer ---------------------------------------------------------------------------------------
int pbccs_scorer_create(pbccs_engine* eng, const pbccs_arrow_config* cfg, const char* tpl, int tpl_len,
                        pbccs_scorer** out)
{
    if (!eng || !cfg || !tpl || tpl_len <= 0 || !out) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        std::unique_ptr<pbccs_scorer> s(new pbccs_scorer());
        s->eng = eng;
        s->cfg = *cfg;
        s->batch.reset(new ArrowBatch(eng->device));
        s->z = s->batch->AddZmw(std::string(tpl, tpl_len), cfg->snr, options_from(cfg));
        *out = s.release();
        return PBCCS_OK;
    });
}

void pbccs_scorer_destroy(pbccs_scorer* s) { delete s; }

int pbccs_scorer_add_read(pbccs_scorer* s, const char* seq, int len, int strand, int tstart, int tend,
                          double threshold, int* result)
{
    if (!s || !seq || len < 0 || !result || (strand != 0 && strand != 1)) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        ArrowBatch& B = *s->batch;
        const int r = B.AppendRead(s->z, std::string(seq, len), strand, tstart, tend);
        B.FillReads({r});
        *result = B.FinishAddRead(r, threshold);
        return PBCCS_OK;
    });
}

int pbccs_scorer_score_many(pbccs_scorer* s, const pbccs_mutation* m, int n, double fast_threshold, double* scores)
{
    if (!s || (n > 0 && (!m || !scores)) || n < 0) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        ArrowBatch& B = *s->batch;
        const int L = (int)B.Template(s->z).size();
        std::vector<std::vector<int>> codes(1);
        for (int i = 0; i < n; ++i) {
            Mutation mu;
            if (!to_mutation(m[i], L, &mu)) return fail(PBCCS_EINVAL, "invalid single-base mutation");
            codes[0].push_back(mutation_code(mu));
        }
        if (n == 0) return PBCCS_OK;
        std::vector<std::vector<double>> sc;
        B.ScoreLists({s->z}, codes, fast_threshold, &sc);
        for (int i = 0; i < n; ++i) scores[i] = sc[0][i];
        return PBCCS_OK;
    });
}

int pbccs_scorer_score(pbccs_scorer* s, const pbccs_mutation* m, double fast_threshold, double* score)
{
    return pbccs_scorer_score_many(s, m, 1, fast_threshold, score);
}

int pbccs_scorer_scores(pbccs_scorer* s, const pbccs_mutation* m, double unscored, double* per_read)
{
    if (!s || !m || !per_read) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        ArrowBatch& B = *s->batch;
        Mutation mu;
        if (!to_mutation(*m, (int)B.Template(s->z).size(), &mu)) return fail(PBCCS_EINVAL, "invalid mutation");
        std::vector<std::vector<double>> sc, pr;
        B.ScoreLists({s->z}, {{mutation_code(mu)}}, -std::numeric_limits<double>::max(), &sc, &pr);
        const int nr = B.NumReads(s->z);
        for (int k = 0; k < nr; ++k) {
            const int r = B.ReadIndex(s->z, k);
            const bool scored = B.ReadActive(r) && read_scores(B.ReadTs(r), B.ReadTe(r), mu);
            per_read[k] = scored ? pr[0][k] : unscored;
        }
        return PBCCS_OK;
    });
}

int pbccs_scorer_is_favorable(pbccs_scorer* s, const pbccs_mutation* m, int fast, int* favorable)
{
    if (!s || !favorable) return fail(PBCCS_EINVAL, "bad argument");
    double v = 0.0;
    const double thr = fast ? s->cfg.fast_score_threshold : -std::numeric_limits<double>::max();
    const int rc = pbccs_scorer_score(s, m, thr, &v);
    if (rc != PBCCS_OK) return rc;
    *favorable = v > kMinFavorableScoreDiff ? 1 : 0;
    return PBCCS_OK;
}

int pbccs_scorer_apply_mutations(pbccs_scorer* s, const pbccs_mutation* m, int n)
{
    if (!s || n < 0 || (n > 0 && !m)) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        ArrowBatch& B = *s->batch;
        const int L = (int)B.Template(s->z).size();
        std::vector<Mutation> muts;
        for (int i = 0; i < n; ++i) {
            Mutation mu;
            if (!to_mutation(m[i], L, &mu)) return fail(PBCCS_EINVAL, "invalid mutation");
            muts.push_back(mu);
        }
        if (!B.ApplyMutations(s->z, muts)) return fail(PBCCS_EINVAL, "mutation outside the template");
        return PBCCS_OK;
    });
}

int pbccs_scorer_template(pbccs_scorer* s, int strand, char* out, int cap, int* len)
{
    if (!s || !len) return fail(PBCCS_EINVAL, "bad argument");
    const std::string t = strand == PBCCS_FORWARD_STRAND ? s->batch->Template(s->z) : s->batch->TemplateRev(s->z);
    *len = (int)t.size();
    if (!out || cap < (int)t.size() + 1) return fail(PBCCS_ERANGE, "buffer too small");
    std::memcpy(out, t.c_str(), t.size() + 1);
    return PBCCS_OK;
}

int pbccs_scorer_template_length(pbccs_scorer* s) { return s ? (int)s->batch->Template(s->z).size() : -1; }

int pbccs_scorer_num_reads(pbccs_scorer* s) { return s ? s->batch->NumReads(s->z) : -1; }

int pbccs_scorer_read_info(pbccs_scorer* s, int i, int* active, int* strand, int* tstart, int* tend)
{
    if (!s || i < 0 || i >= s->batch->NumReads(s->z)) return fail(PBCCS_EINVAL, "bad read index");
    const int r = s->batch->ReadIndex(s->z, i);
    if (active) *active = s->batch->ReadActive(r) ? 1 : 0;
    if (strand) *strand = s->batch->ReadStrand(r);
    if (tstart) *tstart = s->batch->ReadTs(r);
    if (tend) *tend = s->batch->ReadTe(r);
    return PBCCS_OK;
}

int pbccs_scorer_baseline_score(pbccs_scorer* s, double* score)
{
    if (!s || !score) return fail(PBCCS_EINVAL, "bad argument");
    *score = s->batch->BaselineScore(s->z);
    return PBCCS_OK;
}

int pbccs_scorer_baseline_scores(pbccs_scorer* s, double* out, int cap, int* n)
{
    if (!s || !n) return fail(PBCCS_EINVAL, "bad argument");
    std::vector<double> v;
    for (int k = 0; k < s->batch->NumReads(s->z); ++k) {
        const int r = s->batch->ReadIndex(s->z, k);
        if (s->batch->ReadActive(r)) v.push_back(s->batch->ReadScore(r));
    }
    *n = (int)v.size();
    if (!out || cap < (int)v.size()) return fail(PBCCS_ERANGE, "buffer too small");
    std::copy(v.begin(), v.end(), out);
    return PBCCS_OK;
}

int pbccs_scorer_zscores(pbccs_scorer* s, double* zg, double* za, double* per_read)
{
    if (!s || !zg || !za) return fail(PBCCS_EINVAL, "bad argument");
    std::vector<double> zs;
    s->batch->ZScores(s->z, zg, za, &zs);
    if (per_read) std::copy(zs.begin(), zs.end(), per_read);
    return PBCCS_OK;
}

int pbccs_scorer_num_flipflops(pbccs_scorer* s, int* out)
{
    if (!s || !out) return fail(PBCCS_EINVAL, "bad argument");
    for (int k = 0; k < s->batch->NumReads(s->z); ++k) out[k] = s->batch->ReadFlips(s->batch->ReadIndex(s->z, k));
    return PBCCS_OK;
}

int pbccs_refine_consensus(pbccs_scorer* s, const pbccs_refine_options* opts, long long* n_tested,
                           long long* n_applied, int* converged)
{
    if (!s || !n_tested || !n_applied || !converged) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        RefineOptions ro;
        if (opts) {
            ro.maxIterations = opts->max_iterations;
            ro.mutationSeparation = opts->mutation_separation;
            ro.mutationNeighborhood = opts->mutation_neighborhood;
        }
        std::vector<int> conv;
        std::vector<long long> nt, na;
        s->batch->Refine({s->z}, ro, &conv, &nt, &na);
        *n_tested += nt[0];
        *n_applied += na[0];
        if (conv[0] < 0) return fail(PBCCS_EINVAL, "mutation could not be applied");
        *converged = conv[0];
        return PBCCS_OK;
    });
}

int pbccs_consensus_qvs(pbccs_scorer* s, int* qvs, int cap, int* n)
{
    if (!s || !n) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        std::vector<std::vector<int>> q;
        s->batch->QVs({s->z}, &q);
        *n = (int)q[0].size();
        if (!qvs || cap < *n) return fail(PBCCS_ERANGE, "buffer too small");
        std::copy(q[0].begin(), q[0].end(), qvs);
        return PBCCS_OK;
    });
}

// ---- batched polish -------------------------------------------------------------------------------
void pbccs_polish_options_default(pbccs_polish_options* o)
{
    if (!o) return;
    o->min_passes = 3;
    o->min_length = 10;
    o->min_zscore = -5.0;
    o->max_drop_fraction = 0.34;
    o->min_predicted_accuracy = 0.90;
    o->score_diff = 12.5;
    o->refine.max_iterations = 40;
    o->refine.mutation_separation = 10;
    o->refine.mutation_neighborhood = 20;
    o->zmws_per_batch = 0;
}

// Merge a batch's counters and profile into its engine.  Never throws: it runs in worker threads and on
// the way out of the C ABI (a device error while resolving events only loses that batch's timings).
static void merge_engine_stats(pbccs_engine* eng, ArrowBatch& B)
{
    std::lock_guard<std::mutex> lk(eng->statsMu);
    try {
        const Counters& c = B.counters();
        eng->counters.fillLaunches += c.fillLaunches;
        eng->counters.scoreLaunches += c.scoreLaunches;
        eng->counters.scoreTasks += c.scoreTasks;
        eng->counters.mutations += c.mutations;
        eng->counters.deriveNs += c.deriveNs;
        eng->counters.scanReads += c.scanReads;
        eng->counters.uncertainReads += c.uncertainReads;
        eng->counters.exactRounds += c.exactRounds;
        for (int k = 0; k < 4; ++k) eng->counters.uncertainWhy[k] += c.uncertainWhy[k];
        for (int k = 0; k < 16; ++k) eng->counters.fillWork[k] += c.fillWork[k];
        eng->counters.bandTopBytes = std::max(eng->counters.bandTopBytes, c.bandTopBytes);
        eng->counters.bandRegionBytes = std::max(eng->counters.bandRegionBytes, c.bandRegionBytes);
        eng->counters.bandUsedBytes = std::max(eng->counters.bandUsedBytes, c.bandUsedBytes);
        B.ResetCounters();
        B.CollectProfile(eng->stats);
    } catch (...) {
        (void)hipGetLastError();
    }
}

// A batch on an explicit workspace slot (slot < 0: the next slot round-robin).
static int create_batch(pbccs_engine* eng, const pbccs_zmw_input* in, int n, const pbccs_polish_options* opts,
                        int slot, pbccs_batch** out)
{
    if (!eng || n < 0 || (n > 0 && !in) || !out) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        if (hipSetDevice(eng->device) != hipSuccess) return fail(PBCCS_EDEVICE, "hipSetDevice failed");
        const auto t0 = std::chrono::steady_clock::now();
        std::unique_ptr<pbccs_batch> b(new pbccs_batch());
        b->eng = eng;
        pbccs_polish_options_default(&b->o);
        if (opts) b->o = *opts;
        b->n = n;
        b->slot = slot >= 0 ? slot : eng->nextSlot++ % std::max(1, eng->concurrency);
        b->inputs.assign(in, n);
        // every batch gets its own streams (ArrowBatch's ownStreams); a batch made and polished on its slot's thread
        // (slot >= 0: the queue, the ccs chunks, reruns) uses the slot's descriptor arena and read pool
        // PBCCS_SLOT_STREAMS=1 (debug / A/B): the slot workspace's persistent streams instead
        // (read per batch: a test switches it at run time)
        const bool slotStreams = std::getenv("PBCCS_SLOT_STREAMS") && std::getenv("PBCCS_SLOT_STREAMS")[0] == '1';
        b->B.reset(new ArrowBatch(eng->device, eng->Slot(b->slot), !slotStreams, slot >= 0));
        b->B->SetProfiling(eng->profiling);
        ArrowOptions ao;
        ao.scoreDiff = b->o.score_diff;
        b->zOf.assign(n, -1);
        b->preStatus.assign(n, PBCCS_ZMW_OTHER);
        b->nReads.assign(n, 0);
        b->readOf.assign(n, {});
        b->fullPass.assign(n, {});
        for (int i = 0; i < n; ++i) {
            const pbccs_zmw_input& z = in[i];
            b->nReads[i] = z.n_reads;
            if (z.n_reads <= 0) { b->preStatus[i] = PBCCS_ZMW_NO_SUBREADS; continue; }
            if (z.draft_len < b->o.min_length) { b->preStatus[i] = PBCCS_ZMW_TOO_SHORT; continue; }
            const std::string draft(z.draft, z.draft_len);
            if (!is_acgt(draft)) { b->preStatus[i] = PBCCS_ZMW_OTHER; continue; }
            b->zOf[i] = b->B->AddZmw(draft, z.snr, ao);
            for (int k = 0; k < z.n_reads; ++k) {
                int r = -1;
                if (!z.seqs[k]) r = kSkippedRead;   // not added (Consensus.h:448-451): denominator only
                else if (z.tstarts[k] >= 0 && z.tends[k] <= z.draft_len && z.tstarts[k] < z.tends[k] && z.lens[k] > 0)
                    r = b->B->AppendRead(b->zOf[i], std::string(z.seqs[k], z.lens[k]), z.strands[k] ? 1 : 0,
                                         z.tstarts[k], z.tends[k]);
                b->readOf[i].push_back(r);
                b->fullPass[i].push_back(z.full_pass ? z.full_pass[k] : 1);
                if (r >= 0) b->allReads.push_back(r);
            }
        }
        const auto t1 = std::chrono::steady_clock::now();
        b->B->Prepare();
        const auto t2 = std::chrono::steady_clock::now();
        {
            std::lock_guard<std::mutex> lk(eng->statsMu);
            eng->createHostNs += std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
            eng->createUploadNs += std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count();
        }
        *out = b.release();
        return PBCCS_OK;
    });
}

int pbccs_batch_create(pbccs_engine* eng, const pbccs_zmw_input* in, int n, const pbccs_polish_options* opts,
                       pbccs_batch** out)
{
    return create_batch(eng, in, n, opts, -1, out);
}

void pbccs_batch_destroy(pbccs_batch* b) { delete b; }

static int polish_one(pbccs_batch* b, pbccs_zmw_output* out)
{
    if (!b || (b->n > 0 && !out)) return fail(PBCCS_EINVAL, "bad argument");
    if (b->polished) return fail(PBCCS_ESTATE, "a batch polishes once");
    if (!b->B) return fail(PBCCS_ESTATE, "the batch's device state was released");
    return guarded([&] {
        if (hipSetDevice(b->eng->device) != hipSuccess) return fail(PBCCS_EDEVICE, "hipSetDevice failed");
        b->polished = true;
        ArrowBatch& B = *b->B;
        const pbccs_polish_options& o = b->o;
        const int n = b->n;
        for (int i = 0; i < n; ++i) {
            pbccs_zmw_output& q = out[i];
            q.status = b->preStatus[i];
            q.consensus_len = 0;
            q.zg = q.za = std::numeric_limits<double>::quiet_NaN();
            q.predicted_accuracy = 0.0;
            q.n_tested = q.n_applied = 0;
            q.n_passes = 0;
            for (int k = 0; k < 5; ++k) q.status_counts[k] = 0;
            for (int k = 0; k < b->nReads[i]; ++k) {
                if (q.add_read_results) q.add_read_results[k] = -1;
                if (q.zscores) q.zscores[k] = std::numeric_limits<double>::quiet_NaN();
            }
        }
        // PBCCS_RECLAIM=1: bands of ZMWs the batch is done with are dropped as it goes and every refill relays
        // the value pool out (ArrowBatch::Relayout), with ConsensusQVs run in the round a ZMW
        // converges.  Opt-in: it cuts the refine rounds' band top (42.5 -> 39.9 GB per 2000-ZMW batch; the
        // initial fill sets the high-water) but the per-round QVs cost 5.5% (profiles/r2h5_reclaim_ab)
        const char* reclaimEnv = std::getenv("PBCCS_RECLAIM");
        const bool reclaim = reclaimEnv && std::strcmp(reclaimEnv, "1") == 0;
        B.SetReclaim(reclaim);
        // the certified fast path for the batch's tall reads; PBCCS_CERTIFIED_SCAN=0: exact fills only
        const char* ce = std::getenv("PBCCS_CERTIFIED_SCAN");   // read per batch: tests switch it at run time
        const bool certified = !ce || ce[0] != '0';
        B.SetCertifiedScan(certified);
        B.FillReads(b->allReads);
        B.CertifyAddReads(b->allReads, o.min_zscore);
        std::vector<int> refineZ, refineIdx, dropZ;
        for (int i = 0; i < n; ++i) {
            if (b->zOf[i] < 0) continue;
            pbccs_zmw_output& q = out[i];
            int nPasses = 0, nDropped = 0;
            for (int k = 0; k < b->nReads[i]; ++k) {
                const int r = b->readOf[i][k];
                if (r == kSkippedRead) continue;
                const int st = (r >= 0) ? B.FinishAddRead(r, o.min_zscore) : PBCCS_ADD_OTHER;
                if (q.add_read_results) q.add_read_results[k] = st;
                q.status_counts[st] += 1;
                if (st == PBCCS_ADD_SUCCESS && b->fullPass[i][k]) ++nPasses;
                else if (st != PBCCS_ADD_SUCCESS) ++nDropped;
            }
            q.n_passes = nPasses;
            if (nPasses < o.min_passes) {
                q.status = PBCCS_ZMW_TOO_FEW_PASSES;
                dropZ.push_back(b->zOf[i]);
                continue;
            }
            const double frac = (double)nDropped / b->nReads[i];
            if (frac > o.max_drop_fraction) {
                q.status = PBCCS_ZMW_TOO_MANY_UNUSABLE;
                dropZ.push_back(b->zOf[i]);
                continue;
            }
            std::vector<double> zs;
            B.ZScores(b->zOf[i], &q.zg, &q.za, &zs);
            if (q.zscores) {
                int j = 0;
                for (int k = 0; k < b->nReads[i]; ++k)
                    if (b->readOf[i][k] >= 0) q.zscores[k] = zs[j++];
            }
            refineZ.push_back(b->zOf[i]);
            refineIdx.push_back(i);
        }
        RefineOptions ro;
        ro.maxIterations = o.refine.max_iterations;
        ro.mutationSeparation = o.refine.mutation_separation;
        ro.mutationNeighborhood = o.refine.mutation_neighborhood;
        B.Retire(dropZ);
        std::vector<int> conv;
        std::vector<long long> nt, na;
        // ConsensusQVs (Consensus.h:496-512) run inside the refine loop, in the round each ZMW converges
        std::vector<std::vector<int>> qvAll;
        B.Refine(refineZ, ro, &conv, &nt, &na, false, reclaim ? &qvAll : nullptr);
        std::vector<int> qvZ, qvIdx;
        std::vector<std::vector<int>> qvs;
        for (size_t k = 0; k < refineZ.size(); ++k) {
            pbccs_zmw_output& q = out[refineIdx[k]];
            q.n_tested = nt[k];
            q.n_applied = na[k];
            if (conv[k] == 1) {
                qvZ.push_back(refineZ[k]);
                qvIdx.push_back(refineIdx[k]);
                if (reclaim) qvs.push_back(std::move(qvAll[k]));
            } else q.status = conv[k] < 0 ? PBCCS_ZMW_OTHER : PBCCS_ZMW_NON_CONVERGENT;
        }
        if (!reclaim) B.QVs(qvZ, &qvs);
        for (size_t k = 0; k < qvZ.size(); ++k) {
            pbccs_zmw_output& q = out[qvIdx[k]];
            const std::string& t = B.Template(qvZ[k]);
            double acc = 0.0;   // Consensus.h:506-512
            for (int v : qvs[k]) acc += std::pow(10.0, static_cast<double>(v) / -10.0);
            acc = 1.0 - acc / qvs[k].size();
            q.predicted_accuracy = acc;
            if ((int)t.size() + 1 > q.consensus_cap || !q.consensus) {
                q.consensus_len = -(int)t.size();
                q.status = PBCCS_ZMW_OTHER;
                continue;
            }
            std::memcpy(q.consensus, t.c_str(), t.size() + 1);
            q.consensus_len = (int)t.size();
            if (q.qvs) std::copy(qvs[k].begin(), qvs[k].end(), q.qvs);
            q.status = (acc < o.min_predicted_accuracy) ? PBCCS_ZMW_POOR_QUALITY : PBCCS_ZMW_SUCCESS;
        }
        return PBCCS_OK;
    });
}

// Create, polish, account and destroy one device batch of m ZMWs on `slot`.
static int polish_span(pbccs_engine* eng, int slot, const pbccs_zmw_input* in, int m, const pbccs_polish_options* o,
                       pbccs_zmw_output* out)
{
    pbccs_batch* h = nullptr;
    int r = create_batch(eng, in, m, o, slot, &h);
    if (r == PBCCS_OK) r = polish_one(h, out);
    if (h) {
        if (h->B) merge_engine_stats(eng, *h->B);
        pbccs_batch_destroy(h);
    }
    return r;
}

// Rerun ZMWs whose batch ran the device out of memory, alone on `slot` once the other slots have drained
// and every slot's band pool is unmapped; a span that still does not fit is halved.  A ZMW's result does
// not depend on the batch it polishes in (the engine's only cross-ZMW state is the launch grouping), so
// the retry changes the schedule and nothing else.  Outputs land in out[0..n) in input order.
static int polish_retry(pbccs_engine* eng, int slot, const pbccs_zmw_input* in, int n, const pbccs_polish_options* o,
                        pbccs_zmw_output* out)
{
    std::vector<std::pair<int, int>> todo{{0, n}};
    // the slot's outgrown buffers go back to the device before the rerun (nothing of the slot is queued: its batches
    // were destroyed, and the pools were unmapped with the device synchronised)
    eng->Slot(slot)->TrimRetired();
    while (!todo.empty()) {
        const std::pair<int, int> span = todo.back();
        todo.pop_back();
        {
            std::lock_guard<std::mutex> lk(eng->statsMu);
            eng->oomRetries += 1;
        }
        const int r = polish_span(eng, slot, in + span.first, span.second - span.first, o, out + span.first);
        if (r == PBCCS_OK) continue;
        if (r != PBCCS_EOOM || span.second - span.first < 2) return r;
        eng->Slot(slot)->val.unmap_all();
        const int mid = span.first + (span.second - span.first) / 2;
        todo.emplace_back(mid, span.second);
        todo.emplace_back(span.first, mid);
    }
    return PBCCS_OK;
}

int pbccs_batch_polish(pbccs_batch* b, pbccs_zmw_output* out)
{
    int rc = polish_one(b, out);
    if (b && b->B) merge_engine_stats(b->eng, *b->B);
    if (rc == PBCCS_EOOM && b) {   // alone on the device already: free this slot's pool and rerun, halving
        b->B.reset();
        b->eng->Slot(b->slot)->val.unmap_all();
        rc = polish_retry(b->eng, b->slot, b->inputs.in.data(), b->n, &b->o, out);
    }
    return rc;
}

int pbccs_batch_polish_many(pbccs_batch* const* batches, int n, pbccs_zmw_output* const* outs)
{
    if (n < 0 || (n > 0 && (!batches || !outs))) return fail(PBCCS_EINVAL, "bad argument");
    if (n == 0) return PBCCS_OK;
    pbccs_engine* eng = batches[0] ? batches[0]->eng : nullptr;
    for (int i = 0; i < n; ++i)
        if (!batches[i] || batches[i]->eng != eng || (batches[i]->n > 0 && !outs[i]))
            return fail(PBCCS_EINVAL, "batches must be non-null and belong to one engine");
    // one host thread (and HIP stream: each ArrowBatch owns one) per workspace slot
    std::vector<std::vector<int>> bySlot;
    for (int i = 0; i < n; ++i) {
        const int s = batches[i]->slot;
        if ((int)bySlot.size() <= s) bySlot.resize(s + 1);
        bySlot[s].push_back(i);
    }
    std::vector<int> rc(n, PBCCS_OK);
    std::vector<std::string> err(n);
    std::vector<std::thread> pool;
    for (const std::vector<int>& list : bySlot) {
        if (list.empty()) continue;
        pool.emplace_back([&, list] {
            for (int i : list) {   // polish_one and merge_engine_stats never throw
                rc[i] = polish_one(batches[i], outs[i]);
                if (rc[i] != PBCCS_OK) err[i] = g_lastError;
                if (batches[i]->B) merge_engine_stats(eng, *batches[i]->B);
            }
        });
    }
    for (std::thread& t : pool) t.join();
    // Batches that ran the device out of memory while the other slots held their pools are rebuilt from
    // their inputs and rerun one at a time, after every slot's pool is unmapped (halved while they still do
    // not fit).
    std::vector<int> deferred;
    for (int i = 0; i < n; ++i)
        if (rc[i] == PBCCS_EOOM) deferred.push_back(i);
    if (!deferred.empty()) {
        for (int i : deferred) batches[i]->B.reset();
        for (size_t s = 0; s < eng->slots.size(); ++s) eng->slots[s]->val.unmap_all();
        for (int i : deferred) {
            pbccs_batch* b = batches[i];
            rc[i] = polish_retry(eng, b->slot, b->inputs.in.data(), b->n, &b->o, outs[i]);
            if (rc[i] != PBCCS_OK) err[i] = g_lastError;
        }
    }
    for (int i = 0; i < n; ++i)
        if (rc[i] != PBCCS_OK) return fail(rc[i], err[i].c_str());
    return PBCCS_OK;
}

int pbccs_engine_set_concurrency(pbccs_engine* eng, int batches_in_flight)
{
    if (!eng || batches_in_flight < 1 || batches_in_flight > 64) return fail(PBCCS_EINVAL, "bad argument");
    eng->concurrency = batches_in_flight;
    return PBCCS_OK;
}

int pbccs_engine_reserve_pool(pbccs_engine* eng, size_t bytes_per_slot)
{
    if (!eng) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        if (hipSetDevice(eng->device) != hipSuccess) return fail(PBCCS_EDEVICE, "hipSetDevice failed");
        for (int s = 0; s < std::max(1, eng->concurrency); ++s) {
            VmPool& v = eng->Slot(s)->val;
            v.reserve(std::max<size_t>(bytes_per_slot / sizeof(double), 1), true);
            // touch the mapped memory once here, so first-use costs of fresh device pages are not paid by
            // the first fills that land on them
            if (hipMemsetAsync(v.ptr, 0, v.cap * sizeof(double), nullptr) != hipSuccess)
                return fail(PBCCS_EDEVICE, "hipMemset of the band pool failed");
        }
        if (hipDeviceSynchronize() != hipSuccess) return fail(PBCCS_EDEVICE, "device synchronisation failed");
        return PBCCS_OK;
    });
}

// ---- ZMW work queue ------------------------------------------------------------------------------
// Estimated FP64 band footprint of one ZMW at its high-water mark (zmw_est_bytes below).  Per read: two band
// regions of ~32 rows x window plus column metadata (the typical band), plus the expected share of bands that
// explode on the reband, whose fraction of the (I+1)(J+1) matrix grows with the window (oracle band statistics,
// DESIGN.md §6).  Checks: 2 kb / 10 passes ~19 MB (measured 13.5 MB, profiles/r2h6_regrow_slots), 10 kb / 8 passes
// ~150 MB with checkpointed bands (measured 142 MB: 68 GB for 480 ZMWs, profiles/r3b_bench_10kb_ckpt8.json),
// 20 kb ~120 MB per read (the round-4 estimate, 63 MB, let 8 slots run the device out of memory 27 times on the
// configs[3] mix).
// Band-pool bytes the workspace slots hold mapped.
static size_t slot_pool_bytes(pbccs_engine* eng)
{
    size_t b = 0;
    for (const auto& s : eng->slots) b += s->val.mapped_bytes();
    return b;
}

static double zmw_est_bytes(const pbccs_zmw_input& z)
{
    int K = 0, minLen = 0;
    ckpt_policy(&K, &minLen);
    double b = 0.0;
    for (int k = 0; k < z.n_reads; ++k) {
        const double J = std::max(1, z.tends ? z.tends[k] - (z.tstarts ? z.tstarts[k] : 0) : z.draft_len);
        const double I = z.lens ? std::max(0, z.lens[k]) : J;
        const double cells = (I + 1) * (J + 1);
        // the typical band: the first regions ((J + 66) x 16 values per matrix) and the column metadata
        const double typical = J * 0.5 * (2 * 32 * 8 * 1.25 + 80 + 8 * 8);
        // bands that explode on the 4%-of-matrix reband: the oracle's AddRead stores, per matrix, a mean fraction
        // of the (I+1)(J+1) matrix over all reads that grows with the window -- 0.023 / 0.044 / 0.074 / 0.098 at
        // 5 / 10 / 15 / 20 kb (6 reads each; 1 / 2 / 4 / 4 of them exploded to 0.05-0.21) -- held in exact regions
        // (+1/16 slack, regrow_bands), plus the tall reads' abandoned first regions (4% of the matrix, pt of the
        // reads: ~1 in 10 at 2 kb, 2 in 3 at 15-20 kb)
        const double frac = std::min(0.12, 0.005 * J / 1000.0);
        const double pt = std::min(0.7, 0.08 + J / 30000.0);
        double tall = 2.0 * 8.0 * frac * cells * (1.0 + 1.0 / 16) + pt * 2.0 * 8.0 * cells / 25.0;
        // checkpointed tall bands: every K-th column plus the kept tails of both matrices
        if (K > 0 && J >= minLen) tall = tall / K + pt * 2.0 * 8.0 * (kCkptTail + 1) * (I + 1);
        b += typical + tall;
    }
    // the refine rounds' per-ZMW buffers beside the bands: ~9 unique single-base mutations per template base
    // (Prepare's unique_mutation_count + 64), each with a code, a score, a flag and one delta per read (dDelta_:
    // 43 MB for a 20 kb template with 30 reads, which the band-only estimate missed: 5 OOM retries in the 2000-ZMW
    // configs[3] run, profiles/r5_mixed_2000_s8.json)
    const double L = std::max(1, z.draft_len);
    b += (9.0 * L + 64.0) * (8.0 * std::max(1, z.n_reads) + 13.0);
    return std::max(b, 4096.0);
}

int pbccs_plan_batches(const pbccs_zmw_input* in, int n, double budget_bytes, int max_per_batch,
                       double max_len_ratio, int* order, int* batch_start, double* est_bytes, int* n_batches)
{
    if (n < 0 || (n > 0 && (!in || !order || !batch_start)) || !n_batches || max_per_batch < 1 ||
        !(budget_bytes > 0) || !(max_len_ratio >= 1.0))
        return fail(PBCCS_EINVAL, "bad argument");
    std::vector<double> est(n);
    std::vector<int> idx(n);
    for (int i = 0; i < n; ++i) {
        est[i] = zmw_est_bytes(in[i]);
        idx[i] = i;
        if (est_bytes) est_bytes[i] = est[i];
    }
    // length buckets (then pass count): similar windows share launches, whose LDS and band heights are
    // sized by their longest read; the input index breaks ties so the plan is deterministic
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) {
        if (in[a].draft_len != in[b].draft_len) return in[a].draft_len < in[b].draft_len;
        return in[a].n_reads < in[b].n_reads;
    });
    struct Span { int b, e; double bytes; };
    std::vector<Span> spans;
    for (int k = 0; k < n;) {
        Span s{k, k, 0.0};
        const double first = std::max(1, in[idx[k]].draft_len);
        while (s.e < n) {
            const int z = idx[s.e];
            const bool room = s.e - s.b < max_per_batch && s.bytes + est[z] <= budget_bytes &&
                              in[z].draft_len <= max_len_ratio * first;
            if (!room && s.e > s.b) break;   // a ZMW over budget on its own still gets a batch
            s.bytes += est[z];
            ++s.e;
        }
        spans.push_back(s);
        k = s.e;
    }
    // longest templates first, then largest: a batch's time is its rounds' latency, which grows with the template
    // (the tall reads' column sweeps), not with its bytes -- most batches of a mixed input are capped at the same
    // budget, and ordered by bytes the 15-20 kb batches started last and left four of eight slots idle for the last
    // third of a configs[3] run (profiles/r9ze_mixed_slot_gaps.json); the queue's tail is then made of short batches
    std::vector<int> spanLen(spans.size());
    for (size_t k = 0; k < spans.size(); ++k) spanLen[k] = in[idx[spans[k].e - 1]].draft_len;   // ascending inside
    std::vector<size_t> so(spans.size());
    for (size_t k = 0; k < so.size(); ++k) so[k] = k;
    std::stable_sort(so.begin(), so.end(), [&](size_t a, size_t b) {
        if (spanLen[a] != spanLen[b]) return spanLen[a] > spanLen[b];
        return spans[a].bytes > spans[b].bytes;
    });
    std::vector<Span> sorted;
    for (size_t k : so) sorted.push_back(spans[k]);
    spans.swap(sorted);
    int o = 0;
    for (size_t b = 0; b < spans.size(); ++b) {
        batch_start[b] = o;
        for (int k = spans[b].b; k < spans[b].e; ++k) order[o++] = idx[k];
    }
    batch_start[spans.size()] = o;
    *n_batches = (int)spans.size();
    return PBCCS_OK;
}

int pbccs_polish_batch(pbccs_engine* eng, const pbccs_zmw_input* in, int n, const pbccs_polish_options* opts,
                       pbccs_zmw_output* out)
{
    if (!eng || n < 0 || (n > 0 && (!in || !out))) return fail(PBCCS_EINVAL, "bad argument");
    if (n == 0) return PBCCS_OK;
    pbccs_polish_options o;
    pbccs_polish_options_default(&o);
    if (opts) o = *opts;
    const int slots = std::max(1, eng->concurrency);
    std::vector<int> order(n), start(n + 1);
    int nb = 0;
    if (o.zmws_per_batch > 0) {   // caller-sized consecutive chunks
        for (int i = 0; i < n; ++i) order[i] = i;
        for (int b0 = 0; b0 < n; b0 += o.zmws_per_batch) start[nb++] = b0;
        start[nb] = n;
    } else {
        size_t freeB = 0, totalB = 0;
        if (hipSetDevice(eng->device) != hipSuccess || hipMemGetInfo(&freeB, &totalB) != hipSuccess)
            return fail(PBCCS_EDEVICE, "hipMemGetInfo failed");
        // every slot polishes at once: split what is free beyond the growth margin between them (the slots'
        // mapped band pools count as free: a batch on the slot reuses them)
        const double spare = std::max(0.0, (double)freeB + (double)slot_pool_bytes(eng) - (double)kQueueMargin);
        // PBCCS_QUEUE_BUDGET_SCALE (A/B): the per-slot budget against the planner's per-ZMW estimates
        const char* bs = std::getenv("PBCCS_QUEUE_BUDGET_SCALE");
        const double budget = std::max(1.0 * (1 << 30), 0.9 * spare / slots) * (bs ? std::max(0.1, std::atof(bs)) : 1.0);
        int rc = pbccs_plan_batches(in, n, budget, kQueueMaxZmws, 1.5, order.data(), start.data(), nullptr, &nb);
        if (rc != PBCCS_OK) return rc;
        // a last wave with fewer batches than slots leaves slots idle through its whole polish: cap the batch
        // size so the batches come in whole waves (smaller batches stay within the per-slot budget); small
        // inputs keep their plan, since batches of under ~256 ZMWs pay the per-round latency for too few
        if (nb % slots != 0 && n >= 256 * slots) {
            const int waves = (nb + slots - 1) / slots;
            const int per = std::max(1, (n + waves * slots - 1) / (waves * slots));
            rc = pbccs_plan_batches(in, n, budget, std::min(per, kQueueMaxZmws), 1.5, order.data(), start.data(),
                                    nullptr, &nb);
            if (rc != PBCCS_OK) return rc;
        }
    }
    // the workspace slots exist before the workers start (Slot() grows a shared vector)
    for (int s = 0; s < slots; ++s) eng->Slot(s);
    std::atomic<int> next{0};
    std::atomic<bool> stop{false};
    std::vector<int> rc(slots, PBCCS_OK);
    std::vector<std::string> err(slots);
    // a span [b, e) of `order`: inputs gathered, outputs scattered back to input order (also on failure:
    // the output structs only point at the caller's buffers)
    auto gather = [&](int b, int e, std::vector<pbccs_zmw_input>* bin, std::vector<pbccs_zmw_output>* bout) {
        bin->resize(e - b);
        bout->resize(e - b);
        for (int k = 0; k < e - b; ++k) {
            (*bin)[k] = in[order[b + k]];
            (*bout)[k] = out[order[b + k]];
        }
    };
    auto scatter = [&](int b, int e, const std::vector<pbccs_zmw_output>& bout) {
        for (int k = 0; k < e - b; ++k) out[order[b + k]] = bout[k];
    };
    // Batches that ran the device out of memory while the other slots held theirs are deferred and rerun
    // one at a time once every slot's pool is unmapped (polish_retry).
    std::mutex deferMu;
    std::vector<std::pair<int, int>> deferred;
    auto worker = [&](int slot) {
        std::vector<pbccs_zmw_input> bin;
        std::vector<pbccs_zmw_output> bout;
        for (;;) {
            const int b = next.fetch_add(1);
            if (b >= nb || stop.load()) return;
            int r = PBCCS_OK;
            try {
                gather(start[b], start[b + 1], &bin, &bout);
            } catch (...) {
                r = fail(PBCCS_EOOM, "out of host memory");
            }
            if (r == PBCCS_OK) r = polish_span(eng, slot, bin.data(), start[b + 1] - start[b], &o, bout.data());
            if (r == PBCCS_OK) {
                scatter(start[b], start[b + 1], bout);
            } else if (r == PBCCS_EOOM) {
                std::lock_guard<std::mutex> lk(deferMu);
                deferred.emplace_back(start[b], start[b + 1]);
                double est = 0.0;   // one line per deferred batch: what the plan expected, what ran out
                for (const pbccs_zmw_input& z : bin) est += zmw_est_bytes(z);
                std::fprintf(stderr, "[queue] batch %d (%d ZMWs, estimated %.1f GB) deferred on slot %d: %s\n", b,
                             start[b + 1] - start[b], est / 1e9, slot, g_lastError.c_str());
            } else {
                rc[slot] = r;
                err[slot] = g_lastError;
                stop.store(true);
                return;
            }
        }
    };
    std::vector<std::thread> pool;
    for (int s = 0; s < std::min(slots, nb); ++s) pool.emplace_back(worker, s);
    for (std::thread& t : pool) t.join();
    // every batch of the call is destroyed (its streams synchronised): the slots' outgrown buffers can go
    for (int s = 0; s < slots; ++s) eng->Slot(s)->TrimRetired();
    for (int s = 0; s < slots; ++s)
        if (rc[s] != PBCCS_OK) return fail(rc[s], err[s].c_str());
    if (!deferred.empty()) {
        for (int s = 0; s < slots; ++s) eng->Slot(s)->val.unmap_all();
        std::sort(deferred.begin(), deferred.end());
        return guarded([&] {
            std::vector<pbccs_zmw_input> bin;
            std::vector<pbccs_zmw_output> bout;
            for (const std::pair<int, int>& span : deferred) {
                gather(span.first, span.second, &bin, &bout);
                const int r = polish_retry(eng, 0, bin.data(), span.second - span.first, &o, bout.data());
                if (r != PBCCS_OK) return r;
                scatter(span.first, span.second, bout);
            }
            return PBCCS_OK;
        });
    }
    return PBCCS_OK;
}

int pbccs_engine_set_profiling(pbccs_engine* eng, int on)
{
    if (!eng) return fail(PBCCS_EINVAL, "null engine");
    eng->profiling = on != 0;
    return PBCCS_OK;
}

int pbccs_engine_kernel_stats(pbccs_engine* eng, pbccs_kernel_stat* out, int cap, int* n, int reset)
{
    if (!eng || !n) return fail(PBCCS_EINVAL, "bad argument");
    *n = kKernelKinds;
    if (!out || cap < kKernelKinds) return fail(PBCCS_ERANGE, "buffer too small");
    for (int k = 0; k < kKernelKinds; ++k) {
        std::memset(out[k].name, 0, sizeof(out[k].name));
        std::strncpy(out[k].name, kKernelNames[k], sizeof(out[k].name) - 1);
        out[k].launches = eng->stats[k].launches;
        out[k].device_ms = eng->stats[k].ms;
        out[k].cells = eng->stats[k].cells;
        out[k].bytes = eng->stats[k].bytes;
        out[k].wave_s = eng->stats[k].waveTicks / 1e8;   // s_memrealtime runs at 100 MHz
        if (reset) eng->stats[k] = KernelStat();
    }
    return PBCCS_OK;
}

}  // extern "C"

// ================================================================ Quiver family
#include "quiver_engine.hpp"

struct pbccs_quiver_scorer {
    pbccs_engine* eng = nullptr;
    std::unique_ptr<quiver::QuiverBatch> batch;
    std::vector<std::pair<std::string, int>> table;   // QuiverConfigTable: chemistry -> config index
    std::vector<pbccs_quiver_config> cfgs;
    int z = 0;
};

namespace {

quiver::QParams qparams(const pbccs_quiver_config& c)
{
    quiver::QParams p;
    const pbccs_qv_model_params& m = c.params;
    p.Match = m.match;
    p.Mismatch = m.mismatch;
    p.MismatchS = m.mismatch_s;
    p.Branch = m.branch;
    p.BranchS = m.branch_s;
    p.DeletionN = m.deletion_n;
    p.DeletionWithTag = m.deletion_with_tag;
    p.DeletionWithTagS = m.deletion_with_tag_s;
    p.Nce = m.nce;
    p.NceS = m.nce_s;
    for (int k = 0; k < 4; ++k) {
        p.Merge[k] = m.merge[k];
        p.MergeS[k] = m.merge_s[k];
    }
    p.scoreDiff = c.score_diff;
    p.fastThreshold = c.fast_score_threshold;
    p.addThreshold = c.add_threshold;
    p.moves = c.moves_available;
    p.sumProduct = c.sum_product ? 1 : 0;
    p.simple = (c.recursor == PBCCS_QV_RECURSOR_SPARSE_SIMPLE || c.recursor == PBCCS_QV_RECURSOR_DENSE_SIMPLE) ? 1 : 0;
    p.dense = (c.recursor == PBCCS_QV_RECURSOR_DENSE_SSE || c.recursor == PBCCS_QV_RECURSOR_DENSE_SIMPLE) ? 1 : 0;
    return p;
}

// Quiver mutations may lie past the template end: no read scores them (ReadScoresMutation, :60-71)
bool to_quiver_mutation(const pbccs_mutation& in, Mutation* out)
{
    if (in.type < 0 || in.type > 2 || in.start < 0) return false;
    const int width = in.end - in.start;
    if (in.type == PBCCS_INSERTION ? width != 0 : width != 1) return false;   // single-base only
    if (in.type != PBCCS_DELETION && !(in.new_base == 'A' || in.new_base == 'C' || in.new_base == 'G' || in.new_base == 'T'))
        return false;
    *out = Mutation::Make(in.type, in.start, in.new_base);
    return true;
}

int quiver_codes(const pbccs_mutation* m, int n, std::vector<int>* codes)
{
    for (int i = 0; i < n; ++i) {
        Mutation mu;
        if (!to_quiver_mutation(m[i], &mu)) return fail(PBCCS_EINVAL, "invalid single-base mutation");
        codes->push_back(mutation_code(mu));
    }
    return PBCCS_OK;
}

}  // namespace

extern "C" {

int pbccs_quiver_scorer_create(pbccs_engine* eng, const pbccs_quiver_config* configs, const char* const* chemistries,
                               int n_configs, const char* tpl, int tpl_len, pbccs_quiver_scorer** out)
{
    if (!eng || !configs || n_configs < 1 || !tpl || tpl_len <= 0 || !out) return fail(PBCCS_EINVAL, "bad argument");
    for (int k = 0; k < n_configs; ++k)
        if (configs[k].recursor < PBCCS_QV_RECURSOR_SPARSE_SSE || configs[k].recursor > PBCCS_QV_RECURSOR_DENSE_SIMPLE)
            return fail(PBCCS_EINVAL, "unknown recursor type");
    return guarded([&] {
        std::unique_ptr<pbccs_quiver_scorer> s(new pbccs_quiver_scorer());
        s->eng = eng;
        s->batch.reset(new quiver::QuiverBatch(eng->device));
        float fast = 0.0f;   // min over the table, starting at 0 (:129-135)
        for (int k = 0; k < n_configs; ++k) {
            const std::string name = (chemistries && chemistries[k]) ? chemistries[k] : "*";
            bool dup = false;
            for (auto& kv : s->table) dup = dup || kv.first == name;
            if (dup) continue;   // InsertAs_ keeps the first entry of a name (QuiverConfig.cpp:67-78)
            s->table.emplace_back(name, s->batch->AddConfig(qparams(configs[k])));
            s->cfgs.push_back(configs[k]);
            fast = std::min(fast, configs[k].fast_score_threshold);
        }
        s->z = s->batch->AddZmw(std::string(tpl, tpl_len), fast);
        *out = s.release();
        return PBCCS_OK;
    });
}

void pbccs_quiver_scorer_destroy(pbccs_quiver_scorer* s) { delete s; }

int pbccs_quiver_scorer_add_read(pbccs_quiver_scorer* s, const char* seq, int len, const float* ins_qv,
                                 const float* subs_qv, const float* del_qv, const float* del_tag,
                                 const float* merge_qv, const char* chemistry, int strand, int tstart, int tend,
                                 float threshold, int* active)
{
    if (!s || !seq || len <= 0 || !active || (strand != 0 && strand != 1)) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        // QuiverConfigTable::At: exact chemistry, else "*" (QuiverConfig.cpp:112-127)
        const std::string chem = chemistry ? chemistry : "*";
        int cfg = -1;
        size_t pos = 0;
        for (size_t k = 0; k < s->table.size(); ++k)
            if (s->table[k].first == chem) { cfg = s->table[k].second; pos = k; }
        if (cfg < 0)
            for (size_t k = 0; k < s->table.size(); ++k)
                if (s->table[k].first == "*") { cfg = s->table[k].second; pos = k; }
        if (cfg < 0) return fail(PBCCS_EINVAL, "Chemistry not found in QuiverConfigTable");
        quiver::QReadFeatures f;
        f.seq.assign(seq, len);
        auto track = [&](std::vector<float>& v, const float* src) {
            v.assign(len, 0.0f);
            if (src) std::copy(src, src + len, v.begin());
        };
        track(f.ins, ins_qv);
        track(f.subs, subs_qv);
        track(f.del, del_qv);
        track(f.tag, del_tag);
        track(f.merge, merge_qv);
        const float thr = std::isnan(threshold) ? s->cfgs[pos].add_threshold : threshold;
        *active = s->batch->AddRead(s->z, f, strand, tstart, tend, cfg, thr) ? 1 : 0;
        return PBCCS_OK;
    });
}

int pbccs_quiver_scorer_score_many(pbccs_quiver_scorer* s, const pbccs_mutation* m, int n, int fast, float* scores)
{
    if (!s || n < 0 || (n > 0 && (!m || !scores))) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        std::vector<int> codes;
        if (quiver_codes(m, n, &codes) != PBCCS_OK) return PBCCS_EINVAL;
        std::vector<float> d;
        s->batch->Deltas(s->z, codes, &d);
        for (int i = 0; i < n; ++i) scores[i] = s->batch->Score(s->z, d, i, fast != 0);
        return PBCCS_OK;
    });
}

int pbccs_quiver_scorer_read_score_mutation(pbccs_quiver_scorer* s, int i, const pbccs_mutation* m, float* score)
{
    if (!s || !m || !score || i < 0 || i >= s->batch->NumReads(s->z)) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        std::vector<int> codes;
        if (quiver_codes(m, 1, &codes) != PBCCS_OK) return PBCCS_EINVAL;
        *score = s->batch->ReadScoreMutation(s->batch->ReadIndex(s->z, i), codes[0]);
        return PBCCS_OK;
    });
}

int pbccs_quiver_scorer_scores(pbccs_quiver_scorer* s, const pbccs_mutation* m, float unscored, float* per_read)
{
    if (!s || !m || !per_read) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        std::vector<int> codes;
        if (quiver_codes(m, 1, &codes) != PBCCS_OK) return PBCCS_EINVAL;
        std::vector<float> d;
        s->batch->Deltas(s->z, codes, &d);
        const int nr = s->batch->NumReads(s->z);
        for (int k = 0; k < nr; ++k) per_read[k] = std::isnan(d[k]) ? unscored : d[k];
        return PBCCS_OK;
    });
}

int pbccs_quiver_scorer_is_favorable(pbccs_quiver_scorer* s, const pbccs_mutation* m, int fast, int* favorable)
{
    if (!s || !m || !favorable) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        std::vector<int> codes;
        if (quiver_codes(m, 1, &codes) != PBCCS_OK) return PBCCS_EINVAL;
        std::vector<float> d;
        s->batch->Deltas(s->z, codes, &d);
        *favorable = fast ? (s->batch->FastIsFavorable(s->z, d, 0) ? 1 : 0)
                          : ((double)s->batch->Score(s->z, d, 0, false) > 0.04 ? 1 : 0);
        return PBCCS_OK;
    });
}

int pbccs_quiver_scorer_apply_mutations(pbccs_quiver_scorer* s, const pbccs_mutation* m, int n)
{
    if (!s || n < 0 || (n > 0 && !m)) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        std::vector<Mutation> muts;
        for (int i = 0; i < n; ++i) {
            Mutation mu;
            if (!to_quiver_mutation(m[i], &mu)) return fail(PBCCS_EINVAL, "invalid mutation");
            muts.push_back(mu);
        }
        if (!s->batch->ApplyMutations(s->z, muts)) return fail(PBCCS_EINVAL, "mutation outside the template");
        return PBCCS_OK;
    });
}

int pbccs_quiver_scorer_template(pbccs_quiver_scorer* s, int strand, char* out, int cap, int* len)
{
    if (!s || !out || !len) return fail(PBCCS_EINVAL, "bad argument");
    const std::string t = strand ? reverse_complement(s->batch->Template(s->z)) : s->batch->Template(s->z);
    *len = (int)t.size();
    if ((int)t.size() + 1 > cap) return fail(PBCCS_ERANGE, "buffer too small");
    std::memcpy(out, t.c_str(), t.size() + 1);
    return PBCCS_OK;
}

int pbccs_quiver_scorer_num_reads(pbccs_quiver_scorer* s) { return s ? s->batch->NumReads(s->z) : -1; }

int pbccs_quiver_scorer_read_info(pbccs_quiver_scorer* s, int i, int* active, int* strand, int* tstart, int* tend)
{
    if (!s || i < 0 || i >= s->batch->NumReads(s->z)) return fail(PBCCS_EINVAL, "bad argument");
    const int r = s->batch->ReadIndex(s->z, i);
    if (active) *active = s->batch->Active(r) ? 1 : 0;
    if (strand) *strand = s->batch->Strand(r);
    if (tstart) *tstart = s->batch->Ts(r);
    if (tend) *tend = s->batch->Te(r);
    return PBCCS_OK;
}

int pbccs_quiver_scorer_baseline_score(pbccs_quiver_scorer* s, float* score)
{
    if (!s || !score) return fail(PBCCS_EINVAL, "bad argument");
    *score = s->batch->BaselineScore(s->z);
    return PBCCS_OK;
}

int pbccs_quiver_scorer_baseline_scores(pbccs_quiver_scorer* s, float* out, int cap, int* n)
{
    if (!s || !n) return fail(PBCCS_EINVAL, "bad argument");
    std::vector<float> v;
    for (int k = 0; k < s->batch->NumReads(s->z); ++k) {
        const int r = s->batch->ReadIndex(s->z, k);
        if (s->batch->Active(r)) v.push_back(s->batch->ReadScore(r));
    }
    *n = (int)v.size();
    if ((int)v.size() > cap || (!out && !v.empty())) return fail(PBCCS_ERANGE, "buffer too small");
    std::copy(v.begin(), v.end(), out);
    return PBCCS_OK;
}

int pbccs_quiver_scorer_num_flipflops(pbccs_quiver_scorer* s, int* out)
{
    if (!s || !out) return fail(PBCCS_EINVAL, "bad argument");
    for (int k = 0; k < s->batch->NumReads(s->z); ++k) out[k] = s->batch->Flips(s->batch->ReadIndex(s->z, k));
    return PBCCS_OK;
}

int pbccs_quiver_scorer_allocated_entries(pbccs_quiver_scorer* s, int i, long long* alpha, long long* beta)
{
    if (!s || i < 0 || i >= s->batch->NumReads(s->z) || !alpha || !beta) return fail(PBCCS_EINVAL, "bad argument");
    const int r = s->batch->ReadIndex(s->z, i);
    *alpha = s->batch->Allocated(r, 0);
    *beta = s->batch->Allocated(r, 1);
    return PBCCS_OK;
}

int pbccs_quiver_scorer_alignment(pbccs_quiver_scorer* s, int i, char* target, char* query, int cap, int* len)
{
    if (!s || i < 0 || i >= s->batch->NumReads(s->z) || !len) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        std::string t, q;
        if (!s->batch->Alignment(s->batch->ReadIndex(s->z, i), &t, &q))
            return fail(PBCCS_ESTATE, "Alignment needs a Viterbi scorer and a read with a scorer");
        *len = (int)t.size();
        if ((int)t.size() > cap || !target || !query) return fail(PBCCS_ERANGE, "buffer too small");
        memcpy(target, t.data(), t.size());
        memcpy(query, q.data(), q.size());
        return PBCCS_OK;
    });
}

int pbccs_quiver_refine_consensus(pbccs_quiver_scorer* s, const pbccs_refine_options* opts, long long* n_tested,
                                  long long* n_applied, int* converged)
{
    if (!s || !n_tested || !n_applied || !converged) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        RefineOptions ro;
        if (opts) {
            ro.maxIterations = opts->max_iterations;
            ro.mutationSeparation = opts->mutation_separation;
            ro.mutationNeighborhood = opts->mutation_neighborhood;
        }
        bool conv = false;
        if (!s->batch->Refine(s->z, ro, n_tested, n_applied, &conv)) return fail(PBCCS_EINVAL, "invalid edit");
        *converged = conv ? 1 : 0;
        return PBCCS_OK;
    });
}

int pbccs_quiver_consensus_qvs(pbccs_quiver_scorer* s, int* qvs, int cap, int* n)
{
    if (!s || !n) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        const std::vector<int> q = s->batch->QVs(s->z);
        *n = (int)q.size();
        if ((int)q.size() > cap || !qvs) return fail(PBCCS_ERANGE, "buffer too small");
        std::copy(q.begin(), q.end(), qvs);
        return PBCCS_OK;
    });
}

int pbccs_qv_evaluator_moves(pbccs_engine* eng, const pbccs_qv_features* read, const char* tpl, int tpl_len,
                             const pbccs_qv_model_params* params, int pin_start, int pin_end, const int* i,
                             const int* j, int n, float* inc, float* del, float* extra, float* merge)
{
    if (!eng || !read || !read->seq || read->len < 0 || !tpl || tpl_len < 0 || !params || n < 0 ||
        (n > 0 && (!i || !j)))
        return fail(PBCCS_EINVAL, "bad argument");
    if (n == 0) return PBCCS_OK;
    return guarded([&] {
        if (hipSetDevice(eng->device) != hipSuccess) return fail(PBCCS_EDEVICE, "hipSetDevice failed");
        const int I = read->len;
        // one device block: QParams | 5 feature tracks | cells i, j | outputs | read bases | template
        pbccs_quiver_config c{};
        c.params = *params;
        c.moves_available = 15;
        const quiver::QParams qp = qparams(c);
        std::vector<float> feat((size_t)5 * std::max(I, 1), 0.0f);
        const float* tr[5] = {read->ins_qv, read->subs_qv, read->del_qv, read->del_tag, read->merge_qv};
        for (int k = 0; k < 5; ++k)
            if (tr[k]) std::copy(tr[k], tr[k] + I, feat.begin() + (size_t)k * std::max(I, 1));
        auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
        const size_t oP = 0, oF = up(sizeof(qp)), oI = oF + up(feat.size() * 4), oJ = oI + up((size_t)n * 4),
                     oO = oJ + up((size_t)n * 4), oS = oO + up((size_t)16 * n), oT = oS + up((size_t)I + 1),
                     top = oT + up((size_t)tpl_len + 1);
        std::vector<char> h(top, 0);
        std::memcpy(h.data() + oP, &qp, sizeof(qp));
        std::memcpy(h.data() + oF, feat.data(), feat.size() * 4);
        std::memcpy(h.data() + oI, i, (size_t)n * 4);
        std::memcpy(h.data() + oJ, j, (size_t)n * 4);
        std::memcpy(h.data() + oS, read->seq, I);
        std::memcpy(h.data() + oT, tpl, tpl_len);
        DevVec<char> d;
        d.reserve(top, false);
        hipStream_t st = nullptr;
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return fail(PBCCS_EDEVICE, "stream");
        struct StreamGuard {
            hipStream_t s;
            ~StreamGuard() { (void)hipStreamSynchronize(s); (void)hipStreamDestroy(s); }
        } guard{st};
        if (hipMemcpyAsync(d.ptr, h.data(), top, hipMemcpyHostToDevice, st) != hipSuccess)
            return fail(PBCCS_EDEVICE, "upload failed");
        const float* df = reinterpret_cast<const float*>(d.ptr + oF);
        const size_t F = std::max(I, 1);
        quiver::QRead r{d.ptr + oS, df, df + F, df + 2 * F, df + 3 * F, df + 4 * F, I};
        quiver::launch_qv_moves(r, reinterpret_cast<const quiver::QParams*>(d.ptr + oP), d.ptr + oT, tpl_len,
                                pin_start ? 1 : 0, pin_end ? 1 : 0, reinterpret_cast<const int*>(d.ptr + oI),
                                reinterpret_cast<const int*>(d.ptr + oJ), n, reinterpret_cast<float*>(d.ptr + oO), st);
        if (hipGetLastError() != hipSuccess) return fail(PBCCS_EDEVICE, "k_qv_moves launch failed");
        std::vector<float> out((size_t)4 * n);
        if (hipMemcpyAsync(out.data(), d.ptr + oO, out.size() * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return fail(PBCCS_EDEVICE, "download failed");
        float* dst[4] = {inc, del, extra, merge};
        for (int k = 0; k < 4; ++k)
            if (dst[k]) std::copy(out.begin() + (size_t)k * n, out.begin() + (size_t)(k + 1) * n, dst[k]);
        return PBCCS_OK;
    });
}

int pbccs_quiver_polish_batch(pbccs_engine* eng, const pbccs_quiver_config* configs, const char* const* chemistries,
                              int n_configs, const pbccs_quiver_zmw* zmws, int n, const pbccs_refine_options* opts,
                              pbccs_quiver_result* out)
{
    if (!eng || !configs || n_configs < 1 || n < 0 || (n > 0 && (!zmws || !out))) return fail(PBCCS_EINVAL, "bad argument");
    for (int k = 0; k < n_configs; ++k)
        if (configs[k].recursor < PBCCS_QV_RECURSOR_SPARSE_SSE || configs[k].recursor > PBCCS_QV_RECURSOR_DENSE_SIMPLE)
            return fail(PBCCS_EINVAL, "unknown recursor type");
    for (int z = 0; z < n; ++z) {
        if (!zmws[z].tpl || zmws[z].tpl_len <= 0 || zmws[z].n_reads < 0 || (zmws[z].n_reads > 0 && !zmws[z].reads))
            return fail(PBCCS_EINVAL, "bad pbccs_quiver_zmw");
        for (int r = 0; r < zmws[z].n_reads; ++r) {
            const pbccs_quiver_read& q = zmws[z].reads[r];
            if (!q.seq || q.len <= 0 || (q.strand != 0 && q.strand != 1)) return fail(PBCCS_EINVAL, "bad pbccs_quiver_read");
        }
    }
    if (n == 0) return PBCCS_OK;
    return guarded([&] {
        std::lock_guard<std::mutex> lock(eng->quiverMu);
        if (!eng->quiverBatch) {
            eng->quiverBatch.reset(new quiver::QuiverBatch(eng->device));
            eng->quiverBatch->PinHostPools();
        }
        quiver::QuiverBatch& qb = *eng->quiverBatch;
        qb.Reset();
        qb.SetProfiling(eng->profiling);
        // the QuiverConfigTable, as pbccs_quiver_scorer_create builds it
        std::vector<std::pair<std::string, int>> table;
        std::vector<const pbccs_quiver_config*> cfgs;
        float fast = 0.0f;
        for (int k = 0; k < n_configs; ++k) {
            const std::string name = (chemistries && chemistries[k]) ? chemistries[k] : "*";
            bool dup = false;
            for (auto& kv : table) dup = dup || kv.first == name;
            if (dup) continue;
            table.emplace_back(name, qb.AddConfig(qparams(configs[k])));
            cfgs.push_back(&configs[k]);
            fast = std::min(fast, configs[k].fast_score_threshold);
        }
        std::vector<int> zs(n);
        std::vector<quiver::QuiverBatch::ReadSpec> specs;
        std::vector<int> specZmw;
        for (int z = 0; z < n; ++z) {
            zs[z] = qb.AddZmw(std::string(zmws[z].tpl, zmws[z].tpl_len), fast);
            for (int r = 0; r < zmws[z].n_reads; ++r) {
                const pbccs_quiver_read& q = zmws[z].reads[r];
                const std::string chem = q.chemistry ? q.chemistry : "*";
                int cfg = -1;
                size_t pos = 0;
                for (size_t k = 0; k < table.size(); ++k)
                    if (table[k].first == chem) { cfg = table[k].second; pos = k; }
                if (cfg < 0)
                    for (size_t k = 0; k < table.size(); ++k)
                        if (table[k].first == "*") { cfg = table[k].second; pos = k; }
                if (cfg < 0) return fail(PBCCS_EINVAL, "Chemistry not found in QuiverConfigTable");
                quiver::QuiverBatch::ReadSpec sp;
                sp.z = zs[z];
                sp.strand = q.strand;
                sp.ts = q.tstart;
                sp.te = q.tend < 0 ? zmws[z].tpl_len : q.tend;
                sp.config = cfg;
                sp.threshold = std::isnan(q.threshold) ? cfgs[pos]->add_threshold : q.threshold;
                sp.seq = q.seq;
                sp.len = q.len;
                sp.track[0] = q.ins_qv;
                sp.track[1] = q.subs_qv;
                sp.track[2] = q.del_qv;
                sp.track[3] = q.del_tag;
                sp.track[4] = q.merge_qv;
                specs.push_back(sp);
                specZmw.push_back(z);
            }
        }
        // PBCCS_QUIVER_TRACE=1: one stderr line with the wall time of each phase (prepare, AddRead, refine, QVs)
        static const bool qtrace = std::getenv("PBCCS_QUIVER_TRACE") != nullptr;
        auto qt0 = std::chrono::steady_clock::now();
        auto lap = [&]() {
            const auto t = std::chrono::steady_clock::now();
            const double ms = std::chrono::duration<double, std::milli>(t - qt0).count();
            qt0 = t;
            return ms;
        };
        const double msPrep = lap();
        const std::vector<char> act = qb.AddReads(&specs);
        const double msAdd = lap();
        for (int z = 0; z < n; ++z) out[z].n_active = 0;
        for (size_t k = 0; k < act.size(); ++k) out[specZmw[k]].n_active += act[k];
        RefineOptions ro;
        if (opts) {
            ro.maxIterations = opts->max_iterations;
            ro.mutationSeparation = opts->mutation_separation;
            ro.mutationNeighborhood = opts->mutation_neighborhood;
        }
        std::vector<long long> nt, na;
        std::vector<char> conv, ok;
        qb.RefineMany(zs, ro, &nt, &na, &conv, &ok);
        const double msRefine = lap();
        std::vector<int> wantQv;
        for (int z = 0; z < n; ++z)
            if (out[z].qvs && ok[z]) wantQv.push_back(z);
        std::vector<int> qz;
        for (int z : wantQv) qz.push_back(zs[z]);
        const std::vector<std::vector<int>> qv = qz.empty() ? std::vector<std::vector<int>>() : qb.QVsMany(qz);
        if (qtrace)
            std::fprintf(stderr, "[quiver] scorers %d prepare %.1f ms addread %.1f ms refine %.1f ms qvs %.1f ms\n", n,
                         msPrep, msAdd, msRefine, lap());
        for (int z = 0; z < n; ++z) {
            pbccs_quiver_result& o = out[z];
            o.n_tested = nt[z];
            o.n_applied = na[z];
            o.converged = conv[z];
            o.ok = ok[z];
            const std::string& t = qb.Template(zs[z]);
            o.consensus_len = (int)t.size();
            if (o.consensus && o.consensus_cap >= (int)t.size()) memcpy(o.consensus, t.data(), t.size());
        }
        for (size_t k = 0; k < wantQv.size(); ++k) {
            pbccs_quiver_result& o = out[wantQv[k]];
            if (o.consensus_cap >= (int)qv[k].size()) std::copy(qv[k].begin(), qv[k].end(), o.qvs);
        }
        {
            std::lock_guard<std::mutex> lk(eng->statsMu);
            qb.CollectProfile(eng->stats);
        }
        return PBCCS_OK;
    });
}

// ---------------------------------------------------------------- POA draft

struct pbccs_sparse_poa {
    pbccs_engine* eng;
    poa::ZmwPoa z;
};

namespace {

int put_text(const std::string& s, char* out, int cap, int* len)
{
    if (len) *len = (int)s.size();
    if ((int)s.size() > cap || (!out && !s.empty())) return fail(PBCCS_ERANGE, "buffer too small");
    if (!s.empty()) memcpy(out, s.data(), s.size());
    return PBCCS_OK;
}

}  // namespace

int pbccs_poa_batch(pbccs_engine* eng, const pbccs_poa_input* in, int n, long long max_coverage, int min_coverage,
                    pbccs_poa_output* out)
{
    if (!eng || n < 0 || (n > 0 && (!in || !out)) || max_coverage < 1) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        std::vector<std::vector<std::string>> own(n);
        std::vector<std::vector<const std::string*>> reads(n);
        for (int z = 0; z < n; ++z) {
            if (in[z].n_reads < 0 || (in[z].n_reads > 0 && (!in[z].seqs || !in[z].lens)))
                return fail(PBCCS_EINVAL, "bad pbccs_poa_input");
            own[z].resize(in[z].n_reads);
            for (int r = 0; r < in[z].n_reads; ++r) {
                if (in[z].seqs[r] && in[z].lens[r] < 0) return fail(PBCCS_EINVAL, "negative read length");
                if (in[z].seqs[r]) own[z][r].assign(in[z].seqs[r], in[z].lens[r]);   // empty: key -1
            }
            for (int r = 0; r < in[z].n_reads; ++r) reads[z].push_back(in[z].seqs[r] ? &own[z][r] : nullptr);
        }
        std::vector<std::string> css;
        std::vector<std::vector<int>> keys, ext;
        std::vector<std::vector<char>> rc;
        {
            std::lock_guard<std::mutex> lk(eng->poaMu);
            poa::PoaBatch(eng->PoaRunners(), reads, max_coverage, min_coverage, &css, &keys, &rc, &ext);
        }
        bool range = false;
        for (int z = 0; z < n; ++z) {
            pbccs_poa_output& o = out[z];
            o.len = (int)css[z].size();
            o.n_keys = (int)rc[z].size();
            if (o.consensus && o.len <= o.cap) memcpy(o.consensus, css[z].data(), css[z].size());
            else range = true;
            for (int r = 0; r < in[z].n_reads; ++r)
                if (o.keys) o.keys[r] = keys[z][r];
            for (int k = 0; k < o.n_keys; ++k) {
                if (o.rc) o.rc[k] = rc[z][k];
                if (o.extents)
                    for (int e = 0; e < 4; ++e) o.extents[4 * k + e] = ext[z][4 * k + e];
            }
        }
        return range ? fail(PBCCS_ERANGE, "consensus buffer too small") : PBCCS_OK;
    });
}

int pbccs_sparse_poa_create(pbccs_engine* eng, pbccs_sparse_poa** out)
{
    if (!eng || !out) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        *out = new pbccs_sparse_poa{eng, poa::ZmwPoa()};
        return PBCCS_OK;
    });
}

void pbccs_sparse_poa_destroy(pbccs_sparse_poa* p) { delete p; }

int pbccs_sparse_poa_orient_and_add_read(pbccs_sparse_poa* p, const char* seq, int len, float min_score_to_add,
                                         int* key)
{
    if (!p || (!seq && len > 0) || len < 0 || !key) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        if (len == 0) {   // an empty read is never added (the rule of pbccs_poa_batch / pbccs_ccs_batch)
            *key = -1;
            return PBCCS_OK;
        }
        const std::string s(seq, len);
        if (p->z.graph.NumReads() == 0) {
            std::vector<int> path;
            p->z.graph.AddFirstRead(s, &path);
            p->z.readPaths.push_back(std::move(path));
            p->z.rc.push_back(0);
            *key = 0;
            return PBCCS_OK;
        }
        std::vector<poa::AlignRequest> req{poa::AlignRequest{&p->z.graph, s, poa::kLocal, true, min_score_to_add}};
        std::vector<poa::AlignResult> res;
        {
            std::lock_guard<std::mutex> lk(p->eng->poaMu);
            p->eng->Poa().Align(req, &res);
        }
        if (res[0].chosen < 0) {
            *key = -1;
            return PBCCS_OK;
        }
        p->z.readPaths.push_back(std::move(res[0].path));
        p->z.rc.push_back((char)res[0].chosen);
        *key = (int)p->z.readPaths.size() - 1;
        return PBCCS_OK;
    });
}

int pbccs_sparse_poa_find_consensus(pbccs_sparse_poa* p, int min_coverage, char* out, int cap, int* len, int* rc,
                                    int* extents, int* n_keys)
{
    if (!p || !len) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        std::vector<int> ext;
        const std::string css = p->z.readPaths.empty() ? std::string() : p->z.FindConsensus(min_coverage, &ext);
        const int nk = (int)p->z.rc.size();
        if (n_keys) *n_keys = nk;
        for (int k = 0; k < nk; ++k) {
            if (rc) rc[k] = p->z.rc[k];
            if (extents)
                for (int e = 0; e < 4; ++e) extents[4 * k + e] = ext[4 * k + e];
        }
        return put_text(css, out, cap, len);
    });
}

int pbccs_sparse_poa_graphviz(pbccs_sparse_poa* p, int flags, int min_coverage, char* out, int cap, int* len)
{
    if (!p || !len) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        std::vector<int> path;
        if (!p->z.readPaths.empty()) p->z.FindConsensus(min_coverage, nullptr, &path);
        return put_text(p->z.graph.GraphViz(flags & 1, flags & 2, &path), out, cap, len);
    });
}

int pbccs_poa_consensus(pbccs_engine* eng, const char* const* reads, const int* lens, int n, int mode,
                        int min_coverage, char* out, int cap, int* len, int flags, char* dot, int dot_cap,
                        int* dot_len)
{
    if (!eng || n < 0 || (n > 0 && (!reads || !lens)) || !len || mode < 0 || mode > 2)
        return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        poa::PoaGraph g;
        for (int r = 0; r < n; ++r) {
            if (!reads[r] || lens[r] <= 0) return fail(PBCCS_EINVAL, "Input sequences must have nonzero length.");
            const std::string s(reads[r], lens[r]);
            if (g.NumReads() == 0) {
                g.AddFirstRead(s, nullptr);
                continue;
            }
            std::vector<poa::AlignRequest> req{poa::AlignRequest{&g, s, (poa::AlignMode)mode, false, 0.f}};
            std::vector<poa::AlignResult> res;
            std::lock_guard<std::mutex> lk(eng->poaMu);
            eng->Poa().Align(req, &res);
        }
        const std::vector<int> path = g.ConsensusPath((poa::AlignMode)mode, min_coverage);
        if (dot) {
            const int rc = put_text(g.GraphViz(flags & 1, flags & 2, &path), dot, dot_cap, dot_len);
            if (rc != PBCCS_OK) return rc;
        }
        return put_text(g.Sequence(path), out, cap, len);
    });
}

int pbccs_poa_stats_get(pbccs_engine* eng, pbccs_poa_stats* out, int reset)
{
    if (!eng || !out) return fail(PBCCS_EINVAL, "bad argument");
    return guarded([&] {
        std::lock_guard<std::mutex> lk(eng->poaMu);
        poa::PoaStats s;
        for (poa::PoaRunner* r : eng->PoaRunners()) {   // counts add up; wall times are the slices' maxima
            const poa::PoaStats& x = r->stats;
            s.alignments += x.alignments;
            s.cells += x.cells;
            s.launches += x.launches;
            s.traceSteps += x.traceSteps;
            s.fillMs += x.fillMs;
            s.traceMs += x.traceMs;
            s.bytes += x.bytes;
            s.progMs = std::max(s.progMs, x.progMs);
            s.deviceMs = std::max(s.deviceMs, x.deviceMs);
            s.threadMs = std::max(s.threadMs, x.threadMs);
            s.consensusMs = std::max(s.consensusMs, x.consensusMs);
            s.totalMs = std::max(s.totalMs, x.totalMs);
            if (reset) r->stats = poa::PoaStats();
        }
        *out = pbccs_poa_stats{s.alignments, s.cells,  s.launches, s.traceSteps, s.fillMs,     s.traceMs,
                               s.bytes,      s.progMs, s.deviceMs, s.threadMs,  s.consensusMs, s.totalMs};
        return PBCCS_OK;
    });
}

// One POA chunk of the pipelined ccs batch: its live ZMWs and everything their polish inputs point into.
struct CcsChunk {
    std::vector<int> zs;   // caller indices of the chunk's ZMWs
    std::vector<std::string> css;
    std::vector<std::vector<driver::MappedRead>> mapped;
    std::vector<std::vector<const char*>> seqPtr;
    std::vector<std::vector<int>> lens, strands, ts, te;
    std::vector<std::vector<unsigned char>> full;
    std::vector<pbccs_zmw_input> pin;   // the ZMWs that reach the polish
    std::vector<int> pinZ;
    std::vector<pbccs_zmw_output> pout;
    // per-read polish outputs by position in the polish input (FilterReads order up to the maxPoaCov stop);
    // scattered back to the caller's subread order once the chunk's polish is final
    std::vector<std::vector<int>> arr;
    std::vector<std::vector<double>> zsc;
    bool draftRange = false;   // a draft longer than its caller buffer
};

// The chunk's polish outputs: the caller's pbccs_zmw_output fields, but per-read arrays owned by the chunk.
static void bind_polish_outputs(CcsChunk* C, const pbccs_ccs_output* out)
{
    for (size_t q = 0; q < C->pinZ.size(); ++q) {
        C->pout[q] = out[C->pinZ[q]].polish;
        C->pout[q].add_read_results = C->arr[q].data();
        C->pout[q].zscores = C->zsc[q].data();
    }
}

// The POA draft of one chunk (Consensus.h:422-425, 352-390), then TooShort and ExtractMappedRead
// (Consensus.h:427-471) into the chunk's polish inputs.
static void ccs_draft_chunk(pbccs_engine* eng, const pbccs_ccs_input* in, const pbccs_polish_options& o,
                            long long max_poa_coverage, const std::vector<std::vector<driver::Subread>>& sub,
                            const std::vector<std::vector<int>>& order, pbccs_ccs_output* out, CcsChunk* C)
{
    const size_t m = C->zs.size();
    std::vector<std::vector<const std::string*>> poaReads(m);
    for (size_t q = 0; q < m; ++q)
        for (int k : order[C->zs[q]]) poaReads[q].push_back(k >= 0 ? &sub[C->zs[q]][k].seq : nullptr);
    std::vector<std::vector<int>> keys, ext;
    std::vector<std::vector<char>> rc;
    poa::PoaBatch(eng->PoaRunners(), poaReads, max_poa_coverage, -1, &C->css, &keys, &rc, &ext);
    C->mapped.resize(m);
    C->seqPtr.resize(m);
    C->lens.resize(m);
    C->strands.resize(m);
    C->ts.resize(m);
    C->te.resize(m);
    C->full.resize(m);
    for (size_t q = 0; q < m; ++q) {
        const int z = C->zs[q];
        const std::string& css = C->css[q];
        if (out[z].draft) {
            if (out[z].draft_cap >= (int)css.size()) memcpy(out[z].draft, css.data(), css.size());
            else C->draftRange = true;
        }
        out[z].draft_len = (int)css.size();
        if ((int)css.size() < o.min_length) {
            out[z].polish.status = PBCCS_ZMW_TOO_SHORT;
            continue;
        }
        std::vector<unsigned char> added;
        const std::vector<int>& kk = keys[q];
        for (size_t i = 0; i < kk.size() && kk[i] != -2; ++i) {
            driver::MappedRead mr;
            const int key = kk[i];
            const bool ok = key >= 0 &&
                            driver::ExtractMappedRead(sub[z][order[z][i]], rc[q][key] != 0, ext[q][4 * key],
                                                      ext[q][4 * key + 1], ext[q][4 * key + 2], ext[q][4 * key + 3],
                                                      (size_t)o.min_length, &mr);
            C->mapped[q].push_back(ok ? mr : driver::MappedRead());
            added.push_back(ok ? 1 : 0);
            C->full[q].push_back(ok && sub[z][order[z][i]].FullPass() ? 1 : 0);
        }
        for (size_t i = 0; i < C->mapped[q].size(); ++i) {
            const driver::MappedRead& mr = C->mapped[q][i];
            C->seqPtr[q].push_back(added[i] ? mr.seq.data() : nullptr);
            C->lens[q].push_back((int)mr.seq.size());
            C->strands[q].push_back(mr.strand);
            C->ts[q].push_back(mr.ts);
            C->te[q].push_back(mr.te);
        }
        pbccs_zmw_input zi;
        zi.draft = css.data();
        zi.draft_len = (int)css.size();
        for (int b = 0; b < 4; ++b) zi.snr[b] = in[z].snr[b];
        zi.n_reads = (int)C->mapped[q].size();
        zi.seqs = C->seqPtr[q].data();
        zi.lens = C->lens[q].data();
        zi.strands = C->strands[q].data();
        zi.tstarts = C->ts[q].data();
        zi.tends = C->te[q].data();
        zi.full_pass = C->full[q].data();
        C->pin.push_back(zi);
        C->pinZ.push_back(z);
        C->pout.push_back(out[z].polish);
        C->arr.emplace_back(std::max<size_t>(1, C->mapped[q].size()), -1);
        C->zsc.emplace_back(std::max<size_t>(1, C->mapped[q].size()), std::numeric_limits<double>::quiet_NaN());
    }
    bind_polish_outputs(C, out);
}

int pbccs_ccs_batch(pbccs_engine* eng, const pbccs_ccs_input* in, int n, long long max_poa_coverage,
                    const pbccs_polish_options* opts, pbccs_ccs_output* out)
{
    if (!eng || n < 0 || (n > 0 && (!in || !out)) || max_poa_coverage < 1) return fail(PBCCS_EINVAL, "bad argument");
    pbccs_polish_options o;
    if (opts) o = *opts;
    else pbccs_polish_options_default(&o);
    return guarded([&] {
        // FilterReads per ZMW (Consensus.h:411-420)
        std::vector<std::vector<driver::Subread>> sub(n);
        std::vector<std::vector<int>> order(n);
        std::vector<int> live;
        for (int z = 0; z < n; ++z) {
            if (in[z].n_subreads < 0 || (in[z].n_subreads > 0 && (!in[z].seqs || !in[z].lens)))
                return fail(PBCCS_EINVAL, "bad pbccs_ccs_input");
            for (int r = 0; r < in[z].n_subreads; ++r)
                if (in[z].lens[r] < 0 || (in[z].lens[r] > 0 && !in[z].seqs[r]))
                    return fail(PBCCS_EINVAL, "bad subread (NULL sequence or negative length)");
        }
        for (int z = 0; z < n; ++z) {   // every per-read slot starts as "not added"
            for (int r = 0; r < in[z].n_subreads; ++r) {
                if (out[z].add_order) out[z].add_order[r] = -1;
                if (out[z].polish.add_read_results) out[z].polish.add_read_results[r] = -1;
                if (out[z].polish.zscores) out[z].polish.zscores[r] = std::numeric_limits<double>::quiet_NaN();
            }
        }
        for (int z = 0; z < n; ++z) {
            for (int r = 0; r < in[z].n_subreads; ++r) {
                driver::Subread s;
                if (in[z].lens[r] > 0) s.seq.assign(in[z].seqs[r], in[z].lens[r]);
                if (in[z].flags) s.flags = in[z].flags[r];
                sub[z].push_back(std::move(s));
            }
            order[z] = driver::FilterReads(sub[z], (size_t)o.min_length);
            bool any = false;
            for (int k : order[z]) any = any || k >= 0;
            if (any) live.push_back(z);
            else {
                out[z].polish.status = PBCCS_ZMW_NO_SUBREADS;
                out[z].draft_len = 0;
            }
        }
        if (live.empty()) return PBCCS_OK;
        std::lock_guard<std::mutex> poaLock(eng->poaMu);
        // Chunks: one POA batch each, polished as one device batch on a workspace slot while the next chunk's
        // POA runs.  They are planned like pbccs_polish_batch's batches, from each ZMW's filtered subreads
        // (the median length standing in for the draft): length buckets and the per-slot share of the HBM
        // left beside the POA's score pools.  No whole-wave split: the chunks reach the slots one POA apart,
        // and larger chunks keep both stages busier (2000-ZMW chunks measured 1544 ZMWs/s end to end against
        // 1384 for 1000 and 1066 for 500).
        const int slots = std::max(1, eng->concurrency);
        // 40 GB over the slices (kPoaSlicesDefault = 3: 13.3 GB each).  One read round of a 2 kb slice costs
        // ~17.7 MB per ZMW (17.7 GB for 1000 ZMWs), so a 2000-ZMW chunk's ~667-ZMW slices need ~11.8 GB
        const size_t kPoaPoolPerSlice = (40ull << 30) / (size_t)pbccs_engine::PoaSlices();
        for (poa::PoaRunner* r : eng->PoaRunners()) r->SetPoolBudget(kPoaPoolPerSlice);
        std::vector<std::vector<int>> liveLens(live.size());
        std::vector<pbccs_zmw_input> est(live.size());
        for (size_t q = 0; q < live.size(); ++q) {
            const int z = live[q];
            std::vector<int> kept;
            for (int k : order[z])
                if (k >= 0) liveLens[q].push_back(in[z].lens[k]);
            kept = liveLens[q];
            std::sort(kept.begin(), kept.end());
            std::memset(&est[q], 0, sizeof(est[q]));
            est[q].draft_len = kept[kept.size() / 2];
            est[q].n_reads = (int)liveLens[q].size();
            est[q].lens = liveLens[q].data();
        }
        size_t freeB = 0, totalB = 0;
        if (hipSetDevice(eng->device) != hipSuccess || hipMemGetInfo(&freeB, &totalB) != hipSuccess)
            return fail(PBCCS_EDEVICE, "hipMemGetInfo failed");
        size_t poaMapped = 0;
        for (poa::PoaRunner* r : eng->PoaRunners()) poaMapped += r->PoolMappedBytes();
        const double spare = std::max(0.0, (double)freeB + (double)poaMapped + (double)slot_pool_bytes(eng) - kQueueMargin -
                                               (double)(kPoaPoolPerSlice * eng->PoaRunners().size()));
        const double budget = std::max(1.0 * (1 << 30), 0.9 * spare / slots);
        const int nl = (int)live.size();
        std::vector<int> perm(nl), start(nl + 1);
        int nb = 0;
        int rcp = PBCCS_OK;
        if (o.zmws_per_batch > 0) {   // caller-sized consecutive chunks
            for (int i = 0; i < nl; ++i) perm[i] = i;
            for (int b0 = 0; b0 < nl; b0 += o.zmws_per_batch) start[nb++] = b0;
            start[nb] = nl;
        } else {
            // about ten chunks per call, 1000-2000 ZMWs each: the POA of chunk k + 1 runs beside the polish of chunk
            // k, so the first draft and the last polish are the pipeline's fill and drain -- at 10,000 ZMWs 1000-ZMW
            // chunks ran 1943 / 1917 ZMWs/s against 1717 / 1850 for 2000, at 20,000 2000-ZMW chunks won (1986 / 1987
            // vs 1874 / 1852; profiles/r9zt_ccs_chunk_ab.txt)
            const int cap = std::max(std::min(nl / 10, kQueueMaxZmws), std::min(1000, kQueueMaxZmws));
            rcp = pbccs_plan_batches(est.data(), nl, budget, cap, 1.5, perm.data(), start.data(), nullptr, &nb);
        }
        if (rcp != PBCCS_OK) return rcp;
        std::vector<CcsChunk> chunks(nb);
        for (int c = 0; c < nb; ++c)
            for (int k = start[c]; k < start[c + 1]; ++k) chunks[c].zs.push_back(live[perm[k]]);
        // consumers: the polish slots pull drafted chunks as the producer (this thread) finishes them
        for (int s = 0; s < slots; ++s) eng->Slot(s);
        std::mutex qmu;
        std::condition_variable qcv;
        // work items (chunk, first, end) over each chunk's polish inputs: a chunk is one item, except the last
        // one, whose polish is the run's tail with the other slots idle: it is cut into one piece per slot (a
        // polish batch's time is its refine rounds' latency, ~1.1 s for a few hundred ZMWs against ~1.8 s for
        // 2000, so parallel pieces shorten the tail; earlier chunks stay whole, their pieces would only queue)
        std::vector<std::array<int, 3>> work;
        int drafted = 0, next = 0;
        bool stop = false;
        std::vector<int> prc(nb, PBCCS_OK);
        std::vector<std::string> perr(nb);
        // PBCCS_CCS_TRACE=1: one stderr line per chunk stage (ms since the call began)
        static const bool trace = std::getenv("PBCCS_CCS_TRACE") != nullptr;
        const auto tBegin = std::chrono::steady_clock::now();
        auto since = [&] {
            return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tBegin).count();
        };
        auto worker = [&](int slot) {
            for (;;) {
                std::array<int, 3> w;
                {
                    std::unique_lock<std::mutex> lk(qmu);
                    qcv.wait(lk, [&] { return stop || next < drafted; });
                    if (next >= drafted) return;   // stopped with nothing left
                    w = work[next++];
                }
                const int c = w[0], lo = w[1], hi = w[2];
                CcsChunk& C = chunks[c];
                if (hi <= lo) continue;
                const double p0 = since();
                const int rc = polish_span(eng, slot, C.pin.data() + lo, hi - lo, &o, C.pout.data() + lo);
                if (trace)
                    std::fprintf(stderr, "[ccs] chunk %d polish slot %d zmws %d %.1f-%.1f ms\n", c, slot, hi - lo, p0,
                                 since());
                if (rc != PBCCS_OK) {
                    std::lock_guard<std::mutex> lk(qmu);
                    if (prc[c] == PBCCS_OK || rc != PBCCS_EOOM) prc[c] = rc;   // EOOM: the chunk reruns whole below
                    if (rc != PBCCS_EOOM) {
                        perr[c] = g_lastError;
                        stop = true;
                        qcv.notify_all();
                        return;
                    }
                }
            }
        };
        // PBCCS_CCS_SERIAL=1: every chunk drafted before the first polishes (the A/B reference schedule)
        const char* serialEnv = std::getenv("PBCCS_CCS_SERIAL");
        const bool serial = serialEnv && serialEnv[0] == '1';
        std::vector<std::thread> pool;
        if (!serial)
            for (int s = 0; s < std::min(slots, nb); ++s) pool.emplace_back(worker, s);
        int rcDraft = PBCCS_OK;
        std::string errDraft;
        for (int c = 0; c < nb; ++c) {
            {
                std::lock_guard<std::mutex> lk(qmu);
                if (stop) break;
            }
            const double d0 = since();
            try {
                ccs_draft_chunk(eng, in, o, max_poa_coverage, sub, order, out, &chunks[c]);
                if (trace)
                    std::fprintf(stderr, "[ccs] chunk %d draft zmws %zu %.1f-%.1f ms\n", c, chunks[c].zs.size(), d0,
                                 since());
            } catch (const std::bad_alloc&) {
                rcDraft = PBCCS_EOOM;
                errDraft = "out of memory in the POA draft";
            } catch (const std::exception& e) {
                rcDraft = PBCCS_EDEVICE;
                errDraft = e.what();
            }
            std::lock_guard<std::mutex> lk(qmu);
            if (rcDraft != PBCCS_OK) {
                stop = true;
            } else {
                const int m = (int)chunks[c].pin.size();
                const char* pe = std::getenv("PBCCS_CCS_TAIL_PIECE");   // test hook: smaller pieces
                const int piece = pe ? std::max(1, std::atoi(pe)) : kCcsTailPiece;
                const int pieces = c + 1 < nb ? 1 : std::max(1, std::min(slots, m / piece));
                for (int k = 0; k < pieces; ++k)
                    work.push_back({c, (int)((long long)m * k / pieces), (int)((long long)m * (k + 1) / pieces)});
                drafted = (int)work.size();
            }
            qcv.notify_all();
            if (rcDraft != PBCCS_OK) break;
        }
        {
            std::lock_guard<std::mutex> lk(qmu);
            stop = true;   // every drafted chunk is still taken: workers leave once next == drafted
            qcv.notify_all();
        }
        if (serial) {
            for (poa::PoaRunner* r : eng->PoaRunners()) r->ReleasePool();
            for (int s = 0; s < std::min(slots, nb); ++s) pool.emplace_back(worker, s);
        }
        for (std::thread& t : pool) t.join();
        for (int s = 0; s < slots; ++s) eng->Slot(s)->TrimRetired();   // every chunk's batch is destroyed
        for (poa::PoaRunner* r : eng->PoaRunners()) {
            r->ReleasePool();
            r->SetPoolBudget(0);
        }
        if (rcDraft != PBCCS_OK) return fail(rcDraft, errDraft.c_str());
        for (int c = 0; c < nb; ++c)
            if (prc[c] != PBCCS_OK && prc[c] != PBCCS_EOOM) return fail(prc[c], perr[c].c_str());
        // chunks that ran the device out of memory beside the others: rerun alone once every pool is unmapped
        bool unmapped = false;
        for (int c = 0; c < nb; ++c) {
            if (prc[c] != PBCCS_EOOM) continue;
            if (!unmapped) {
                for (int s = 0; s < slots; ++s) eng->Slot(s)->val.unmap_all();
                unmapped = true;
            }
            CcsChunk& C = chunks[c];
            bind_polish_outputs(&C, out);
            const int r = polish_retry(eng, 0, C.pin.data(), (int)C.pin.size(), &o, C.pout.data());
            if (r != PBCCS_OK) return r;
        }
        bool draftRange = false;
        for (const CcsChunk& C : chunks) {
            draftRange = draftRange || C.draftRange;
            for (size_t q = 0; q < C.pinZ.size(); ++q) {
                const int z = C.pinZ[q];
                pbccs_zmw_output& po = out[z].polish;
                int* const arrOut = po.add_read_results;
                double* const zsOut = po.zscores;
                po = C.pout[q];
                po.add_read_results = arrOut;
                po.zscores = zsOut;
                // polish position i is FilterReads' i-th read, i.e. caller subread order[z][i]; the scorer's reads
                // (AddRead calls) are the positions with a result, in position order
                int added = 0;
                for (size_t i = 0; i < C.mapped[q].size(); ++i) {
                    const int k = order[z][i];
                    if (k < 0) continue;
                    if (arrOut) arrOut[k] = C.arr[q][i];
                    if (zsOut) zsOut[k] = C.zsc[q][i];
                    if (out[z].add_order && C.arr[q][i] >= 0) out[z].add_order[added++] = k;
                }
            }
        }
        return draftRange ? fail(PBCCS_ERANGE, "draft buffer too small") : PBCCS_OK;
    });
}

}  // extern "C"
