#!/usr/bin/env python3
"""CCS polish throughput on MI355X (BASELINE.json metric: CCS ZMWs/sec and GCUPS).

A step polishes one batch of synthetic ZMWs (2 kb insert, 10 full passes, 2000
ZMWs per batch) end to end on the GPU: AddRead fills + z-score gates, RefineConsensus, ConsensusQVs -- the
per-ZMW polish that pbccs' Consensus.h runs after the POA.  Inputs are copied to HBM before the timed region
(pbccs_batch_create); the timed region is exactly K steps, bracketed by a barrier and
torch.cuda.synchronize() on both sides; the job time is the max over ranks.  The K steps are pipelined over
S workspace slots (pbccs_batch_polish_many: one host thread + HIP stream per slot), so one batch's
convergence tail -- the last refine rounds of its few slow ZMWs -- overlaps the others' work, the way ccs's
ZMW thread pool overlaps ZMWs.  Each step's ZMWs are polished as BATCH_SPLIT device batches on S = 8 slots (the
measured best shape, profiles/r4u_batch_shape.txt), capped by what fits in HBM.

Multi-GPU: `--gpus N` without a launcher spawns N ranks itself (one process per GPU, RANK/LOCAL_RANK/
WORLD_SIZE set before any HIP call; the parent never touches the GPU); under torch.distributed.run the
launcher's ranks are used.  Each rank polishes its own K steps (weak scaling, no data-path collective);
rank 0 prints one JSON line.
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# Every batch in flight polishes on its own HIP streams; with HIP's default of 4 hardware queues the
# streams of different batches share queues and a long fill of one batch blocks the others' short
# kernels.  Must be set before the HIP runtime initialises (measured: 634 -> 1180 ZMWs/s).
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:   # the boxes export HIP's default (4)
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# PMC HBM bytes per launch of each fill kind (tools/gpu_steps.sh traffic -> tools/pmc_traffic.py); used only while
# the kernel sources still hash to the digest the profile was taken at
TRAFFIC_PROFILES = {"k_fill_tall": "r6_traffic_fill_tall.json", "k_fill": "r6_traffic_fill.json",
                    "k_score": "r6_traffic_score.json"}
# the same command on one workspace slot (--streams 1): the dominant kernel's launch duration there is not
# time-shared with other batches' launches; used only while the kernel sources hash to its digest
SINGLE_SLOT_PROFILE = "r6_streams1_bench.json"
FP64_VALU_PEAK_TFLOPS = 78.6   # MI355X FP64 vector peak (spec)
FLOP_PER_CELL = 11             # fill cell 6 mul + 3 add + <= 1 div, + the column rescale
CHAIN_ROW_CYCLES = 21.5        # one band row of the tall fills' chain at 2 rows per lane (tools/ubench/chain_step.hip
                               # variant C2; 29.3 with a DPP hand-off per row, profiles/r4a_chain_ubench.txt)
BEST_SLOTS = 8                 # 2 kb: eight slots of 1000-ZMW device batches (each 2000-ZMW step polished as two batches,
                               # BATCH_SPLIT): 3677 / 3665 ZMWs/s against 3538 / 3525 for five slots of whole steps and
                               # 3094 / 3049 for ten of halves (twenty streams on sixteen hardware queues),
                               # profiles/r4u_batch_shape.txt; 40 half-steps fill the eight slots in five full waves
BATCH_SPLIT = 2                # device batches per 2 kb step
BEST_SLOTS_CCS = 8             # ccs: polish chunks planned from free HBM beside the POA (profiles/r4y_ccs_shape_ab.txt: 8 > 5)
BEST_SLOTS_LONG = 8            # configs[2] / [3] through the work queue: 10 kb at 2000 ZMWs 4 / 5 / 8 / 10 / 12 slots 27.5 / 26.3 / 29.1-30.4 / 28.0 / 26.5 ZMWs/s (profiles/r3ad_*, r3af_*); mixed at 240 ZMWs 8 / 12 slots 7.19 / 5.09 (profiles/r3ag_*): more, smaller batches in flight while the tall fills set each round's latency
SLOT_BYTES_PER_ZMW = 15 << 20  # measured band high-water per 2 kb / 10-pass ZMW in a slot (13.4 MB, exact regrow)
HBM_MARGIN = 24 << 30          # device memory left to scratch, selection buffers and the runtime


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--zmws-per-step", type=int, default=2000)
    ap.add_argument("--length", type=int, default=2000)
    ap.add_argument("--passes", type=int, default=10)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--workload", choices=["2kb", "10kb", "mixed", "smrtcell"], default="2kb",
                    help="2kb: configs[1], the headline line (pre-created batches, inputs resident in HBM). "
                         "10kb / mixed: configs[2] / configs[3] through the ZMW work queue (polish_stream: "
                         "length/pass buckets, memory-sized batches, largest first); smrtcell: configs[4], a mix "
                         "of the three (steps x zmws-per-step ZMWs in total, strong scaling) pulled by the ranks "
                         "from a dynamic queue.  For the queue workloads the timed region includes the read upload")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="ZMWs polished by the CPU baseline (0 = skip; default 256 for 2kb, 0 otherwise)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--streams", type=int, default=0,
                    help="workspace slots = batches polished concurrently (0 = the measured best for the stage, capped by HBM)")
    ap.add_argument("--batch-split", type=int, default=BATCH_SPLIT,
                    help="2 kb: device batches per step (each step's ZMWs polished as this many batches)")
    ap.add_argument("--batch-zmws", type=int, default=0,
                    help="queue workloads: ZMWs per device batch (0 = planned from free HBM)")
    ap.add_argument("--ccs-chunk", type=int, default=0,
                    help="ccs stage: ZMWs per POA chunk / polish batch (0 = planned from free HBM)")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--one-stream", action="store_true",
                    help="A/B: each batch on one HIP stream (the tall fills behind the 16-lane fill), PBCCS_ONE_STREAM")
    ap.add_argument("--stage", choices=["polish", "poa", "ccs", "quiver"], default="polish",
                    help="polish: the headline line (Consensus.h's Arrow polish, from the draft on); poa: the POA "
                         "draft step before it (SparsePoa over each ZMW's raw subreads, SURVEY.md §8(f) row 1) on "
                         "the same configs[1] ZMWs; ccs: both, end to end from raw subreads (FilterReads, POA, "
                         "ExtractMappedRead, polish), the POA of the next steps overlapping the polish; quiver: "
                         "the Quiver family (QV-feature reads, FP32 log-space recursions) through "
                         "pbccs_quiver_polish_batch on configs[1]-shaped ZMWs")
    a = ap.parse_args()
    if a.one_stream:   # read by the engine when it makes a batch (before any HIP call here)
        os.environ["PBCCS_ONE_STREAM"] = "1"
    return a


_JSON_OUT = None   # the process's real stdout while fd 1 is pointed at stderr (multi-rank runs)


def quiet_stdout():
    """Point fd 1 at stderr for the rest of the run: libraries (gloo's connection report) print to stdout, and
    the bench's stdout must be exactly its one JSON line.  emit() writes to the saved stdout."""
    global _JSON_OUT
    sys.stdout.flush()
    _JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


def emit(out):
    f = _JSON_OUT or sys.stdout
    f.write(json.dumps(out) + "\n")
    f.flush()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------------------------------------
# self-launch of N ranks (the parent never initialises HIP)
# ---------------------------------------------------------------------------------------------------------
def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # a rank that fails ends the job: the others would wait on it (the queue's collector, the final barrier), so
    # they are terminated -- the processes this launcher started, by PID
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            rc = rc or c
            if c != 0:
                for q in live:
                    q.terminate()
                for q in live:
                    try:
                        q.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        q.kill()
                        q.wait()
                return c
        time.sleep(0.2)
    return rc


# ---------------------------------------------------------------------------------------------------------
# CPU baseline
# ---------------------------------------------------------------------------------------------------------
def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads(args, n):
    """This process's CPU share: the GPU boxes give one GPU's job 16 cores of a larger machine (OMP_NUM_THREADS),
    so hardware_concurrency() would oversubscribe."""
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    threads = args.cpu_threads or max(1, min(share, os.cpu_count() or 1))
    return max(1, min(threads, n))


def full_host(cb, threads):
    """The node-wide CPU figure beside the measured one: this job's CPU share is `threads` of the host's
    hardware threads (the boxes give one GPU's job 16 cores: OMP_NUM_THREADS / affinity), so the whole host's rate
    is not measured here -- it is the measured rate scaled linearly to every hardware thread (an upper bound: SMT
    siblings share cores), labelled as such in the line."""
    nproc = os.cpu_count() or threads
    cb["full_host_value"] = round(cb["value"] * nproc / threads, 4)
    cb["full_host_method"] = (f"not measured: the {threads}-thread rate scaled linearly to all {nproc} hardware "
                              f"threads (SMT siblings share cores, so an upper bound on the host's rate); "
                              f"the job's affinity allows {len(os.sched_getaffinity(0))} threads")
    return cb


def oracle_record(z, settings):
    """Consensus.h:436-512 for one ZMW on the CPU restatement (oracle/arrow_oracle.cpp), with the gates the batch
    polish applies (capi.hip polish_one): AddRead of every read, MinPasses / MaxDropFraction, ZScores,
    RefineConsensus, ConsensusQVs and the predicted-accuracy gate.  Returns the fields a GPU record carries."""
    from oracle import oracle as O
    rec = {"status": "Other", "consensus": "", "qvs": [], "n_tested": 0, "n_applied": 0, "add_read_results": []}
    reads = z["reads"]
    if not reads:
        rec["status"] = "NoSubreads"
        return rec
    if len(z["draft"]) < settings.min_length:
        rec["status"] = "TooShort"
        return rec
    sc = O.Scorer(z["draft"], z["snr"], score_diff=settings.score_diff)
    st = [sc.add_read(r["seq"], r["strand"], r["ts"], r["te"], settings.min_zscore) for r in reads]
    rec["add_read_results"] = st
    n_passes = sum(1 for r, s in zip(reads, st) if s == 0 and r.get("full_pass", True))
    if n_passes < settings.min_passes:
        rec["status"] = "TooFewPasses"
        return rec
    if sum(1 for s in st if s != 0) / len(reads) > settings.max_drop_fraction:
        rec["status"] = "TooManyUnusable"
        return rec
    sc.zscores()
    ref = sc.refine(settings.max_iterations, settings.mutation_separation, settings.mutation_neighborhood)
    rec["n_tested"], rec["n_applied"] = ref["n_tested"], ref["n_applied"]
    if not ref["converged"]:
        rec["status"] = "Other" if ref["error"] else "NonConvergent"
        return rec
    q = sc.qvs()
    acc = 1.0 - sum(10.0 ** (v / -10.0) for v in q) / max(1, len(q))
    rec.update(consensus=sc.template(), qvs=q,
               status="PoorQuality" if acc < settings.min_predicted_accuracy else "Success")
    return rec


def zmw_cost(z):
    """Cost model of one ZMW's CPU polish: template length x read bases (the scoring rounds dominate: every
    unique mutation of the template against every read's band)."""
    return float(len(z["draft"])) * float(sum(len(r["seq"]) for r in z["reads"] if r["seq"]))


def sampled_cpu_baseline(args, settings, zs, res, idx, costs=None):
    """The CPU baseline and the parity check of the timed run, on the same ZMWs.

    idx: indices into the timed ZMWs `zs` (a list, or synth.SmrtCell) whose GPU records `res` the run produced.
    Each sampled ZMW is polished by the CPU restatement (oracle_record) one ZMW per task on the host threads, as
    `ccs --numThreads` runs the reference (src/main/ccs.cpp:222-230), and its record is compared with the GPU's:
    status, AddRead results, nTested / nApplied, consensus (bit-exact) and QVs (+-1).
    costs: the cost model of every timed ZMW (queue workloads): the CPU rate of the whole workload is then
    extrapolated from the sample by the ratio estimator (CPU seconds per unit of cost on the sample x the
    workload's mean cost), since a small subsample of heterogeneous ZMWs is not their mean.
    Returns (cpu_baseline, parity_sample)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    n = len(idx)
    threads = cpu_threads(args, n)
    O.lib()
    sample = [zs[i] for i in idx]

    def one(z):
        t = time.perf_counter()
        r = oracle_record(z, settings)
        return r, time.perf_counter() - t

    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=threads) as ex:   # ctypes releases the GIL: native threads in parallel
        out = list(ex.map(one, sample))
    dt = time.perf_counter() - t0
    # ---- parity of the timed run's records against the restatement ----
    bad, counts_eq, cons_eq, arr_eq, status_eq, max_qv = [], 0, 0, 0, 0, 0
    for i, (e, _), g in zip(idx, out, [res[i] for i in idx]):
        ok_status = g["status"] == e["status"]
        ok_arr = list(g["add_read_results"]) == list(e["add_read_results"])
        refined = e["status"] in ("Success", "PoorQuality", "NonConvergent")
        ok_counts = (not refined) or (g["n_tested"], g["n_applied"]) == (e["n_tested"], e["n_applied"])
        ok_cons = g["consensus"] == e["consensus"]
        qd = 0
        if e["qvs"] or g["qvs"]:
            qd = max(abs(a - b) for a, b in zip(g["qvs"], e["qvs"])) if len(g["qvs"]) == len(e["qvs"]) else 999
        max_qv = max(max_qv, qd)
        status_eq += ok_status
        arr_eq += ok_arr
        counts_eq += ok_counts
        cons_eq += ok_cons
        if not (ok_status and ok_arr and ok_counts and ok_cons and qd <= 1):
            bad.append(i)
    parity = {"n": n, "status_equal": status_eq, "add_read_equal": arr_eq, "counts_equal": counts_eq,
              "consensus_equal": cons_eq, "max_qv_diff": max_qv, "mismatched_zmws": bad[:16],
              "ok": not bad,
              "checked": "GPU records of the timed run against oracle/arrow_oracle.cpp on the same ZMWs: status, "
                         "AddRead results, nTested/nApplied, consensus bit-exact, QVs within +-1"}
    # ---- CPU rate ----
    secs = [t for _, t in out]
    cb = {"unit": "ZMWs/s", "cores": threads, "kind": "port", "cpu": cpu_model(), "nproc": os.cpu_count(),
          "sample_wall_s": round(dt, 2), "sample_rate": round(n / dt, 4)}
    desc = (f"{n} of the timed ZMWs ({args.workload}; indices {idx[0]}..{idx[-1]}), oracle/arrow_oracle.cpp "
            f"restatement of Consensus.h:436-512 (AddRead, gates, RefineConsensus, ConsensusQVs) one ZMW per task on "
            f"{threads} host threads, {dt:.1f} s wall")
    if costs is None:
        cb["value"] = round(n / dt, 4)
    else:
        c_s = sum(costs[i] for i in idx)
        mean_all = sum(costs) / len(costs)
        ratio_core_s = (sum(secs) / c_s) * mean_all   # ratio estimator x the workload's mean cost (linear in cost)
        # CPU time grows faster than the cost model (the survey: 48x the time for 20x the cost), so the linear ratio
        # estimator, fed by a capped sample, understates the expensive ZMWs.  The stratified sample spans the
        # eligible cost range; a power law t = a c^alpha fitted to it by least squares in log-log predicts every
        # timed ZMW's time (alpha floored at 1: never below the linear estimate)
        fit = power_law_fit([costs[i] for i in idx], secs)
        if fit is not None:
            a, alpha = fit
            alpha_used = max(1.0, alpha)
            a_used = a if alpha >= 1.0 else math.log(sum(secs) / sum(costs[i] ** alpha_used for i in idx))
            core_s_per_zmw = sum(math.exp(a_used) * c ** alpha_used for c in costs) / len(costs)
        else:
            alpha = alpha_used = None
            core_s_per_zmw = ratio_core_s
        cb["value"] = round(threads / core_s_per_zmw, 4)
        cb["extrapolated"] = {"core_s_per_zmw": round(core_s_per_zmw, 3), "sample_core_s": round(sum(secs), 2),
                              "cost_sample_mean": c_s / n, "cost_workload_mean": mean_all,
                              "alpha_fitted": None if alpha is None else round(alpha, 3),
                              "alpha_used": None if alpha_used is None else round(alpha_used, 3),
                              "ratio_estimator_core_s_per_zmw": round(ratio_core_s, 3),
                              "ratio_estimator_value": round(threads / ratio_core_s, 4),
                              "method": "sample stratified by cost (template length x read bases) over the eligible "
                                        "range; power law t = a cost^alpha fitted in log-log on the sample (alpha >= "
                                        "1), summed over every timed ZMW's cost, on `cores` threads; the linear "
                                        "ratio estimator beside it"}
        desc += "; the workload's rate extrapolated from it (BASELINE.md CPU-baseline plan)"
    cb["sample"] = desc
    # the host's whole thread count, if the pool scaled linearly to it (an upper bound: SMT threads share cores)
    full_host(cb, threads)
    return cb, parity


def power_law_fit(costs, secs):
    """Least squares of log t = a + alpha log c over the sample (ZMWs with positive cost and time); None when the
    sample cannot determine a slope."""
    pts = [(math.log(c), math.log(t)) for c, t in zip(costs, secs) if c > 0 and t > 0]
    if len(pts) < 3:
        return None
    mx = sum(x for x, _ in pts) / len(pts)
    my = sum(y for _, y in pts) / len(pts)
    sxx = sum((x - mx) ** 2 for x, _ in pts)
    if sxx <= 1e-12:
        return None
    alpha = sum((x - mx) * (y - my) for x, y in pts) / sxx
    return my - alpha * mx, alpha


SAMPLE_COST_CAP = 8.5e8   # zmw_cost of a 10 kb / 8-pass ZMW: the largest ZMW a bounded CPU sample polishes


def sample_indices(args, n_timed, costs=None):
    """Which timed ZMWs the CPU leg polishes: every (N/n)-th ZMW of a homogeneous workload; for a heterogeneous
    one a seeded simple random sample of the ZMWs no costlier than a 10 kb / 8-pass ZMW (a 20 kb / 30-pass ZMW
    alone takes ~15 core-minutes on the restatement), the rest reached by the ratio estimator."""
    import random
    n = max(1, min(args.cpu_sample, n_timed))
    if costs is None:
        step = max(1, n_timed // n)
        return list(range(0, n_timed, step))[:n]
    elig = sorted((i for i in range(n_timed) if 0 < costs[i] <= SAMPLE_COST_CAP), key=lambda i: (costs[i], i))
    rng = random.Random(args.seed + 99991)
    if len(elig) <= n:
        return sorted(elig)
    # stratified: the eligible ZMWs in cost order cut into n strata of equal count, one seeded draw
    # from each -- the sample spans the eligible cost range instead of clustering where the cheap ZMWs are
    out = []
    for k in range(n):
        lo, hi = len(elig) * k // n, len(elig) * (k + 1) // n
        out.append(elig[rng.randrange(lo, hi)])
    return sorted(out)


def coverage(costs, idx_pool_cap=SAMPLE_COST_CAP):
    elig = [c for c in costs if c <= idx_pool_cap]
    return {"eligible_zmws_frac": round(len(elig) / max(1, len(costs)), 4),
            "eligible_cost_frac": round(sum(elig) / max(1.0, sum(costs)), 4),
            "cap": f"ZMWs with template length x read bases <= {idx_pool_cap:.3g} (a 10 kb / 8-pass ZMW)"}


class HostUsage:
    """The rank's host cost over a timed region: CPU seconds of all its threads (getrusage RUSAGE_SELF: the
    engine's slot threads, the POA workers and Python) and the process's peak RSS."""

    def __init__(self):
        import resource
        self._r = resource
        u = resource.getrusage(resource.RUSAGE_SELF)
        self.t0 = u.ru_utime + u.ru_stime

    def report(self, zmws_local, world):
        u = self._r.getrusage(self._r.RUSAGE_SELF)
        cpu = u.ru_utime + u.ru_stime - self.t0
        rss = u.ru_maxrss / 2**20   # KiB -> GiB
        out = {"cpu_s": round(cpu, 3), "cpu_ms_per_zmw": round(1e3 * cpu / max(1, zmws_local), 4),
               "rss_gb": round(rss, 3)}
        if world > 1:
            out["cpu_s_max_rank"] = round(max_over_ranks(cpu, world), 3)
            out["rss_gb_max_rank"] = round(max_over_ranks(rss, world), 3)
        out["note"] = ("rank 0's host CPU seconds (user + system, every thread) over the timed region, per ZMW it "
                       "polished, and its peak resident set")
        return out


def cpu_share_note():
    return ("vs_cpu: against the CPU restatement on this job's CPU share (`cpu_baseline.cores` threads); "
            "vs_cpu_full_host: against that rate scaled linearly to all `nproc` hardware threads of the node")


KERNEL_SOURCES = ("arrow_device.hpp", "arrow_kernels.hip", "arrow_kernels.hpp", "coop_chain.hpp", "fill_coop.hip")


def kernel_source_digest():
    """sha256 (16 hex) of the Arrow path's device code (KERNEL_SOURCES): a committed PMC profile (traffic, VALU per
    launch) or single-slot / occupancy run is valid for the kernels it was taken on, and stale once any of them
    changes.  Host-side engine edits (engine.hip, capi.hip) do not change a launch's instructions or bytes."""
    import hashlib
    d = os.path.join(ROOT, "pbccs_amd", "csrc")
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        h.update(f.encode())
        h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()[:16]


def workload_kw(args):
    """synth.make_zmws keywords of the workload."""
    if args.workload == "10kb":
        return dict(length=10000, passes=8)
    if args.workload == "mixed":
        return dict(length=None, passes=None, length_range=(500, 20000), passes_range=(3, 30), random_snr=True)
    return dict(length=args.length, passes=args.passes)


# ---------------------------------------------------------------------------------------------------------
# queue workloads (configs[2], [3], [4])
# ---------------------------------------------------------------------------------------------------------
def heartbeat(rank, t0):
    import threading
    done = threading.Event()

    def beat():
        while not done.wait(30.0):
            log(rank, f"[bench] work queue running t={time.perf_counter() - t0:.0f}s")
    threading.Thread(target=beat, daemon=True).start()
    return done


def queue_workload(args, rank, world, eng, settings, seed0):
    """configs[2] / [3] through the work queue, configs[4] through the ranks' dynamic queue; returns
    (job_time, local_time, results, workload, scaling)."""
    import pbccs_amd
    import torch
    import torch.distributed as dist
    from pbccs_amd import shard, synth
    n = args.steps * args.zmws_per_step
    if args.workload == "smrtcell":
        desc = (f"configs[4]: SMRT-cell mix of configs[1]-[3] (2 kb x 10, 10 kb x 8, 0.5-20 kb x 3-30 passes; "
                f"one third each), {n} ZMWs in total over {world} GPU(s), dynamic pull queue; each rank generates "
                f"only the chunks it pulls (synth.SmrtCell), inside the timed region")
        kw = None
    else:
        kw = workload_kw(args)
        desc = (f"configs[2]: synthetic 10000 bp insert, 8 full passes, {n} ZMWs per GPU" if args.workload == "10kb"
                else f"configs[3]: synthetic 0.5-20 kb inserts, 3-30 passes, per-ZMW SNR U[4,20], {n} ZMWs per GPU")
    for w in range(args.warmup):
        wz = synth.SmrtCell(4, seed=seed0 + 1000 + w)[:] if kw is None else \
            synth.make_zmws(4, seed=seed0 + 1000 + w, **kw)
        pbccs_amd.polish_stream(wz, settings, eng)
    log(rank, "[bench] warmup done")
    if kw is None:
        # the same cell on every rank, generated lazily: a rank materialises only the chunks it pulls.  The
        # shapes (length, passes) are drawn before the timed region, as ccs would know them from the .pbi index
        zs = synth.SmrtCell(n, seed=args.seed + 3)
        zs.shapes()
    else:
        zs = synth.make_zmws(n, seed=seed0, **kw)
    eng.kernel_stats(reset=True)
    eng.counters(reset=True)
    if world > 1:
        dist.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    host = HostUsage()
    t0 = time.perf_counter()
    done = heartbeat(rank, t0)
    qstats = {}
    try:
        if kw is None:
            # chunks of at most 512 ZMWs, at least four per rank: the cost-ordered pull queue balances the ranks only
            # when the last chunks are small (four 1500-ZMW chunks left a 156 s tail on two ranks), and a chunk must
            # still hold enough ZMWs of each shape to fill the rank's workspace slots
            res = shard.polish_dynamic(zs, settings, eng, rank, world,
                                       chunk=max(1, min(512, n // (4 * world))), stats=qstats)
        else:
            res = pbccs_amd.polish_stream(zs, settings, eng)
    finally:
        done.set()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    local_time = time.perf_counter() - t0
    job_time = max_over_ranks(local_time, world)
    local_n = qstats.pop("zmws_local", n) if kw is None else n
    hostu = host.report(local_n, world)
    if kw is None:   # host memory high-water of the ranks (the cell is generated per chunk; rank 0 holds the records)
        qstats["host_rss_gb_rank0"] = hostu["rss_gb"]
        qstats["host_rss_gb_max"] = hostu.get("rss_gb_max_rank", hostu["rss_gb"])
        qstats["gen_ms_max"] = round(max_over_ranks(qstats.get("gen_ms", 0.0), world), 1)
    costs = zs.costs() if kw is None else [zmw_cost(z) for z in zs]
    extra = {"host": hostu, "zs": zs, "costs": costs}
    if kw is None:   # rank 0 holds the whole cell's records; the count is the cell
        return job_time, local_time, (res or []), desc, "strong", n, qstats, extra
    return job_time, local_time, res, desc + " (work queue; timed region includes the read upload)", "weak", \
        n * world, None, extra


def max_over_ranks(t, world):
    if world == 1:
        return t
    import torch
    import torch.distributed as dist
    v = torch.tensor([t], dtype=torch.float64)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    return float(v.item())


# ---------------------------------------------------------------------------------------------------------
def choose_slots(args, local):
    """Workspace slots: the measured best split, capped by the steps and by the HBM the slots' band pools
    need at their high-water mark (a 2 kb / 10-pass batch of 2000 ZMWs peaks near 27 GB)."""
    import torch
    queue = args.workload in ("10kb", "mixed", "smrtcell") and args.stage == "polish"
    if args.stage == "ccs":   # pbccs_ccs_batch plans its own chunks: the step count does not bound the slots
        best, batches = BEST_SLOTS_CCS, BEST_SLOTS_CCS
        batch_zmws = args.ccs_chunk or max(1, args.zmws_per_step // 2)
    else:
        best, batches, batch_zmws = BEST_SLOTS, args.steps * args.batch_split, max(1, args.zmws_per_step // args.batch_split)
    if queue:
        best = BEST_SLOTS_LONG
    # (the work queue splits its ZMWs into memory-sized batches whatever the step count: slots = concurrent batches)
    want = args.streams or (best if queue else max(1, min(batches, best)))
    if queue or not torch.cuda.is_available():   # the queue plans its own batches from free HBM and the slots
        return want
    free_b, _ = torch.cuda.mem_get_info(local)
    per_slot = batch_zmws * SLOT_BYTES_PER_ZMW
    fit = max(1, int((free_b - HBM_MARGIN) // per_slot))
    return max(1, min(want, fit))


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    if args.cpu_sample is None:   # ~10-60 s of the restatement on the box's 16 threads
        args.cpu_sample = {"2kb": 256, "10kb": 16, "mixed": 32, "smrtcell": 32}[args.workload]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # PBCCS_BENCH_DEVICE pins every rank to one device: a rehearsal of the multi-rank launch, gather and
    # max-over-ranks timing on a one-GPU box (ranks then share the device; give them few --streams)
    if os.environ.get("PBCCS_BENCH_DEVICE"):
        local = int(os.environ["PBCCS_BENCH_DEVICE"])
    if world != args.gpus:
        log(rank, f"[bench] note: --gpus {args.gpus} but the launcher started {world} rank(s); using {world}")
    # torch first: the engine then binds to the same HIP runtime instance (both carry soname libamdhip64.so.7)
    import torch
    import torch.distributed as dist
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    if world > 1:
        quiet_stdout()
        dist.init_process_group(backend="gloo")   # barrier + max-time + the queue's counter: no device collective

    import pbccs_amd
    from pbccs_amd import synth

    def barrier():
        if world > 1:
            dist.barrier()

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    eng = pbccs_amd.Engine(local)
    slots = choose_slots(args, local)
    eng.set_concurrency(slots)
    if not args.no_profile:
        eng.set_profiling(True)   # HIP events on the launch streams + in-kernel algorithmic counters
    settings = pbccs_amd.ConsensusSettings()
    if args.batch_zmws and args.workload != "2kb":
        settings.zmws_per_batch = args.batch_zmws
    seed0 = args.seed + 7919 * rank

    if args.stage == "poa":
        return poa_stage(args, rank, world, eng, barrier, sync, seed0)
    if args.stage == "ccs":
        return ccs_stage(args, rank, world, eng, slots, settings, barrier, sync, seed0)
    if args.stage == "quiver":
        return quiver_stage(args, rank, world, eng, barrier, sync, seed0)
    if args.workload != "2kb":
        job_time, local_time, res, workload, scaling, total, qstats, extra = queue_workload(args, rank, world, eng,
                                                                                            settings, seed0)
        return report(args, rank, world, eng, slots, job_time, local_time, res, workload, scaling, total, qstats,
                      extra=extra, settings=settings)

    # the K steps as device batches of zmws_per_step / BATCH_SPLIT ZMWs, each made (pbccs_batch_create's per-ZMW
    # setup and upload) and polished by a slot thread of the engine's queue (pbccs_polish_batch): batch creation
    # is inside the timed region, pipelined with the other slots' polishes (made ahead it was
    # 9% of the timed region, profiles/r5a_bench.json `prepare`)
    import ctypes
    from pbccs_amd import lib as L
    from pbccs_amd.polish import _Marshalled
    qset = pbccs_amd.ConsensusSettings(zmws_per_batch=-(-args.zmws_per_step // max(1, args.batch_split)))

    def polish_queue(m):
        opts = qset._c()
        L.check(L.load().pbccs_polish_batch(eng._h, m._ins, len(m.zmws), ctypes.byref(opts), m._outs))

    # ---- warmup (untimed): W steps, concurrently over the slots like the timed ones ------------------
    wz = [z for w in range(args.warmup)
          for z in synth.make_zmws(args.zmws_per_step, args.length, args.passes, seed=seed0 + 1000 + w)]
    if wz:
        polish_queue(_Marshalled(wz))
    log(rank, f"[bench] warmup done ({args.warmup} x {args.zmws_per_step} ZMWs over {slots} slots)")

    # ---- engine pools mapped before the timed region (a long run maps them once and reuses them) ----
    if torch.cuda.is_available():
        free_b, _ = torch.cuda.mem_get_info(local)
        per_slot = int(min(0.6 * free_b / slots, 30 << 30))
        eng.reserve_pool(per_slot)
        log(rank, f"[bench] band pools: {per_slot / 2**30:.1f} GB mapped per slot x {slots}")

    # ---- inputs before the timed region: the synthetic generation (Python strings: the stand-in for reading the
    # subreads) and their marshalling into the C structs of the boundary (the stand-in for the reader's records)
    t_prep = time.perf_counter()
    zs_all = []
    for k in range(args.steps):
        zs_all.extend(synth.make_zmws(args.zmws_per_step, args.length, args.passes, seed=seed0 + k))
    synth_s = time.perf_counter() - t_prep
    tm = time.perf_counter()
    marshalled = _Marshalled(zs_all)
    prep = {"synth_s": round(synth_s, 3), "marshal_s": round(time.perf_counter() - tm, 3)}
    log(rank, f"[bench] prepared {args.steps} steps x {args.zmws_per_step} ZMWs in {time.perf_counter() - t_prep:.1f}s "
              f"{prep}")
    eng.counters(reset=True)
    eng.kernel_stats(reset=True)

    # ---- timed region: exactly K steps --------------------------------------------------------
    barrier()
    sync()
    host = HostUsage()
    t0 = time.perf_counter()
    polish_queue(marshalled)   # the K steps: batches made and polished by the slots' host threads / HIP streams
    sync()
    barrier()
    local_time = time.perf_counter() - t0
    log(rank, f"[bench] {args.steps} steps done t={local_time:.2f}s")
    job_time = max_over_ranks(local_time, world)

    res = marshalled.results()
    hostu = host.report(len(res), world)
    c0 = eng.counters()
    prep["create_thread_s_in_timed"] = round((c0["create_host_ns"] + c0["create_upload_ns"]) / 1e9, 3)
    prep["create_host_s"] = round(c0["create_host_ns"] / 1e9, 3)
    prep["create_upload_s"] = round(c0["create_upload_ns"] / 1e9, 3)
    prep["note"] = ("outside the timed region: synth_s the synthetic subreads, marshal_s the boundary's C structs "
                    "(the reader's part).  Inside it, on the slot threads: pbccs_batch_create per device batch "
                    "(create_host_s the batch's copy of its inputs and the read pool, create_upload_s the "
                    "reservations and the read upload) and the per-ZMW setup of Consensus.h:437-453 (transition "
                    "tables, expectations, reverse-complement template, descriptor arena: derive_thread_s_in_timed)")
    workload = (f"configs[1]: synthetic {args.length} bp insert, {args.passes} full passes, "
                f"{args.zmws_per_step} ZMWs per step")
    report(args, rank, world, eng, slots, job_time, local_time, res, workload, "weak", len(res) * world,
           extra={"host": hostu, "zs": zs_all, "costs": None, "prepare": prep}, settings=settings)


def poa_cpu_baseline(args, steps_in, res, n):
    """The POA restatement (oracle/poa_oracle.cpp, SparsePoa as Consensus.h drives it) one ZMW per task on the
    host threads, like the polish baseline, on every (N/n)-th ZMW of the timed steps; each draft, read key and
    extent is checked against the GPU's record of the timed run (bit-exact)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    flat_in = [z for step in steps_in for z in step]
    flat_res = [r for step in res for r in step]
    args_n = argparse.Namespace(**vars(args))
    args_n.cpu_sample = n
    idx = sample_indices(args_n, len(flat_in))
    threads = cpu_threads(args, len(idx))
    O.lib()
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=threads) as ex:
        exp = list(ex.map(O.sparse_poa, [flat_in[i] for i in idx]))
    dt = time.perf_counter() - t0
    bad = []
    for i, e in zip(idx, exp):
        g = flat_res[i]
        if (g["consensus"], list(g["keys"]), g["summaries"]) != (e["consensus"], e["keys"], e["summaries"]):
            bad.append(i)
    n = len(idx)
    cb = {"value": round(n / dt, 4), "unit": "ZMWs/s", "cores": threads, "kind": "port", "cpu": cpu_model(),
          "nproc": os.cpu_count(),
          "sample": f"{n} of the timed ZMWs (every {max(1, len(flat_in) // n)}-th), oracle/poa_oracle.cpp SparsePoa "
                    f"(OrientAndAddRead per subread, FindConsensus) one ZMW per task on {threads} host threads, "
                    f"{dt:.1f} s wall"}
    full_host(cb, threads)
    parity = {"n": n, "draft_equal": n - len(bad), "mismatched_zmws": bad[:16], "ok": not bad,
              "checked": "GPU drafts, read keys and PoaAlignmentSummary extents of the timed run against "
                         "oracle/poa_oracle.cpp on the same subreads, bit-exact"}
    return cb, parity


def poa_stage(args, rank, world, eng, barrier, sync, seed0):
    """The POA draft step of configs[1]: a step hands one batch of ZMWs' raw subreads (alternate passes
    reverse-complemented, as sequenced) to pbccs_poa_batch, which adds every ZMW's next read in the same
    device round (k_poa_fill over all (ZMW, orientation) alignments, k_poa_trace over the committed ones,
    host threading of the graphs) and ends with FindConsensus + the per-read extents.  The graphs are host
    state, so the timed region includes the host threading and the per-round uploads of the column
    programs; the subreads themselves start in host memory, as the reference's do."""
    from pbccs_amd import poa, synth

    def subreads(n, seed):
        return [[r["seq"] for r in z["reads"]] for z in synth.make_zmws(n, args.length, args.passes, seed=seed)]

    for w in range(args.warmup):   # full-size steps: the score pool and staging buffers reach their high-water
        poa.poa_batch(subreads(args.zmws_per_step, seed0 + 1000 + w), engine=eng)
    steps_in = [subreads(args.zmws_per_step, seed0 + k) for k in range(args.steps)]
    poa.poa_stats(eng, reset=True)
    barrier()
    sync()
    host = HostUsage()
    t0 = time.perf_counter()
    res = [poa.poa_batch(x, engine=eng) for x in steps_in]
    sync()
    barrier()
    local_time = time.perf_counter() - t0
    job_time = max_over_ranks(local_time, world)
    hostu = host.report(args.steps * args.zmws_per_step, world)
    st = poa.poa_stats(eng, reset=True)
    total = args.steps * args.zmws_per_step * world
    launches = max(1, st["launches"])
    avg_ms = st["fill_ms"] / launches
    bpl = st["bytes"] / launches
    achieved = bpl / (avg_ms / 1e3) / 1e9 if avg_ms > 0 else 0.0
    out = {
        "metric": "POA draft ZMWs/sec (SparsePoa over raw subreads) on MI355X vs host-CPU",
        "value": round(total / job_time, 3), "unit": "ZMWs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(job_time / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int32/uint16",
        "data": "synthetic subreads (SURVEY.md §8(d): truth iid ACGT; 7%/4%/1% ins/del/sub; odd passes RC)",
        "config": {"workload": f"configs[1] POA: {args.length} bp insert, {args.passes} subreads per ZMW, "
                               f"{args.zmws_per_step} ZMWs per step", "zmws_per_step": args.zmws_per_step,
                   "zmws_total": total, "parallelism": f"zmw-shard x{world}"},
        "gcups": round(st["cells"] / local_time / 1e9, 3),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": None, "kernel": "k_poa_fill",
                     "avg_launch_ms": round(avg_ms, 4), "launches": st["launches"], "bytes_per_launch": bpl,
                     "cells_per_launch": st["cells"] / launches},
        "poa": {"alignments": st["alignments"], "gcells": round(st["cells"] / 1e9, 3),
                "fill_ms": round(st["fill_ms"], 2), "trace_ms": round(st["trace_ms"], 2),
                "trace_steps": st["trace_steps"],
                "host_ms": {k: round(st[k], 1) for k in ("prog_ms", "device_ms", "thread_ms", "consensus_ms",
                                                             "total_ms")},
                "draft_len_mean": round(sum(len(r["consensus"]) for b in res for r in b) / max(1, total // world), 1)},
    }
    out["host"] = hostu
    parity_ok = True
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        cb, parity = poa_cpu_baseline(args, steps_in, res, min(args.cpu_sample, 48))
        out["cpu_baseline"], out["parity_sample"] = cb, parity
        out["vs_cpu"] = round(out["value"] / cb["value"], 2)
        out["vs_cpu_full_host"] = round(out["value"] / cb["full_host_value"], 3)
        out["vs_cpu_note"] = cpu_share_note()
        parity_ok = parity["ok"]
    if rank == 0:
        emit(out)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    if not parity_ok:
        log(rank, f"[bench] PARITY FAILURE on the timed POA run's sample: {out['parity_sample']}")
        sys.exit(3)


def quiver_cpu_baseline(args, zs, res):
    """The Quiver CPU restatement (oracle/quiver_oracle.cpp: the SSE recursor's single-precision operations
    in order) on host threads, one ZMW per task -- AddRead, RefineConsensus, ConsensusQVs -- on every (N/n)-th of
    the timed scorers, whose GPU records it checks: converged, nTested / nApplied, consensus and QVs, all exact."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    from pbccs_amd import synth
    idx = sample_indices(args, len(zs))
    n = len(idx)
    threads = cpu_threads(args, n)
    O.lib()

    def one(z):
        o = O.QuiverScorer(z["tpl"], synth.QUIVER_PARAMS, score_diff=synth.QUIVER_SCORE_DIFF)
        for r in z["reads"]:
            o.add_read(r["seq"], r["strand"], r["ts"], r["te"], r["features"])
        ref = o.refine()
        return {"converged": ref["converged"], "n_tested": ref["n_tested"], "n_applied": ref["n_applied"],
                "consensus": o.template(), "qvs": o.qvs()}

    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=threads) as ex:
        exp = list(ex.map(one, [zs[i] for i in idx]))
    dt = time.perf_counter() - t0
    bad, cons_eq, counts_eq, qv_eq = [], 0, 0, 0
    for i, e in zip(idx, exp):
        g = res[i]
        ok_c = g["consensus"] == e["consensus"]
        ok_n = (bool(g["converged"]), g["n_tested"], g["n_applied"]) == (e["converged"], e["n_tested"], e["n_applied"])
        ok_q = list(g["qvs"] or []) == list(e["qvs"])
        cons_eq += ok_c
        counts_eq += ok_n
        qv_eq += ok_q
        if not (ok_c and ok_n and ok_q):
            bad.append(i)
    cb = {"value": round(n / dt, 4), "unit": "ZMWs/s", "cores": threads, "kind": "port", "cpu": cpu_model(),
          "nproc": os.cpu_count(),
          "sample": f"{n} of the timed Quiver ZMWs (every {max(1, len(zs) // n)}-th), oracle/quiver_oracle.cpp AddRead + "
                    f"RefineConsensus + ConsensusQVs one ZMW per task on {threads} host threads, {dt:.1f} s wall"}
    full_host(cb, threads)
    parity = {"n": n, "consensus_equal": cons_eq, "counts_equal": counts_eq, "qvs_equal": qv_eq,
              "mismatched_zmws": bad[:16], "ok": not bad,
              "checked": "GPU records of the timed run against oracle/quiver_oracle.cpp on the same scorers: "
                         "converged, nTested/nApplied, consensus and QVs exact"}
    return cb, parity


def quiver_roofline(stats, local_time):
    """The Quiver stage's dominant kernel (by device time) priced against HBM: the fills store every pass's FP32
    band (4 B per cell) and column metadata (12 B per column), counted in-kernel over the completed fills."""
    fills = {k: v for k, v in stats.items() if k.startswith("k_qfill") and v["launches"]}
    if not fills:
        return None
    dom_name, dom = max(stats.items(), key=lambda kv: kv[1]["device_ms"])
    fk, fv = max(fills.items(), key=lambda kv: kv[1]["device_ms"])
    launches = max(1, fv["launches"])
    avg_ms = fv["device_ms"] / launches
    bpl = fv["bytes"] / launches
    achieved = bpl / (avg_ms / 1e3) / 1e9 if avg_ms > 0 else 0.0
    in_flight = fv["device_ms"] / (local_time * 1e3) if local_time > 0 else None
    return {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": None, "kernel": fk,
            "dominant_kernel": dom_name, "avg_launch_ms": round(avg_ms, 4), "launches": fv["launches"],
            "bytes_per_launch": bpl, "cells_per_launch": fv["cells"] / launches,
            "in_flight": round(in_flight, 3) if in_flight is not None else None,
            "wall": {"achieved": round(fv["bytes"] / local_time / 1e9, 3),
                     "frac": round(fv["bytes"] / local_time / 1e9 / HBM_PEAK_GBS, 6), "unit": "GB/s"},
            "per_launch_note": "achieved/frac: algorithmic bytes per launch (4 B per stored FP32 band cell + 12 B per "
                               "column per pass, counted in-kernel) / HIP-event launch time on the kernel's stream",
            "binding": "latency: a band column is a chain of dependent LDS round trips (Inc/Merge/Del, then the "
                       "serial Extra cascade and the block band-end test); ~10 rows per column use 16 lanes of "
                       "four reads per wavefront (DESIGN.md §3.8); neither HBM nor FP32 VALU"}


def quiver_stage(args, rank, world, eng, barrier, sync, seed0):
    """The Quiver family on configs[1]-shaped ZMWs with QV features: per ZMW a
    scorer over the default QuiverConfig, AddRead of every read, RefineConsensus and ConsensusQVs, all
    steps x zmws-per-step scorers in one pbccs_quiver_polish_batch.  value = ZMWs/s; the inputs are marshalled
    (PreparedQuiverBatch, host structures over the reads' arrays) before the timed region, which starts from host
    memory: the reads' upload to the device is inside it."""
    import pbccs_amd as P
    from pbccs_amd import quiver, synth
    cfg = P.QuiverConfig(P.QvModelParams(**synth.QUIVER_PARAMS), score_diff=synth.QUIVER_SCORE_DIFF)
    warm_ms = []   # the first call's extra cost (buffer growth) against the next ones
    for w in range(args.warmup):   # full-size: the engine's device buffers reach their steady-state size untimed
        wz = synth.make_quiver_zmws(args.steps * args.zmws_per_step, args.length, args.passes, seed=seed0 + 1000 + w)
        sync()
        tw = time.perf_counter()
        quiver.polish_batch(wz, cfg, engine=eng)
        sync()
        warm_ms.append(round((time.perf_counter() - tw) * 1e3, 1))
    zs = synth.make_quiver_zmws(args.steps * args.zmws_per_step, args.length, args.passes, seed=seed0)
    prep = quiver.PreparedQuiverBatch(zs, cfg)   # host marshalling before the timed region (as PreparedBatch)
    eng.kernel_stats(reset=True)
    barrier()
    sync()
    host = HostUsage()
    t0 = time.perf_counter()
    res = prep.run(engine=eng)
    sync()
    barrier()
    local_time = time.perf_counter() - t0
    job_time = max_over_ranks(local_time, world)
    hostu = host.report(len(zs), world)
    stats = eng.kernel_stats(reset=True)
    total = len(zs) * world
    out = {"metric": "Quiver ZMWs/sec (AddRead, RefineConsensus, ConsensusQVs per scorer) on MI355X",
           "value": round(total / job_time, 3), "unit": "ZMWs/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(job_time / args.steps * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f32 (log space)",
           "data": "synthetic QV-feature reads (synth.make_quiver_zmws)",
           "config": {"workload": f"configs[1]-shaped Quiver: {args.length} bp draft, {args.passes} reads per ZMW "
                                  f"(ins/del/sub {synth.QUIVER_READ_ERRORS}), ScoreDiff {synth.QUIVER_SCORE_DIFF}, "
                                  f"{len(zs)} scorers in one pbccs_quiver_polish_batch",
                      "parallelism": f"zmw-shard x{world}"},
           "converged": sum(r["converged"] for r in res), "mean_iterations_applied":
               round(sum(r["n_applied"] for r in res) / max(1, len(res)), 2), "warmup_call_ms": warm_ms,
           "timed_call_ms": round(local_time * 1e3, 1),
           "gcups": round(sum(v["cells"] for k, v in stats.items() if k.startswith("k_qfill")) / local_time / 1e9, 3),
           "roofline": quiver_roofline(stats, local_time),
           "kernels": {k: {"launches": v["launches"], "device_ms": round(v["device_ms"], 3),
                           "gcells": round(v["cells"] / 1e9, 4), "gbytes": round(v["bytes"] / 1e9, 4)}
                       for k, v in stats.items() if v["launches"]},
           "host": hostu}
    parity_ok = True
    if rank == 0 and args.cpu_sample:
        cb, parity = quiver_cpu_baseline(args, zs, res)
        out["cpu_baseline"], out["parity_sample"] = cb, parity
        out["vs_cpu"] = round(out["value"] / cb["value"], 2)
        out["vs_cpu_full_host"] = round(out["value"] / cb["full_host_value"], 3)
        out["vs_cpu_note"] = cpu_share_note()
        parity_ok = parity["ok"]
    if rank == 0:
        emit(out)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    if not parity_ok:
        log(rank, f"[bench] PARITY FAILURE on the timed Quiver run's sample: {out['parity_sample']}")
        sys.exit(3)


def ccs_cpu_baseline(args, settings, work, res, n):
    """Consensus.h's per-ZMW path on the host (include/pacbio/ccs/Consensus.h:395-552): FilterReads and
    ExtractMappedRead (pbccs_amd.driver, host code), the SparsePoa restatement (oracle/poa_oracle.cpp) and the
    polish restatement (oracle/arrow_oracle.cpp: AddRead, the gates, RefineConsensus, ConsensusQVs), one ZMW per
    task on the host threads like `ccs --numThreads` (src/main/ccs.cpp:222-230), on every (N/n)-th ZMW of the timed
    run; each record (status, consensus, nTested / nApplied, QVs +-1) is checked against the GPU's."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    from pbccs_amd import driver
    args_n = argparse.Namespace(**vars(args))
    args_n.cpu_sample = n
    idx = sample_indices(args_n, len(work))
    threads = cpu_threads(args, len(idx))
    O.lib()

    def one(c):
        rec = {"status": "Other", "consensus": "", "qvs": [], "n_tested": 0, "n_applied": 0}
        reads = driver.filter_reads(c["reads"], settings.min_length)
        if not reads or all(r is None for r in reads):
            rec["status"] = "NoSubreads"
            return rec
        p = O.sparse_poa([None if r is None else r["seq"] for r in reads])
        if len(p["consensus"]) < settings.min_length:
            rec["status"] = "TooShort"
            return rec
        mapped = [driver.extract_mapped_read(reads[i], p["summaries"][k], settings.min_length)
                  for i, k in enumerate(p["keys"]) if k >= 0]
        # Consensus.h:474-491's gates, as pbccs_ccs_batch applies them: reads FilterReads, the POA or
        # ExtractMappedRead dropped count in the drop fraction's denominator only
        sc = O.Scorer(p["consensus"], c["snr"], score_diff=settings.score_diff)
        st = [sc.add_read(m["seq"], m["strand"], m["ts"], m["te"], settings.min_zscore) for m in mapped if m is not None]
        ok = sum(1 for x in st if x == 0)
        if ok < settings.min_passes:
            rec["status"] = "TooFewPasses"
            return rec
        if (len(st) - ok) / len(c["reads"]) > settings.max_drop_fraction:
            rec["status"] = "TooManyUnusable"
            return rec
        sc.zscores()
        ref = sc.refine(settings.max_iterations, settings.mutation_separation, settings.mutation_neighborhood)
        rec["n_tested"], rec["n_applied"] = ref["n_tested"], ref["n_applied"]
        if not ref["converged"]:
            rec["status"] = "NonConvergent"
            return rec
        q = sc.qvs()
        acc = 1.0 - sum(10.0 ** (v / -10.0) for v in q) / max(1, len(q))
        rec.update(consensus=sc.template(), qvs=q,
                   status="PoorQuality" if acc < settings.min_predicted_accuracy else "Success")
        return rec

    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=threads) as ex:
        exp = list(ex.map(one, [work[i] for i in idx]))
    dt = time.perf_counter() - t0
    bad, max_qv = [], 0
    for i, e in zip(idx, exp):
        g = res[i]
        qd = 0
        if e["qvs"] or g["qvs"]:
            qd = max(abs(a - b) for a, b in zip(g["qvs"], e["qvs"])) if len(g["qvs"]) == len(e["qvs"]) else 999
        max_qv = max(max_qv, qd)
        refined = e["status"] in ("Success", "PoorQuality", "NonConvergent")
        if g["status"] != e["status"] or g["consensus"] != e["consensus"] or qd > 1 or \
                (refined and (g["n_tested"], g["n_applied"]) != (e["n_tested"], e["n_applied"])):
            bad.append(i)
    n = len(idx)
    statuses = [e["status"] for e in exp]
    cb = {"value": round(n / dt, 4), "unit": "ZMWs/s", "cores": threads, "kind": "port", "cpu": cpu_model(),
          "nproc": os.cpu_count(), "zmw_status": {k: statuses.count(k) for k in sorted(set(statuses))},
          "sample": f"{n} of the timed ZMWs (every {max(1, len(work) // n)}-th): FilterReads, oracle/poa_oracle.cpp "
                    f"SparsePoa, ExtractMappedRead, oracle/arrow_oracle.cpp AddRead, the TooFewPasses / "
                    f"TooManyUnusable gates, RefineConsensus and ConsensusQVs of converged ZMWs, one ZMW per task on "
                    f"{threads} host threads, {dt:.1f} s wall"}
    full_host(cb, threads)
    parity = {"n": n, "record_equal": n - len(bad), "max_qv_diff": max_qv, "mismatched_zmws": bad[:16],
              "ok": not bad,
              "checked": "GPU records of the timed run against the CPU pipeline on the same subreads: status, "
                         "consensus bit-exact, nTested/nApplied, QVs within +-1"}
    return cb, parity


def ccs_stage(args, rank, world, eng, slots, settings, barrier, sync, seed0):
    """configs[1] end to end from raw subreads in one native call (pbccs_ccs_batch): Consensus.h's
    FilterReads, the POA draft on the GPU, TooShort, ExtractMappedRead and the polish through the ZMW work
    queue, for steps x zmws-per-step ZMWs.  value = ZMWs/s from raw subreads (host memory) to polished
    consensus; the ZMWs that end before the polish count in the status table."""
    import pbccs_amd
    from pbccs_amd import driver, synth

    def chunks(n, seed):
        return [{"snr": z["snr"], "reads": [{"seq": r["seq"]} for r in z["reads"]]}
                for z in synth.make_zmws(n, args.length, args.passes, seed=seed)]

    settings.zmws_per_batch = args.ccs_chunk
    for w in range(args.warmup):
        driver.ccs_batch(chunks(args.zmws_per_step, seed0 + 1000 + w), settings, eng)
    work = [c for k in range(args.steps) for c in chunks(args.zmws_per_step, seed0 + k)]
    eng.kernel_stats(reset=True)
    barrier()
    sync()
    host = HostUsage()
    t0 = time.perf_counter()
    res = driver.ccs_batch(work, settings, eng)
    sync()
    barrier()
    local_time = time.perf_counter() - t0
    job_time = max_over_ranks(local_time, world)
    hostu = host.report(len(work), world)
    kstats = eng.kernel_stats(reset=True)
    statuses = {}
    for r in res:
        statuses[r["status"]] = statuses.get(r["status"], 0) + 1
    from pbccs_amd import poa
    st = poa.poa_stats(eng, reset=True)
    total = len(work) * world
    out = {"metric": "CCS ZMWs/sec end to end from raw subreads (FilterReads, POA, polish) on MI355X",
           "value": round(total / job_time, 3), "unit": "ZMWs/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(job_time / args.steps * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f64 (polish) / int32-uint16 (POA)",
           "data": "synthetic subreads (SURVEY.md §8(d): truth iid ACGT; 7%/4%/1% ins/del/sub; odd passes RC)",
           "config": {"workload": f"configs[1] end to end: {args.length} bp insert, {args.passes} subreads per "
                                  f"ZMW, {args.steps} x {args.zmws_per_step} ZMWs in one pbccs_ccs_batch",
                      "slots": slots, "chunk": args.ccs_chunk or "planned", "parallelism": f"zmw-shard x{world}"},
           "zmw_status": statuses, "poa_wall_ms": round(st["total_ms"], 1),
           "poa_device_ms": round(st["device_ms"], 1), "poa_thread_ms": round(st["thread_ms"], 1),
           "host": hostu}
    if any(v["launches"] for v in kstats.values()):   # the polish half's dominant kernel (the POA's: --stage poa)
        out["roofline"] = make_roofline(kstats, local_time, None)
        out["roofline"]["scope"] = "the polish kernels of the ccs run (the POA kernels' roofline is the --stage poa line)"
        out["kernels"] = {k: {"launches": v["launches"], "device_ms": round(v["device_ms"], 3),
                              "gcells": round(v["cells"] / 1e9, 4), "gbytes": round(v["bytes"] / 1e9, 4)}
                          for k, v in kstats.items() if v["launches"]}
    parity_ok = True
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        cb, parity = ccs_cpu_baseline(args, settings, work, res, min(args.cpu_sample, 160))
        out["cpu_baseline"], out["parity_sample"] = cb, parity
        out["vs_cpu"] = round(out["value"] / cb["value"], 2)
        out["vs_cpu_full_host"] = round(out["value"] / cb["full_host_value"], 3)
        out["vs_cpu_note"] = cpu_share_note()
        parity_ok = parity["ok"]
    if rank == 0:
        emit(out)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    if not parity_ok:
        log(rank, f"[bench] PARITY FAILURE on the timed ccs run's sample: {out['parity_sample']}")
        sys.exit(3)


def make_roofline(stats, local_time, workload):
    """The dominant kernel (by device time) priced three ways, each labelled:
    - per launch (the bench contract): algorithmic bytes per launch / the launch's average duration from HIP
      events on its own stream.  With several workspace slots the slots' launches of one kind run at the same
      time, so this duration is time-shared (`in_flight` = device time / wall time);
    - on wall time: the kernel's algorithmic bytes over the whole timed region / the region's wall time;
    - FP64 VALU: FLOP_PER_CELL x its DP cell-updates over the wall time, against the FP64 vector peak.
    Neither roof binds: the fill is a serial insertion chain (per band row a dependent mul + add + add, a DPP
    hand-off per two rows, CHAIN_ROW_CYCLES), so its bound is latency; `binding` says so.  `traffic` = PMC HBM
    bytes per launch of the same kernel from a committed profile, only while the kernel sources hash to the
    profile's digest.  `time_shared` is true when the launches overlap (in_flight > 1); `single_slot` then gives
    the same kernel's per-launch figure from the committed --streams 1 run of the same sources, whose launches
    do not overlap."""
    dom_name, dom = max(stats.items(), key=lambda kv: kv[1]["device_ms"])
    launches = max(1, dom["launches"])
    avg_ms = dom["device_ms"] / launches
    bytes_per_launch = dom["bytes"] / launches
    achieved = (bytes_per_launch / (avg_ms / 1e3)) / 1e9 if avg_ms > 0 else 0.0
    wall_gbs = dom["bytes"] / local_time / 1e9 if local_time > 0 else 0.0
    fp64_tf = FLOP_PER_CELL * dom["cells"] / local_time / 1e12 if local_time > 0 else 0.0
    traffic, traffic_src = None, None
    digest = kernel_source_digest()
    prof = TRAFFIC_PROFILES.get(dom_name)
    tpath = os.path.join(ROOT, "profiles", prof) if prof else None
    if tpath and os.path.exists(tpath):
        t = json.load(open(tpath))
        if t.get("bench_kernel") == dom_name and t.get("workload") == workload:
            if t.get("source_digest") == digest:
                traffic = t["traffic_bytes_per_launch"]
                traffic_src = (f"profiles/{prof} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, "
                               f"{t['dispatches_fetch_pass']} dispatches, sources {digest})")
            else:
                traffic_src = f"profiles/{prof} is stale: taken at sources {t.get('source_digest')}, built {digest}"
    single = None
    spath = os.path.join(ROOT, "profiles", SINGLE_SLOT_PROFILE)
    if os.path.exists(spath):
        s = json.load(open(spath))
        sr = s.get("roofline", {})
        if sr.get("kernel") == dom_name and sr.get("source_digest") == digest:
            single = {"frac": sr.get("frac"), "achieved": sr.get("achieved"), "avg_launch_ms": sr.get("avg_launch_ms"),
                      "in_flight": sr.get("in_flight"),
                      "source": f"profiles/{SINGLE_SLOT_PROFILE} (bench.py --streams 1, sources {digest})"}
        else:
            single = {"source": f"profiles/{SINGLE_SLOT_PROFILE} is stale: sources {sr.get('source_digest')}, "
                                f"built {digest}"}
    in_flight = dom["device_ms"] / (local_time * 1e3) if local_time > 0 else None
    return {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic, "traffic_source": traffic_src,
            "kernel": dom_name, "avg_launch_ms": round(avg_ms, 4), "launches": dom["launches"],
            "bytes_per_launch": bytes_per_launch, "cells_per_launch": dom["cells"] / launches,
            "per_launch_note": "achieved/frac: algorithmic bytes per launch / HIP-event launch time on the "
                               "kernel's stream; time-shared when in_flight > 1",
            "in_flight": round(in_flight, 3) if in_flight is not None else None,
            "time_shared": bool(in_flight is not None and in_flight > 1.0),
            "single_slot": single,
            "wall": {"achieved": round(wall_gbs, 3), "frac": round(wall_gbs / HBM_PEAK_GBS, 6), "unit": "GB/s",
                     "note": "the kernel's algorithmic bytes over the timed region / its wall time"},
            "fp64_valu": {"achieved": round(fp64_tf, 4), "peak": FP64_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                          "frac": round(fp64_tf / FP64_VALU_PEAK_TFLOPS, 6),
                          "note": f"{FLOP_PER_CELL} FLOP per DP cell-update over the timed region's wall time"},
            "bound_note": "the roofline axis the contract names (HBM bytes); not the binding resource, see binding",
            "binding": "no device resource saturates: VALU issue ~0.55 of the SIMDs' cycles, ~0.27 of the wave slots "
                       "and ~0.66 of the VGPR file held (occupancy), HBM < 0.1; more slots do not help (ten and twelve "
                       "lose, profiles/r4u_batch_shape.txt).  Each family is bound inside its own wavefronts: the fills "
                       "issue on ~0.6 of their wave cycles and are parked on LDS / memory waits ~0.35, with ~0.04 "
                       "dependency stalls -- per-wave instruction issue, the tall fill a lone wave on its SIMD -- and "
                       "k_score is parked on memory ~0.64 of its wave cycles (wave_cycles, tools/binding.py; "
                       "DESIGN.md section 6)",
            "source_digest": digest}


# MI355X_MICROARCH.md: 256 CUs x 4 SIMDs; per SIMD 8 wave slots and a 512-entry-per-lane VGPR file (allocation
# granule 8); a wave64 VALU instruction issues over 4 cycles of the SIMD's 16 lanes; engine clock 2.4 GHz
SIMDS, WAVE_SLOTS_PER_SIMD, VGPRS_PER_SIMD_LANE, VALU_CYCLES_PER_INST, ENGINE_HZ = 1024, 8, 512, 4, 2.4e9
# the kernel families whose wavefronts stamp their resident time (arrow_device.hpp WaveSlot) and their kernels'
# mangled-name stems in the build's resource table (pbccs_amd/_lib/kernel_resources.json, check_resources.py)
WAVE_FAMILIES = {"k_fill": ("k_fill_coopILi16E",), "k_fill_tall": ("k_fill_coopILi64E",),
                 "k_score": ("7k_scoreE",), "k_suffix": ("8k_suffixE",),
                 "k_reduce": ("8k_reduceE",)}
VALU_PROFILE = "r6_valu_per_cell.json"
BINDING_PROFILE = "r6_binding_summary.json"   # wave-cycle decomposition per family (tools/gpu_steps.sh binding)   # SQ_INSTS_VALU per kernel family (tools/gpu_steps.sh valu)
OCC_PROFILE = "r6_occupancy_bench.json"  # the driver's command on the occupancy build (tools/gpu_steps.sh occ)


def occupancy_report(stats, local_time):
    """Which device resource the concurrent batches fill, from in-kernel wave stamps: each
    wavefront of the fill / score / suffix / reduce kernels adds its start-to-end time (`wave_s`), so over the timed
    region a family's wave_s / wall = its average resident wavefronts.  Against the device: wave slots (8 per SIMD),
    the VGPR file (a family's allocation per wave from the build's resource table, x its resident waves, over
    1024 SIMDs x 512), and VALU issue (SQ_INSTS_VALU per launch from the committed PMC pass of the same sources x
    this run's launches x 4 cycles, over the SIMDs' cycles).  Wave time counts waiting waves too: the fraction of
    the VGPR file held is the occupancy the batches reach, the VALU fraction what they issue with it."""
    if local_time <= 0 or not any(s.get("wave_s") for s in stats.values()):
        return None   # the default build has the stamps compiled out (PBCCS_WAVE_STAMPS; they cost 5%)
    from pbccs_amd import lib as _L
    rpath = os.path.join(os.path.dirname(_L.LIB_PATH), "kernel_resources.json")   # the loaded build's table
    res = json.load(open(rpath)) if os.path.exists(rpath) else {}
    fams, waves_tot, vgpr_tot = {}, 0.0, 0.0
    for fam, stems in WAVE_FAMILIES.items():
        s = stats.get(fam)
        if not s or not s.get("wave_s"):
            continue
        allocs = [((v.get("vgprs", 0) + v.get("agprs", 0) + 7) // 8) * 8 for k, v in res.items()
                  if any(st in k for st in stems)]
        alloc = max(allocs) if allocs else None
        waves = s["wave_s"] / local_time
        waves_tot += waves
        if alloc:
            vgpr_tot += waves * alloc
        fams[fam] = {"resident_waves": round(waves, 1), "vgprs_per_lane": alloc,
                     "waves_per_simd_limit": min(WAVE_SLOTS_PER_SIMD, VGPRS_PER_SIMD_LANE // alloc) if alloc else None}
    out = {"families": fams, "resident_waves": round(waves_tot, 1),
           "waves_per_simd": round(waves_tot / SIMDS, 3),
           "wave_slot_frac": round(waves_tot / (SIMDS * WAVE_SLOTS_PER_SIMD), 4),
           "vgpr_file_frac": round(vgpr_tot / (SIMDS * VGPRS_PER_SIMD_LANE), 4) if res else None,
           "resource_table": os.path.relpath(rpath, ROOT) if res else "missing (build the library)",
           "build": "PBCCS_WAVE_STAMPS=1 (the occupancy build, tools/gpu_steps.sh occ)"}
    vpath = os.path.join(ROOT, "profiles", VALU_PROFILE)
    if os.path.exists(vpath):
        v = json.load(open(vpath))
        if v.get("source_digest") == kernel_source_digest():
            cyc = 0.0
            for fam, d in v.get("kernels", {}).items():
                if fam in stats and d.get("valu_insts") and d.get("dispatches"):
                    cyc += d["valu_insts"] / d["dispatches"] * stats[fam]["launches"] * VALU_CYCLES_PER_INST
            out["valu_issue_frac"] = round(cyc / (local_time * ENGINE_HZ * SIMDS), 4)
            out["valu_source"] = f"profiles/{VALU_PROFILE} (rocprofv3 --pmc SQ_INSTS_VALU, same sources)"
        else:
            out["valu_source"] = f"profiles/{VALU_PROFILE} is stale: sources {v.get('source_digest')}"
    return out


FILL_WORK_SLOTS = ("counted_cells", "tall_abort_cells", "regrow_cells", "overflow_cells", "group_chunk_steps",
                   "wave_chunk_issues", "reads", "passes")


def fill_work_report(w):
    """PBCCS_FILL_WORK=1 (CoopFill::work): where each fill kind's computed cells went, and how busy its wavefronts'
    groups were.  computed = counted + thrown away by a tall abort + count-only regrow passes + count-only overflow
    fills; lockstep = the groups' chunk steps / (groups per wave x the wave's chunk issues)."""
    out = {}
    for k, (name, groups) in enumerate((("k_fill", 4), ("k_fill_tall", 1))):
        d = dict(zip(FILL_WORK_SLOTS, w[8 * k:8 * k + 8]))
        comp = d["counted_cells"] + d["tall_abort_cells"] + d["regrow_cells"] + d["overflow_cells"]
        d["computed_cells"] = comp
        d["counted_frac"] = round(d["counted_cells"] / comp, 4) if comp else None
        d["lockstep_eff"] = round(d["group_chunk_steps"] / (groups * d["wave_chunk_issues"]), 4) \
            if d["wave_chunk_issues"] else None
        out[name] = d
    return out


def report(args, rank, world, eng, slots, job_time, local_time, res, workload, scaling, total_zmws, qstats=None,
           extra=None, settings=None):
    import torch.distributed as dist
    extra = extra or {}
    stats = eng.kernel_stats(reset=True)
    counters = eng.counters(reset=True)
    statuses = {}
    for r in res:
        statuses[r["status"]] = statuses.get(r["status"], 0) + 1

    value = total_zmws / job_time
    n_gated = sum(v for k, v in statuses.items() if k in ("TooFewPasses", "TooManyUnusable", "NoSubreads", "TooShort"))
    n_polished = sum(statuses.values()) - n_gated
    if world > 1 and scaling == "weak":   # each rank holds its own records: sum the counts
        import torch
        from pbccs_amd import ZMW_STATUS
        names = list(ZMW_STATUS)   # the same list on every rank (a record's status is one of these)
        t = torch.tensor([n_polished, n_gated] + [statuses.get(k, 0) for k in names], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        n_polished, n_gated = int(t[0].item()), int(t[1].item())
        statuses = {k: int(v) for k, v in zip(names, t[2:].tolist()) if v}
    cells = sum(s["cells"] for s in stats.values())
    gcups_local = cells / local_time / 1e9 if local_time > 0 else 0.0
    gcups = gcups_local * world
    if world > 1:   # sum of the ranks' cells over the job time
        import torch
        t = torch.tensor([cells], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        gcups = float(t.item()) / job_time / 1e9

    roofline = make_roofline(stats, local_time, workload)
    occ = occupancy_report(stats, local_time)
    if occ is None and workload.startswith("configs[1]"):
        # the default build has no wave stamps: the committed occupancy run of the same sources stands in
        opath = os.path.join(ROOT, "profiles", OCC_PROFILE)
        if os.path.exists(opath):
            o = json.load(open(opath))
            if o.get("roofline", {}).get("source_digest") == kernel_source_digest():
                occ = dict(o["roofline"].get("occupancy") or {})
                occ["source"] = f"profiles/{OCC_PROFILE} (the occupancy build, same kernel sources, same command)"
    if occ:
        roofline["occupancy"] = occ
        roofline["binding_measured"] = (
            f"over the timed region {occ['waves_per_simd']} waves resident per SIMD ({occ['wave_slot_frac']} of the "
            f"wave slots), holding {occ['vgpr_file_frac']} of the VGPR file; VALU issue "
            f"{occ.get('valu_issue_frac', 'n/a')} of the SIMDs' cycles (roofline.occupancy)")
        tw = (occ.get("families", {}).get("k_fill_tall") or {}).get("resident_waves")
        tall = stats.get("k_fill_tall")
        if tw and tall and local_time > 0:   # the tall fill against its own serial-chain bound
            bound = tw * ENGINE_HZ / CHAIN_ROW_CYCLES
            got = tall["cells"] / local_time
            roofline["chain_bound"] = {
                "achieved_cells_per_s": round(got / 1e9, 3), "bound_cells_per_s": round(bound / 1e9, 3),
                "unit": "G cells/s", "frac": round(got / bound, 4), "resident_tall_waves": tw,
                "cycles_per_row": CHAIN_ROW_CYCLES,
                "note": "resident tall waves x clock / the exact chain's cycles per band row (tools/ubench/"
                        "chain_step.hip); the certified scan path (DESIGN.md 3.12) has no per-row chain, so its "
                        "reads can exceed this bound"}
    bpath = os.path.join(ROOT, "profiles", BINDING_PROFILE)
    if workload.startswith("configs[1]") and os.path.exists(bpath):
        bp = json.load(open(bpath))
        if bp.get("source_digest") == kernel_source_digest():
            roofline["wave_cycles"] = {k: {x: v.get(x) for x in ("issuing_frac", "issue_stalled_frac",
                                                                 "waitcnt_parked_frac", "valu_issuing_frac",
                                                                 "l2_hit_frac")}
                                       for k, v in bp.get("kernels", {}).items()}
            roofline["wave_cycles_source"] = (f"profiles/{BINDING_PROFILE} (rocprofv3 --pmc SQ_WAVE_CYCLES, "
                                              f"SQ_ACTIVE_INST_ANY, SQ_WAIT_INST_ANY, SQ_WAIT_ANY, ...; same sources)")
        else:
            roofline["wave_cycles_source"] = f"profiles/{BINDING_PROFILE} is stale: sources {bp.get('source_digest')}"
    out = {
        "metric": "CCS ZMWs/sec (and GCUPS) at 1/2/4/8 MI355X vs host-CPU ccs",
        "stage": "polish: Consensus.h:436-552 from the POA draft on (AddRead gates, RefineConsensus, "
                 "ConsensusQVs); FilterReads and the POA are the --stage ccs line",
        "value": round(value, 3),
        "unit": "ZMWs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(job_time / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY.md §8(d): truth iid ACGT; subreads 7%/4%/1% ins/del/sub; draft 0.5/0.5/0.2%)",
        "config": {"workload": workload,
                   "zmws_per_step": args.zmws_per_step,
                   "zmws_total": total_zmws,
                   "insert_bp": args.length if args.workload == "2kb" else
                   {"10kb": 10000, "mixed": "500-20000", "smrtcell": "mix"}[args.workload],
                   "passes": args.passes if args.workload == "2kb" else
                   {"10kb": 8, "mixed": "3-30", "smrtcell": "mix"}[args.workload],
                   "slots": slots,
                   "device_batch_zmws": (max(1, args.zmws_per_step // max(1, args.batch_split))
                                         if args.workload == "2kb" else "planned"),
                   "parallelism": f"zmw-shard x{world}"},
        "gcups": round(gcups, 3),
        "zmw_status": statuses,
        # ZMWs that reached RefineConsensus (Consensus.h:493-512) against those the AddRead gates dropped before
        # it (TooFewPasses / TooManyUnusable): the polish rate of the configs[3] mix is the first figure
        "polished": {"zmws": n_polished, "zmws_per_s": round(n_polished / job_time, 3) if job_time > 0 else None,
                     "gated_zmws": n_gated},
        "roofline": roofline,
        "kernels": {k: {"launches": v["launches"], "device_ms": round(v["device_ms"], 3),
                        "gcells": round(v["cells"] / 1e9, 4), "gbytes": round(v["bytes"] / 1e9, 4)}
                    for k, v in stats.items() if v["launches"]},
        "score_tasks": counters["score_tasks"],
        "mutations_scored": counters["mutations"],
        "band_memory_gb": {k: round(counters[k] / 2**30, 3) for k in
                           ("band_top_bytes", "band_region_bytes", "band_used_bytes", "pool_mapped_bytes")},
        "oom_retries": counters["oom_retries"],
        # the certified fast path: tall reads filled by the reassociated chain, reads re-run exactly
        # for an uncertain fill decision or AddRead gate, ZMW rounds re-scored on exact bands for an uncertain score
        # decision (PBCCS_CERTIFIED_SCAN=0 turns the path off)
        "certified_scan": {"scan_reads": counters.get("scan_reads", 0),
                           "uncertain_reads": counters.get("uncertain_reads", 0),
                           "exact_rounds": counters.get("exact_rounds", 0),
                           "uncertain_why": dict(zip(("band_end", "begin_hint", "loop_entry", "final_mismatch"),
                                                     counters.get("uncertain_why", [0] * 4))),
                           "on": os.environ.get("PBCCS_CERTIFIED_SCAN", "1") != "0"},
    }
    if qstats:   # configs[4]: records stream to rank 0 per chunk; tail_ms = rank 0's wait after its last chunk
        out["queue"] = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in qstats.items()}
    if any(counters.get("fill_work") or []):
        out["fill_work"] = fill_work_report(counters["fill_work"])
    if "host" in extra:
        out["host"] = extra["host"]
    if "prepare" in extra:
        out["prepare"] = extra["prepare"]
        out["prepare"]["derive_thread_s_in_timed"] = round(counters.get("derive_ns", 0) / 1e9, 3)
        # the reader's share outside the timed region, as a fraction of it (in ccs reading overlaps the polish;
        # here it is not pipelined: VERDICT r5 item 7)
        timed_s = out.get("ms_per_step", 0.0) * out.get("steps", 0) / 1e3
        if timed_s > 0 and "marshal_s" in out["prepare"]:
            out["prepare"]["marshal_frac_of_timed"] = round(out["prepare"]["marshal_s"] / timed_s, 4)
    parity_ok = True
    # the CPU leg on rank 0 (one rank: its records are the run's; several ranks: rank 0 holds the whole cell's
    # records for the strong-scaling cell, its own for the weak-scaling lines)
    if rank == 0 and args.cpu_sample > 0 and res and extra.get("zs") is not None and settings is not None:
        zs, costs = extra["zs"], extra.get("costs")
        if world == 1 or scaling == "strong":
            idx = sample_indices(args, len(res), costs)
            log(rank, f"[bench] CPU leg: {len(idx)} of the timed ZMWs on the restatement")
            cb, parity = sampled_cpu_baseline(args, settings, zs, res, idx, costs)
            if costs is not None:
                cb["coverage"] = coverage(costs)
            out["cpu_baseline"] = cb
            out["parity_sample"] = parity
            out["vs_cpu"] = round(value / cb["value"], 2)
            out["vs_cpu_full_host"] = round(value / cb["full_host_value"], 3)
            out["vs_cpu_note"] = cpu_share_note()
            parity_ok = parity["ok"]
    if rank == 0:
        emit(out)
    if world > 1:
        dist.destroy_process_group()
    if not parity_ok:
        log(rank, f"[bench] PARITY FAILURE on the timed run's sample: {out['parity_sample']}")
        sys.exit(3)


if __name__ == "__main__":
    main()
