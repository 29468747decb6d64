#!/usr/bin/env python3
"""CCS polish throughput on MI355X (BASELINE.json metric: CCS ZMWs/sec and GCUPS).

A step polishes one batch of synthetic ZMWs (2 kb insert, 10 full passes)
end to end on the GPU: AddRead fills + z-score gates, RefineConsensus, ConsensusQVs -- the per-ZMW
polish that pbccs' Consensus.h runs after the POA.  Inputs are copied to HBM before the timed region
(pbccs_batch_create); the timed region is exactly K steps, bracketed by a barrier and
torch.cuda.synchronize() on both sides; the job time is the max over ranks.  The K steps are pipelined
(pbccs_batch_polish_many: one host thread + HIP stream per batch in flight), so one batch's convergence
tail -- the last refine rounds of its few slow ZMWs -- overlaps the others' work, the way ccs's ZMW thread
pool overlaps ZMWs.  Default: 5 steps x 2000 ZMWs = the 10k-ZMW workload of configs[1].  Multi-GPU: each rank polishes its own shard (weak scaling,
no data-path collective).  rank 0 prints one JSON line.
"""
import argparse
import json
import math
import os
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
TRAFFIC_PROFILE = "r1i_traffic_fill.json"   # PMC HBM bytes of the roofline kernel (tools/gpu_traffic.sh)
FP64_VALU_PEAK_TFLOPS = 78.6   # MI355X FP64 vector peak (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--zmws-per-step", type=int, default=2000)
    ap.add_argument("--warmup-zmws", type=int, default=0,
                    help="ZMWs per warmup step (0 = --zmws-per-step: a warmup step is a full-size step, so the "
                         "engine's score and selection buffers reach their steady-state size before timing)")
    ap.add_argument("--length", type=int, default=2000)
    ap.add_argument("--passes", type=int, default=10)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--workload", choices=["2kb", "10kb", "mixed"], default="2kb",
                    help="2kb: configs[1], the headline line (pre-created batches, inputs resident in HBM). "
                         "10kb / mixed: configs[2] / configs[3] through the ZMW work queue (polish_stream: "
                         "length/pass buckets, memory-sized batches, largest first); the timed region then "
                         "includes the host->device copy of the reads")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="ZMWs polished by the CPU baseline (0 = skip; default 192 for 2kb, 0 otherwise)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--streams", type=int, default=0,
                    help="batches polished concurrently (0 = min(steps, 8)); each has its own HIP stream")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def cpu_baseline(args, rank):
    """The oracle (bit-faithful CPU restatement, test infrastructure) on host cores, one ZMW per task on a
    thread pool like `ccs --numThreads` (src/main/ccs.cpp:222-230)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    from pbccs_amd import synth

    n = args.cpu_sample
    threads = args.cpu_threads or min(16, os.cpu_count() or 1)
    threads = max(1, min(threads, n))
    zmws = synth.make_zmws(n, seed=args.seed + 99991, **workload_kw(args))
    O.lib()
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=threads) as ex:
        list(ex.map(lambda z: O.polish_zmw(z["draft"], z["reads"], z["snr"]), zmws))
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "ZMWs/s", "cores": threads, "kind": "port",
            "sample": f"{n} synthetic ZMWs of the same config ({args.workload}), "
                      f"oracle/arrow_oracle.cpp polish (AddRead, RefineConsensus, ConsensusQVs) on {threads} "
                      f"host threads, {dt:.1f} s wall"}


def workload_kw(args):
    """synth.make_zmws keywords of the workload."""
    if args.workload == "10kb":
        return dict(length=10000, passes=8)
    if args.workload == "mixed":
        return dict(length=None, passes=None, length_range=(500, 20000), passes_range=(3, 30), random_snr=True)
    return dict(length=args.length, passes=args.passes)


def queue_workload(args, rank, world, eng, settings, seed0):
    """configs[2] / configs[3] through the work queue; returns (job_time, local_time, results, workload)."""
    import pbccs_amd
    import torch
    import torch.distributed as dist
    from pbccs_amd import synth
    n = args.steps * args.zmws_per_step
    kw = workload_kw(args)
    if args.workload == "10kb":
        desc = f"configs[2]: synthetic 10000 bp insert, 8 full passes, {n} ZMWs per GPU"
    else:
        desc = f"configs[3]: synthetic 0.5-20 kb inserts, 3-30 passes, per-ZMW SNR U[4,20], {n} ZMWs per GPU"
    for w in range(args.warmup):
        pbccs_amd.polish_stream(synth.make_zmws(max(1, args.warmup_zmws), seed=seed0 + 1000 + w, **kw), settings, eng)
    log(rank, "[bench] warmup done")
    zs = synth.make_zmws(n, seed=seed0, **kw)
    eng.kernel_stats(reset=True)
    eng.counters(reset=True)
    if world > 1:
        dist.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    # one native call polishes the whole stream; a heartbeat on stderr shows it is alive (ctypes drops the GIL)
    import threading
    done = threading.Event()

    def heartbeat():
        while not done.wait(30.0):
            log(rank, f"[bench] work queue running t={time.perf_counter() - t0:.0f}s")
    hb = threading.Thread(target=heartbeat, daemon=True)
    hb.start()
    try:
        res = pbccs_amd.polish_stream(zs, settings, eng)
    finally:
        done.set()
        hb.join()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    local_time = time.perf_counter() - t0
    job_time = local_time
    if world > 1:
        t = torch.tensor([local_time], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        job_time = float(t.item())
    return job_time, local_time, res, desc + " (work queue; timed region includes the read upload)"


def main():
    args = parse()
    if args.cpu_sample is None:
        args.cpu_sample = 192 if args.workload == "2kb" else 0
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # torch first: the engine then binds to the same HIP runtime instance (both carry soname libamdhip64.so.7)
    import torch
    import torch.distributed as dist
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group(backend="gloo")   # barrier + max-time only: the polish path has no collective

    import pbccs_amd
    from pbccs_amd import synth

    def barrier():
        if world > 1:
            dist.barrier()

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    eng = pbccs_amd.Engine(local)
    streams = args.streams or max(1, min(args.steps, 8))
    eng.set_concurrency(streams)
    if not args.no_profile:
        eng.set_profiling(True)   # HIP events on the engine stream + in-kernel algorithmic counters
    settings = pbccs_amd.ConsensusSettings()
    seed0 = args.seed + 7919 * rank

    if args.workload != "2kb":
        job_time, local_time, res, workload = queue_workload(args, rank, world, eng, settings, seed0)
        return report(args, rank, world, eng, streams, job_time, local_time, res, workload)

    # ---- warmup (untimed) -------------------------------------------------------------------
    if args.warmup_zmws <= 0:
        args.warmup_zmws = args.zmws_per_step
    # a warmup step polishes one batch per workspace slot, concurrently like the timed steps, so every
    # slot's score/selection buffers and band pool reach steady-state size (their growth would otherwise
    # allocate -- and synchronise the device -- inside the timed region)
    for w in range(args.warmup):
        wb = [pbccs_amd.PreparedBatch(synth.make_zmws(args.warmup_zmws, args.length, args.passes,
                                                      seed=seed0 + 1000 + 37 * w + s), settings, eng)
              for s in range(streams)]
        pbccs_amd.polish_many(wb)
        for b in wb:
            b.close()
    log(rank, f"[bench] warmup done ({args.warmup} x {streams} x {args.warmup_zmws} ZMWs)")

    # ---- engine pools mapped before the timed region (a long run maps them once and reuses them) ----
    if torch.cuda.is_available():
        free_b, _ = torch.cuda.mem_get_info(local)
        per_slot = int(min(0.6 * free_b / streams, 48 << 30))
        eng.reserve_pool(per_slot)
        log(rank, f"[bench] mapped {per_slot / 2**30:.1f} GB of band pool per slot x {streams}")

    # ---- inputs resident in HBM before the timed region ------------------------------------------
    t_prep = time.perf_counter()
    batches = []
    for k in range(args.steps):
        zs = synth.make_zmws(args.zmws_per_step, args.length, args.passes, seed=seed0 + k)
        batches.append(pbccs_amd.PreparedBatch(zs, settings, eng))
        log(rank, f"[bench] prepared step {k} ({args.zmws_per_step} ZMWs) t={time.perf_counter() - t_prep:.1f}s")
    eng.kernel_stats(reset=True)
    eng.counters(reset=True)

    # ---- timed region: exactly K steps --------------------------------------------------------
    barrier()
    sync()
    t0 = time.perf_counter()
    pbccs_amd.polish_many(batches)   # the K steps, pipelined over `streams` HIP streams / host threads
    log(rank, f"[bench] {args.steps} steps done t={time.perf_counter() - t0:.2f}s")
    sync()
    barrier()
    t1 = time.perf_counter()
    local_time = t1 - t0
    if world > 1:
        t = torch.tensor([local_time], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        job_time = float(t.item())
    else:
        job_time = local_time

    res = [r for b in batches for r in b.results()]
    for b in batches:
        b.close()
    workload = (f"configs[1]: synthetic {args.length} bp insert, {args.passes} full passes, "
                f"{args.zmws_per_step * args.steps} ZMWs per GPU ({args.steps} steps x {args.zmws_per_step})")
    report(args, rank, world, eng, streams, job_time, local_time, res, workload)


def report(args, rank, world, eng, streams, job_time, local_time, res, workload):
    import torch.distributed as dist
    stats = eng.kernel_stats(reset=True)
    counters = eng.counters(reset=True)
    n_local = len(res)
    statuses = {}
    for r in res:
        statuses[r["status"]] = statuses.get(r["status"], 0) + 1

    total_zmws = n_local * world
    value = total_zmws / job_time
    cells = sum(s["cells"] for s in stats.values())
    gcups_local = cells / local_time / 1e9 if local_time > 0 else 0.0

    # dominant kernel (by device time) -> roofline: algorithmic band bytes / its device time
    dom_name, dom = max(stats.items(), key=lambda kv: kv[1]["device_ms"])
    launches = max(1, dom["launches"])
    avg_ms = dom["device_ms"] / launches
    bytes_per_launch = dom["bytes"] / launches
    achieved = (bytes_per_launch / (avg_ms / 1e3)) / 1e9 if avg_ms > 0 else 0.0
    # HBM traffic per launch: PMC counters cannot be read from inside this process, so `traffic` comes from
    # the committed rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this same default command
    # (tools/gpu_traffic.sh -> tools/pmc_traffic.py, gfx950 correction 2*FETCH_SIZE + WRITE_SIZE) when
    # they were taken on this kernel family and workload; null otherwise.
    traffic, traffic_src = None, None
    tpath = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", TRAFFIC_PROFILE)
    if os.path.exists(tpath):
        t = json.load(open(tpath))
        if t.get("kernel") == dom_name and t.get("workload") == workload:
            traffic = t["traffic_bytes_per_launch"]
            traffic_src = f"profiles/{TRAFFIC_PROFILE} (rocprofv3 --pmc, {t['dispatches_fetch_pass']} dispatches)"
    roofline = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic, "traffic_source": traffic_src,
                "kernel": dom_name, "avg_launch_ms": round(avg_ms, 4), "launches": dom["launches"],
                "bytes_per_launch": bytes_per_launch, "cells_per_launch": dom["cells"] / launches}

    out = {
        "metric": "CCS ZMWs/sec (and GCUPS) at 1/2/4/8 MI355X vs host-CPU ccs",
        "value": round(value, 3),
        "unit": "ZMWs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(job_time / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY.md §8(d): truth iid ACGT; subreads 7%/4%/1% ins/del/sub; draft 0.5/0.5/0.2%)",
        "config": {"workload": workload,
                   "zmws_per_step": args.zmws_per_step,
                   "insert_bp": args.length if args.workload == "2kb" else
                   (10000 if args.workload == "10kb" else "500-20000"),
                   "passes": args.passes if args.workload == "2kb" else (8 if args.workload == "10kb" else "3-30"),
                   "streams": streams,
                   "parallelism": f"zmw-shard x{world}"},
        "gcups": round(gcups_local * world, 3),
        "zmw_status": statuses,
        "roofline": roofline,
        "kernels": {k: {"launches": v["launches"], "device_ms": round(v["device_ms"], 3),
                        "gcells": round(v["cells"] / 1e9, 4), "gbytes": round(v["bytes"] / 1e9, 4)}
                    for k, v in stats.items()},
        "score_tasks": counters["score_tasks"],
        "mutations_scored": counters["mutations"],
    }
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        out["cpu_baseline"] = cpu_baseline(args, rank)
        out["vs_cpu"] = round(value / out["cpu_baseline"]["value"], 2)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
