"""Multi-GPU ccs polish: ZMWs shard across ranks (one process per GPU), results gather in input order.

ZMWs are independent, so the data path has no collective: each rank polishes its own
shard on its own GPU, and only the finished per-ZMW records travel to rank 0, which reassembles them in
input order -- the ordering contract of pbccs' writer FIFO (include/pacbio/ccs/WorkQueue.h:128-167).  The
dynamic queue streams them chunk by chunk as they finish; the static plan gathers once.
The shard assignment is a deterministic cost-balanced partition (longest-processing-time first over an
estimate of each ZMW's DP work), so every rank computes the same plan without communicating.
"""
import heapq


def zmw_cost(z):
    """Work estimate of one ZMW's polish: template length x total read bases (fills and scoring both scale
    with the band area J x I per read, SURVEY.md §8 sizing)."""
    return max(1, len(z["draft"])) * max(1, sum(len(r["seq"]) for r in z["reads"]))


def shard_plan(costs, world):
    """LPT partition of work items over `world` ranks: largest first onto the least-loaded rank (ties by
    rank, then by input index).  Returns one ascending index list per rank."""
    loads = [(0, r) for r in range(world)]
    heapq.heapify(loads)
    parts = [[] for _ in range(world)]
    for i in sorted(range(len(costs)), key=lambda i: (-costs[i], i)):
        load, r = heapq.heappop(loads)
        parts[r].append(i)
        heapq.heappush(loads, (load + costs[i], r))
    return [sorted(p) for p in parts]


def gather_in_order(local_results, local_indices, n_total, rank, world, group=None):
    """Gather (index, record) pairs to rank 0 and return the records in input order there (None elsewhere).
    One gather_object of the finished records: the only inter-rank traffic of the job."""
    import torch.distributed as dist
    payload = list(zip(local_indices, local_results))
    if world == 1:
        gathered = [payload]
    else:
        gathered = [None] * world if rank == 0 else None
        dist.gather_object(payload, gathered, dst=0, group=group)
    if rank != 0:
        return None
    out = [None] * n_total
    for part in gathered:
        for i, rec in part:
            out[i] = rec
    missing = [i for i, rec in enumerate(out) if rec is None]
    if missing:
        raise RuntimeError(f"ZMWs missing after the gather: {missing[:8]}")
    return out


_queue_calls = [0]


def dynamic_chunks(zmws, chunk):
    """The pull queue's work items: ZMW indices in decreasing cost (largest first, so the ranks' last pulls are
    the cheap chunks), cut into chunks of at most `chunk` ZMWs and of at most 1 / ceil(n / chunk) of the total
    cost each.  The cost cap splits the expensive end finer: equal-count chunks put the cell's 500 costliest
    ZMWs (20 kb, up to 30 passes) in one chunk, which one rank then polished for 527 s after the other had run
    out of work (configs[4] at 10,000 ZMWs on two ranks, profiles/r9x_smrtcell_10000_gpus2_rehearsal.json).
    A lazily generated cell (synth.SmrtCell) gives its costs from the ZMW shapes, without materialising a
    sequence."""
    costs = zmws.costs() if hasattr(zmws, "costs") else [zmw_cost(z) for z in zmws]
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    n_target = max(1, -(-len(order) // max(1, chunk)))
    cap = sum(costs) / n_target
    out, cur, cur_cost = [], [], 0
    for i in order:
        if cur and (len(cur) >= chunk or cur_cost + costs[i] > cap):
            out.append(cur)
            cur, cur_cost = [], 0
        cur.append(i)
        cur_cost += costs[i]
    if cur:
        out.append(cur)
    return out


STORE_PART = 4 << 20   # bytes per value put on the rank-0 key-value store (whose values are capped at 8 MB)


def _store_timeout_s(store, default=1800.0):
    try:
        return float(store.timeout.total_seconds())
    except Exception:
        return default


def polish_dynamic(zmws, settings=None, engine=None, rank=None, world=None, chunk=256, polish_fn=None, store=None,
                   group=None, stats=None, collect_timeout=None):
    """Polish `zmws` across ranks through a dynamic pull queue: every rank takes the next
    chunk index from one shared counter -- an atomic fetch-add on the rank-0 key-value store, host-side, not a
    device collective -- until the queue is empty, so a rank that drew slow ZMWs (tall bands, long templates)
    simply pulls fewer chunks.

    Results stream to rank 0 as chunks finish (the ordered FIFO of WorkQueue.h:128-167 fed as workers
    complete): a rank > 0 puts each finished chunk's records under its own key on the same store, and a
    collector thread on rank 0 takes them as they arrive while rank 0's own thread keeps polishing -- a long
    chunk on rank 0 never delays the collection.  Once the queue is empty only the chunks still running
    elsewhere are left to wait for; nothing is gathered in one piece at the end.

    `zmws` may be a list or a lazily generated cell (synth.SmrtCell): a rank then materialises only the chunks
    it pulls, the next one on a helper thread while the current one polishes.

    A rank claims the next chunk before polishing the current one (so its generation overlaps the polish) only
    while at least `world` chunks are left: near the end a pre-claimed chunk would sit idle on one rank while the
    others have nothing to pull.

    Rank 0 returns every ZMW's result in input order; the other ranks return None.  If no record arrives for
    `collect_timeout` seconds (default: the store's timeout) while chunks other ranks took are outstanding, rank 0
    raises instead of waiting forever on a rank that died.  `stats` (a dict, optional) receives the queue's
    counters: on every rank `zmws_local` (ZMWs this rank polished) and `gen_ms` (its time waiting for chunk
    generation); on rank 0 chunks per rank and `tail_ms` (the time from rank 0's last chunk to the last record)."""
    import pickle
    import threading
    import time
    from concurrent.futures import ThreadPoolExecutor
    import torch.distributed as dist
    if rank is None:
        rank = dist.get_rank() if dist.is_initialized() else 0
    if world is None:
        world = dist.get_world_size() if dist.is_initialized() else 1
    chunks = dynamic_chunks(zmws, chunk)
    if polish_fn is None:
        from . import polish_stream

        def polish_fn(zs):
            return polish_stream(zs, settings, engine)
    _queue_calls[0] += 1
    key = f"pbccs_queue_{_queue_calls[0]}"
    if world > 1 and store is None:
        store = dist.distributed_c10d._get_default_store()
    lock = threading.Lock()   # one store client, used by the puller and by rank 0's collector
    out = [None] * len(zmws) if rank == 0 else None
    mine = set()       # chunks this rank polished
    taken = [0] * world
    lazy = hasattr(zmws, "costs")

    # ---- rank 0's collector: records of the chunks other ranks took, as soon as they are stored ----------
    pending = set()    # chunk indices handed to other ranks whose records are not collected yet
    final = threading.Event()
    collector_err = []

    def collect_one(c):
        k = f"{key}/done/{c}"
        with lock:
            if not store.check([k]):
                return False
            nparts = int(store.get(k))
            parts = []
            for q in range(nparts):
                parts.append(store.get(f"{k}/p{q}"))
                store.delete_key(f"{k}/p{q}")
            store.delete_key(k)
        who, recs = pickle.loads(b"".join(parts))
        taken[who] += 1
        for i, rec in zip(chunks[c], recs):
            out[i] = rec
        return True

    deadline_s = collect_timeout if collect_timeout is not None else _store_timeout_s(store)

    def collector():
        try:
            last = time.perf_counter()   # the last record collected, `final` being set, or pending filling again
            seen_final = False
            was_empty = True
            while True:
                with lock:
                    todo = sorted(pending)
                if todo and was_empty:   # chunks handed out after an idle spell: their clock starts now
                    last = time.perf_counter()
                was_empty = not todo
                got = [c for c in todo if collect_one(c)]
                with lock:
                    pending.difference_update(got)
                    empty = not pending
                if final.is_set() and not seen_final:
                    seen_final, last = True, time.perf_counter()
                if final.is_set() and empty:
                    return
                if got:
                    last = time.perf_counter()
                elif todo and time.perf_counter() - last > deadline_s:
                    raise RuntimeError(f"no record from the other ranks for {deadline_s:.0f} s; chunks still "
                                       f"outstanding: {todo[:8]} (a rank died?)")
                else:
                    time.sleep(0.005)
        except Exception as e:   # surfaced by the main thread
            collector_err.append(e)

    coll = None
    if rank == 0 and world > 1:
        coll = threading.Thread(target=collector, daemon=True)
        coll.start()

    serial = [0]
    high = [0]         # rank 0: chunk indices below `high` were handed out

    def pull():
        if world > 1:
            with lock:
                c = store.add(key, 1) - 1
        else:
            c = serial[0]
            serial[0] += 1
        if rank == 0 and world > 1:
            with lock:   # handed to other ranks since our last pull
                pending.update(range(high[0], min(c, len(chunks))))
            high[0] = max(high[0], c + 1)
        return c

    def materialise(c):
        return [zmws[i] for i in chunks[c]] if c < len(chunks) else None

    gen = ThreadPoolExecutor(max_workers=1) if lazy else None
    gen_ms = 0.0
    n_local = 0
    try:
        c = pull()
        fut = gen.submit(materialise, c) if gen else None
        while c < len(chunks):
            t0 = time.perf_counter()
            zs = fut.result() if gen else materialise(c)
            gen_ms += (time.perf_counter() - t0) * 1e3
            nxt = None
            # claim and generate the next chunk while this one polishes, but only while at least `world` chunks
            # are left: a chunk claimed early near the end would wait on this rank while the others run dry
            if gen and len(chunks) - (c + 1) >= world:
                nxt = pull()
                fut = gen.submit(materialise, nxt)
            recs = polish_fn(zs)
            n_local += len(zs)
            mine.add(c)
            if rank == 0:
                taken[0] += 1
                for i, rec in zip(chunks[c], recs):
                    out[i] = rec
            else:
                blob = pickle.dumps((rank, recs))
                # the store takes values of up to 8 MB: the records go in parts, the part count last (the
                # collector reads a chunk once its count key exists)
                nparts = max(1, (len(blob) + STORE_PART - 1) // STORE_PART)
                with lock:
                    for q in range(nparts):
                        store.set(f"{key}/done/{c}/p{q}", blob[q * STORE_PART:(q + 1) * STORE_PART])
                    store.set(f"{key}/done/{c}", str(nparts))
            if nxt is not None:
                c = nxt
            else:
                c = pull()
                if gen:
                    fut = gen.submit(materialise, c)
    finally:
        if gen:
            gen.shutdown(wait=True)
    if stats is not None:
        stats["gen_ms"] = gen_ms
        stats["zmws_local"] = n_local
    if rank != 0:
        return None
    t0 = time.perf_counter()
    if coll is not None:
        with lock:
            pending.update(x for x in range(high[0], len(chunks)) if x not in mine)
        final.set()
        coll.join()
        if collector_err:
            raise collector_err[0]
    if stats is not None:
        stats.update({"chunks": len(chunks), "chunks_by_rank": taken, "tail_ms": (time.perf_counter() - t0) * 1e3})
    missing = [i for i, rec in enumerate(out) if rec is None]
    if missing:
        raise RuntimeError(f"ZMWs missing after the queue drained: {missing[:8]}")
    return out


def polish_sharded(zmws, settings=None, engine=None, rank=None, world=None, polish_fn=None, group=None):
    """Polish `zmws` across the ranks of the default process group; rank 0 returns every ZMW's result in
    input order, the other ranks return None.  `polish_fn(list_of_zmws) -> list_of_results` defaults to this
    rank's HIP engine (pbccs_amd.polish_zmws)."""
    import torch.distributed as dist
    if rank is None:
        rank = dist.get_rank() if dist.is_initialized() else 0
    if world is None:
        world = dist.get_world_size() if dist.is_initialized() else 1
    plan = shard_plan([zmw_cost(z) for z in zmws], world)
    mine = plan[rank]
    if polish_fn is None:
        from . import polish_zmws

        def polish_fn(zs):
            return polish_zmws(zs, settings, engine)
    local = polish_fn([zmws[i] for i in mine]) if mine else []
    return gather_in_order(local, mine, len(zmws), rank, world, group)
