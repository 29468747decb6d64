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
    """The pull queue's work items: ZMW indices in decreasing cost, cut into chunks of `chunk` ZMWs (largest
    first, so the ranks' last pulls are the cheap chunks)."""
    order = sorted(range(len(zmws)), key=lambda i: (-zmw_cost(zmws[i]), i))
    return [order[k:k + chunk] for k in range(0, len(order), chunk)]


def polish_dynamic(zmws, settings=None, engine=None, rank=None, world=None, chunk=256, polish_fn=None, store=None,
                   group=None, stats=None):
    """Polish `zmws` across ranks through a dynamic pull queue: every rank takes the next
    chunk index from one shared counter -- an atomic fetch-add on the rank-0 key-value store, host-side, not a
    device collective -- until the queue is empty, so a rank that drew slow ZMWs (tall bands, long templates)
    simply pulls fewer chunks.

    Results stream to rank 0 as chunks finish (the ordered FIFO of WorkQueue.h:128-167 fed as workers
    complete): a rank > 0 puts each finished chunk's records under its own key on the same store; rank 0 takes
    whatever has arrived between its own chunks, and once the queue is empty only the chunks still running
    elsewhere are left to wait for.  Nothing is gathered in one piece at the end.  Rank 0 returns every ZMW's
    result in input order; the other ranks return None.  `stats` (a dict, optional) receives the queue's
    counters on rank 0: chunks per rank and `tail_ms`, the time from rank 0's last chunk to the last record."""
    import pickle
    import time
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
    out = [None] * len(zmws) if rank == 0 else None
    mine = []          # chunks this rank polished
    pending = set()    # rank 0: chunks another rank took, records not yet collected
    taken = [0] * world

    def collect(c, block):
        k = f"{key}/done/{c}"
        if not block and not store.check([k]):
            return False
        who, recs = pickle.loads(store.get(k))
        store.delete_key(k)
        taken[who] += 1
        for i, rec in zip(chunks[c], recs):
            out[i] = rec
        return True

    serial = 0
    high = 0           # rank 0: chunk indices below `high` were handed out
    while True:
        if world > 1:
            c = store.add(key, 1) - 1
        else:
            c, serial = serial, serial + 1
        if rank == 0:
            pending.update(range(high, min(c, len(chunks))))   # handed to other ranks since our last pull
            high = max(high, c + 1)
            for p in sorted(pending):
                if collect(p, block=False):
                    pending.discard(p)
        if c >= len(chunks):
            break
        recs = polish_fn([zmws[i] for i in chunks[c]])
        mine.append(c)
        if rank == 0:
            taken[0] += 1
            for i, rec in zip(chunks[c], recs):
                out[i] = rec
        else:
            store.set(f"{key}/done/{c}", pickle.dumps((rank, recs)))
    if rank != 0:
        return None
    t0 = time.perf_counter()
    pending.update(c for c in range(high, len(chunks)) if c not in mine)
    for p in sorted(pending):
        collect(p, block=True)   # store.get waits for the key
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
