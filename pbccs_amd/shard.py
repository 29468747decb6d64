"""Multi-GPU ccs polish: ZMWs shard across ranks (one process per GPU), results gather in input order.

ZMWs are independent, so the data path has no collective: each rank polishes its own
shard on its own GPU, and only the finished per-ZMW records travel, once, to rank 0, which reassembles
them in input order -- the ordering contract of pbccs' writer FIFO (include/pacbio/ccs/WorkQueue.h:128-167).
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
                   group=None):
    """Polish `zmws` across ranks through a dynamic pull queue: every rank takes the next
    chunk index from one shared counter -- an atomic fetch-add on the rank-0 key-value store, host-side, not a
    device collective -- until the queue is empty, so a rank that drew slow ZMWs (tall bands, long templates)
    simply pulls fewer chunks.  Rank 0 returns every ZMW's result in input order (one ordered gather, as
    WorkQueue.h:128-167); the other ranks return None."""
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
    mine, local = [], []
    serial = 0
    while True:
        if world > 1:
            c = store.add(key, 1) - 1
        else:
            c, serial = serial, serial + 1
        if c >= len(chunks):
            break
        idx = chunks[c]
        local.extend(polish_fn([zmws[i] for i in idx]))
        mine.extend(idx)
    return gather_in_order(local, mine, len(zmws), rank, world, group)


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
