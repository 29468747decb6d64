"""Multi-GPU sharding (pbccs_amd/shard.py): the static cost-balanced plan and the dynamic pull queue, both
with the ordered gather.  CPU tests run the N > 1 paths with the gloo backend at world size 2 (a stand-in
polish function: no GPU); the GPU tests run two ranks on cuda:0 through the HIP engine and check the
gathered results against an unsharded polish."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from pbccs_amd import shard


def test_plan_partitions_and_balances():
    costs = [5, 1, 9, 3, 3, 7, 2, 8, 4, 6]
    plan = shard.shard_plan(costs, 3)
    flat = sorted(i for p in plan for i in p)
    assert flat == list(range(len(costs)))
    loads = [sum(costs[i] for i in p) for p in plan]
    assert max(loads) - min(loads) <= max(costs)
    assert plan == shard.shard_plan(costs, 3)   # deterministic: every rank computes the same plan
    assert shard.shard_plan(costs, 1) == [list(range(len(costs)))]
    assert shard.shard_plan([], 2) == [[], []]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stand_in(rank, slow_rank=None):
    import time

    def polish(zs):
        if rank == slow_rank:
            time.sleep(0.05 * len(zs))
        return [{"rank": rank, "draft": z["draft"][::-1]} for z in zs]
    return polish


def _worker(rank, world, port, zmws, out_q, use_gpu, mode="static"):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if mode == "dynamic":
            res = shard.polish_dynamic(zmws, chunk=2, polish_fn=None if use_gpu else _stand_in(rank, slow_rank=1))
        elif use_gpu:
            res = shard.polish_sharded(zmws)
        else:
            res = shard.polish_sharded(zmws, polish_fn=_stand_in(rank))
        if rank == 0:
            out_q.put(res)
    finally:
        dist.destroy_process_group()


def _run(world, zmws, use_gpu=False, mode="static"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, zmws, q, use_gpu, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _toy_zmws(n):
    import random
    rng = random.Random(7)
    out = []
    for i in range(n):
        L = rng.randint(20, 200)
        draft = "".join(rng.choice("ACGT") for _ in range(L))
        out.append({"draft": draft, "snr": [10, 7, 5, 11], "reads": [{"seq": draft}] * rng.randint(1, 6)})
    return out


def test_gloo_world2_gathers_in_input_order():
    zmws = _toy_zmws(23)
    res = _run(2, zmws)
    assert [r["draft"] for r in res] == [z["draft"][::-1] for z in zmws]
    assert {r["rank"] for r in res} == {0, 1}   # both ranks did work


def test_dynamic_chunks_are_a_cost_ordered_partition():
    zmws = _toy_zmws(23)
    chunks = shard.dynamic_chunks(zmws, 4)
    flat = [i for c in chunks for i in c]
    assert sorted(flat) == list(range(23)) and all(len(c) <= 4 for c in chunks)
    costs = [shard.zmw_cost(zmws[i]) for i in flat]
    assert costs == sorted(costs, reverse=True)


def test_gloo_world2_dynamic_queue_balances_and_keeps_order():
    """Rank 1 is slow (its stand-in sleeps per ZMW): through the pull queue rank 0 takes more chunks, and
    the gathered records still come back in input order."""
    zmws = _toy_zmws(24)
    res = _run(2, zmws, mode="dynamic")
    assert [r["draft"] for r in res] == [z["draft"][::-1] for z in zmws]
    by_rank = [sum(1 for r in res if r["rank"] == k) for k in (0, 1)]
    assert by_rank[1] >= 2 and by_rank[0] > by_rank[1], by_rank


@pytest.mark.gpu
def test_two_ranks_dynamic_queue_on_one_gpu_match_unsharded():
    import pbccs_amd
    from pbccs_amd import synth
    zmws = synth.make_zmws(8, 300, 5, seed=809)
    res = _run(2, zmws, use_gpu=True, mode="dynamic")
    ref = pbccs_amd.polish_zmws(zmws)
    for a, b in zip(res, ref):
        assert (a["consensus"], a["n_tested"], a["n_applied"], a["status"]) == \
               (b["consensus"], b["n_tested"], b["n_applied"], b["status"])


@pytest.mark.gpu
def test_two_ranks_on_one_gpu_match_unsharded():
    import pbccs_amd
    from pbccs_amd import synth
    zmws = synth.make_zmws(8, 300, 5, seed=808)
    res = _run(2, zmws, use_gpu=True)
    ref = pbccs_amd.polish_zmws(zmws)
    for a, b in zip(res, ref):
        assert (a["consensus"], a["n_tested"], a["n_applied"], a["status"]) == \
               (b["consensus"], b["n_tested"], b["n_applied"], b["status"])
