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


def _stand_in(rank, pad=0):
    def polish(zs):
        return [{"rank": rank, "draft": z["draft"][::-1], "pad": "A" * pad} for z in zs]
    return polish


def _stand_in_held(rank, world, fast_chunks=4):
    """A stand-in whose schedule is fixed by store keys, not by timing: every rank's first chunk waits until every
    rank holds a chunk (so each rank takes at least one); rank 1's first chunk then also waits until rank 0 has
    finished `fast_chunks` chunks of its own (so rank 0, the fast rank, takes at least that many)."""
    import torch.distributed as dist
    store = dist.distributed_c10d._get_default_store()
    state = {"calls": 0}

    def polish(zs):
        state["calls"] += 1
        if state["calls"] == 1:
            if store.add("test/started", 1) == world:
                store.set("test/all_started", "1")
            store.wait(["test/all_started"])
            if rank == 1 and world == 2:   # (with more ranks the others may drain the queue before rank 0's fourth)
                store.wait(["test/fast_done"])
        out = [{"rank": rank, "draft": z["draft"][::-1], "pad": ""} for z in zs]
        if rank == 0 and state["calls"] == fast_chunks:
            store.set("test/fast_done", "1")
        return out
    return polish


def _stand_in_dies(rank, world):
    """Rank 1 fails in its first chunk; every rank's first chunk waits until each rank holds one (store keys), so
    rank 1 always gets a chunk to fail in (rank 0 cannot drain the queue first)."""
    import torch.distributed as dist
    store = dist.distributed_c10d._get_default_store()
    state = {"calls": 0}

    def polish(zs):
        state["calls"] += 1
        if state["calls"] == 1:
            if store.add("test/started", 1) == world:
                store.set("test/all_started", "1")
            store.wait(["test/all_started"])
        if rank == 1:
            raise RuntimeError("rank 1 fails mid-chunk")
        return [{"rank": rank, "draft": z["draft"][::-1], "pad": ""} for z in zs]
    return polish


def _worker(rank, world, port, zmws, out_q, use_gpu, mode="static", chunk=2):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if mode == "dead_peer":
            try:
                shard.polish_dynamic(zmws, chunk=chunk, polish_fn=_stand_in_dies(rank, world), collect_timeout=3.0)
                res = "no error"
            except RuntimeError as e:
                res = f"raised: {e}"
        elif mode in ("dynamic", "dynamic_big"):
            st = {}
            pad = (3 << 20) if mode == "dynamic_big" else 0   # 3 MB per record: chunks beyond the store's 8 MB values
            fn = None if use_gpu else (_stand_in(rank, pad=pad) if pad else _stand_in_held(rank, world))
            res = shard.polish_dynamic(zmws, chunk=chunk, polish_fn=fn, stats=st)
            if rank == 0:
                res = (res, st)
        elif use_gpu:
            res = shard.polish_sharded(zmws)
        else:
            res = shard.polish_sharded(zmws, polish_fn=_stand_in(rank))
        if rank == 0:
            out_q.put(res)
    finally:
        dist.destroy_process_group()


def _run(world, zmws, use_gpu=False, mode="static", chunk=2, ok_exit=(0,)):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, zmws, q, use_gpu, mode, chunk)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=600)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode in ok_exit
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
    # no chunk of more than one ZMW above 1 / ceil(23 / 4) of the total cost
    cap = sum(costs) / 6
    assert all(len(c) == 1 or sum(shard.zmw_cost(zmws[i]) for i in c) <= cap for c in chunks)


def test_gloo_world2_dynamic_queue_balances_and_keeps_order():
    """Rank 1 is slow -- its first chunk is held until rank 0 has finished four chunks (store keys, no timing) --
    so through the pull queue rank 0 takes more chunks, and the gathered records still come back in input order."""
    zmws = _toy_zmws(24)
    res, st = _run(2, zmws, mode="dynamic")
    assert [r["draft"] for r in res] == [z["draft"][::-1] for z in zmws]
    by_rank = [sum(1 for r in res if r["rank"] == k) for k in (0, 1)]
    assert by_rank[1] >= 1 and by_rank[0] >= 8, by_rank   # (rank 1's one chunk may hold one ZMW: cost-capped)
    # records streamed per chunk: rank 0 saw every chunk, the other rank's through the store
    n_ch = len(shard.dynamic_chunks(zmws, 2))   # 2 ZMWs per chunk at most, the costliest end cut finer
    assert st["chunks"] == n_ch and sum(st["chunks_by_rank"]) == n_ch and st["chunks_by_rank"][1] >= 1
    assert st["chunks_by_rank"][0] >= 4 and st["zmws_local"] == by_rank[0]


def test_gloo_world8_dynamic_queue_every_rank_pulls_and_order_holds():
    """Eight ranks (the node's eight GPUs) on one queue: every rank holds a chunk before any finishes (store keys),
    so all eight take work; the chunks come back complete and in input order."""
    zmws = _toy_zmws(128)
    res, st = _run(8, zmws, mode="dynamic")
    assert [r["draft"] for r in res] == [z["draft"][::-1] for z in zmws]
    n_ch = len(shard.dynamic_chunks(zmws, 2))
    assert n_ch >= 64 and st["chunks"] == n_ch and sum(st["chunks_by_rank"]) == n_ch and min(st["chunks_by_rank"]) >= 1
    assert {r["rank"] for r in res} == set(range(8))


def test_gloo_world2_dynamic_queue_raises_when_a_peer_dies():
    """A rank that fails mid-chunk never stores its records: rank 0 must raise once no record has arrived for the
    collect timeout, instead of waiting forever (bench.py's launcher is not the only caller)."""
    zmws = _toy_zmws(12)
    res = _run(2, zmws, mode="dead_peer", ok_exit=(0, 1))
    assert res.startswith("raised:") and "no record" in res, res


def test_gloo_world2_dynamic_queue_records_larger_than_a_store_value():
    """A chunk's records beyond the key-value store's 8 MB value limit (a 2500-ZMW chunk of a SMRT cell is ~55 MB)
    travel in parts and are reassembled in input order."""
    zmws = _toy_zmws(12)
    res, st = _run(2, zmws, mode="dynamic_big", chunk=4)
    assert [r["draft"] for r in res] == [z["draft"][::-1] for z in zmws]
    assert all(len(r["pad"]) == 3 << 20 for r in res)
    assert st["chunks_by_rank"][1] >= 1


@pytest.mark.gpu
def test_two_ranks_dynamic_queue_on_one_gpu_match_unsharded():
    import pbccs_amd
    from pbccs_amd import synth
    zmws = synth.make_zmws(8, 300, 5, seed=809)
    res, _ = _run(2, zmws, use_gpu=True, mode="dynamic")
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


@pytest.mark.gpu
def test_smrtcell_mix_two_ranks_dynamic_queue_match_oracle_and_fixtures():
    """configs[4] reduced: an SMRT-cell mix -- 12 ZMWs of 2 kb x 10 passes, the two 10 kb x 8-pass ZMWs of
    tests/golden/polish_10kb.json and the three configs[3] ZMWs of polish_mixed_long.json (15.2 kb x 21 passes,
    0.7 kb x 3, 4.8 kb x 14) -- shuffled, through shard.polish_dynamic on two ranks sharing cuda:0 (records
    streamed to rank 0 per chunk).  Every gathered record is checked against the oracle (2 kb) or the
    committed oracle fixtures (10 kb, mixed), not only against an unsharded run."""
    import json
    import random
    import sys
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    from pbccs_amd import synth
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    sys.path.insert(0, gold)
    from make_polish_fixtures import digest, mixed_long_zmws
    short = synth.make_zmws(12, 2000, 10, seed=4404)
    fx10 = json.load(open(os.path.join(gold, "polish_10kb.json")))["zmws"]
    fxm = json.load(open(os.path.join(gold, "polish_mixed_long.json")))["zmws"]
    long10, mixed = synth.make_zmws(2, 10000, 8, seed=82), mixed_long_zmws()
    cell = [("oracle", z, None) for z in short] + [("fx", z, e) for z, e in zip(long10 + mixed, fx10 + fxm)]
    for kind, z, e in cell:
        assert kind == "oracle" or digest(z) == e["digest"]
    random.Random(4).shuffle(cell)
    zmws = [z for _, z, _ in cell]
    (res, st) = _run(2, zmws, use_gpu=True, mode="dynamic", chunk=2)
    assert len(res) == len(cell) and sum(st["chunks_by_rank"]) == st["chunks"] and min(st["chunks_by_rank"]) >= 1
    O.lib()
    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        orc = list(ex.map(lambda z: O.polish_zmw(z["draft"], z["reads"], z["snr"]),
                          [z for k, z, _ in cell if k == "oracle"]))
    it = iter(orc)
    for (kind, z, e), r in zip(cell, res):
        if kind == "oracle":
            o = next(it)
            assert r["add_read_results"] == o["add_read_results"]
            assert (r["n_tested"], r["n_applied"]) == (o["n_tested"], o["n_applied"])
            if o["converged"]:
                assert r["consensus"] == o["template"]
                assert max(abs(a - b) for a, b in zip(r["qvs"], o["qvs"])) <= 1
            continue
        assert r["add_read_results"] == e["add_read_results"]
        stt = e["add_read_results"]
        if sum(1 for s in stt if s == 0) < 3:          # Consensus.h:473-490 gates before the polish
            assert r["status"] == "TooFewPasses"
            continue
        if sum(1 for s in stt if s != 0) / len(stt) > 0.34:
            assert r["status"] == "TooManyUnusable"
            continue
        assert (r["n_tested"], r["n_applied"]) == (e["n_tested"], e["n_applied"])
        if e["converged"]:
            assert r["consensus"] == e["consensus"]
            got = [min(max(q, 0), 93) for q in r["qvs"]]
            exp = [ord(c) - 33 for c in e["qvs"]]
            assert len(got) == len(exp) and max(abs(a - b) for a, b in zip(got, exp)) <= 1


def test_smrtcell_is_generated_per_zmw():
    """configs[4]'s lazy cell: ZMW i depends only on (seed, i) -- any rank materialises any chunk alone -- and the
    queue orders the cell by the shapes' cost estimate without generating a sequence."""
    from pbccs_amd import synth
    a, b = synth.SmrtCell(40, seed=9), synth.SmrtCell(400, seed=9)
    for i in (0, 17, 39):
        assert a[i] == b[i]
        kind, L, P, snr = a.shape(i)
        z = a[i]
        assert z["kind"] == synth.SmrtCell.KINDS[kind] and len(z["reads"]) == P and z["snr"] == list(snr)
        assert abs(len(z["draft"]) - L) <= 0.05 * L + 5
    kinds = [b.shape(i)[0] for i in range(400)]
    assert all(90 <= kinds.count(k) <= 180 for k in range(3))   # one third each
    chunks = shard.dynamic_chunks(b, 16)
    assert sorted(i for c in chunks for i in c) == list(range(400))
    costs = b.costs()
    flat = [i for c in chunks for i in c]
    assert [costs[i] for i in flat] == sorted(costs, reverse=True)


def test_gloo_world2_dynamic_queue_lazy_cell_keeps_order():
    """The dynamic queue over a lazily generated cell: each rank materialises only the chunks it pulls (the next
    one on a helper thread), rank 0's collector thread gathers the other rank's records, input order is kept."""
    from pbccs_amd import synth
    cell = synth.SmrtCell(12, seed=5)
    res, st = _run(2, cell, mode="dynamic", chunk=2)
    assert [r["draft"] for r in res] == [z["draft"][::-1] for z in cell]
    n_ch = len(shard.dynamic_chunks(cell, 2))
    assert n_ch >= 6 and st["chunks"] == n_ch and sum(st["chunks_by_rank"]) == n_ch and st["chunks_by_rank"][1] >= 1
    assert st["gen_ms"] >= 0.0
