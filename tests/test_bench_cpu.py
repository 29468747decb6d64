"""bench.py host logic on CPU: the driver parses the bench's stdout as its one JSON line, so a multi-rank run
must keep library chatter (gloo's connection report) off fd 1 -- quiet_stdout() points fd 1 at stderr and
emit() writes the line to the saved stdout."""
import json
import os
import subprocess
import sys
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_multi_rank_stdout_is_the_json_line_only():
    code = (
        "import os, sys; sys.path.insert(0, %r); import bench\n"
        "bench.quiet_stdout()\n"
        "print('chatter from a library', flush=True)\n"
        "os.write(1, b'raw fd-1 chatter\\n')\n"
        "bench.emit({'metric': 'm', 'value': 1.5})\n" % ROOT)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    lines = p.stdout.splitlines()
    assert len(lines) == 1 and json.loads(lines[0]) == {"metric": "m", "value": 1.5}
    assert "chatter from a library" in p.stderr and "raw fd-1 chatter" in p.stderr


def test_single_rank_emit_goes_to_stdout():
    code = "import sys; sys.path.insert(0, %r); import bench; bench.emit({'value': 2})\n" % ROOT
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert json.loads(p.stdout) == {"value": 2}


def test_roofline_marks_time_shared_launches_and_single_slot_figure(tmp_path, monkeypatch):
    """make_roofline prices the dominant kernel per launch; with launches overlapping (device time > wall time)
    the figure is flagged time_shared, and the single-slot profile of the same sources supplies the
    non-overlapped per-launch figure (a stale one is named as such)."""
    sys.path.insert(0, ROOT)
    import bench
    stats = {"k_fill_tall": {"device_ms": 3000.0, "launches": 30, "bytes": 30 * 6e9, "cells": 30 * 7e8},
             "k_score": {"device_ms": 1000.0, "launches": 10, "bytes": 1e9, "cells": 1e9}}
    prof = tmp_path / "profiles"
    prof.mkdir()
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "kernel_source_digest", lambda: "abc")
    r = bench.make_roofline(stats, 1.5, "w")
    assert r["kernel"] == "k_fill_tall" and r["time_shared"] and r["in_flight"] == 2.0
    assert r["single_slot"] is None and r["traffic"] is None
    assert abs(r["achieved"] - 6e9 / 0.1 / 1e9) < 1e-6
    single = {"roofline": {"kernel": "k_fill_tall", "source_digest": "abc", "frac": 0.0123, "achieved": 98.4,
                           "avg_launch_ms": 61.0, "in_flight": 0.6}}
    (prof / bench.SINGLE_SLOT_PROFILE).write_text(json.dumps(single))
    r = bench.make_roofline(stats, 1.5, "w")
    assert r["single_slot"]["frac"] == 0.0123 and r["single_slot"]["avg_launch_ms"] == 61.0
    single["roofline"]["source_digest"] = "old"
    (prof / bench.SINGLE_SLOT_PROFILE).write_text(json.dumps(single))
    r = bench.make_roofline(stats, 1.5, "w")
    assert "stale" in r["single_slot"]["source"] and "frac" not in r["single_slot"]


def _args(**kw):
    import argparse
    d = dict(cpu_sample=4, cpu_threads=2, seed=1, workload="2kb")
    d.update(kw)
    return argparse.Namespace(**d)


def test_sample_indices_stride_and_capped_random_sample():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.sample_indices(_args(cpu_sample=4), 40) == [0, 10, 20, 30]
    assert bench.sample_indices(_args(cpu_sample=64), 10) == list(range(10))
    costs = [1e8] * 10 + [5e9] * 10   # the second half is costlier than a 10 kb / 8-pass ZMW
    idx = bench.sample_indices(_args(cpu_sample=6), 20, costs)
    assert len(idx) == 6 and idx == sorted(idx) and all(i < 10 for i in idx)
    assert idx == bench.sample_indices(_args(cpu_sample=6), 20, costs)   # seeded
    cov = bench.coverage(costs)
    assert cov["eligible_zmws_frac"] == 0.5 and abs(cov["eligible_cost_frac"] - 1e9 / 51e9) < 1e-4


def test_cpu_leg_checks_the_timed_records_and_fails_on_a_mismatch():
    """The CPU leg polishes the sampled ZMWs on the restatement and compares them with the run's records: equal
    records pass; one consensus edited, one nTested changed and one QV moved by 2 each fail that ZMW.  With a
    cost model the rate is the ratio estimator's (the sample's CPU seconds per unit of cost x the mean cost)."""
    sys.path.insert(0, ROOT)
    import copy
    import bench
    import pbccs_amd
    from pbccs_amd import synth
    settings = pbccs_amd.ConsensusSettings()
    zs = synth.make_zmws(6, 200, 5, seed=5)
    recs = [bench.oracle_record(z, settings) for z in zs]
    assert all(r["status"] in ("Success", "PoorQuality", "NonConvergent", "TooFewPasses", "TooManyUnusable")
               for r in recs)
    idx = [0, 2, 4]
    cb, par = bench.sampled_cpu_baseline(_args(cpu_sample=3), settings, zs, recs, idx)
    assert par["ok"] and par["n"] == 3 and par["consensus_equal"] == 3 and par["max_qv_diff"] == 0
    assert cb["value"] > 0 and cb["cores"] == 2 and cb["full_host_value"] >= cb["value"]
    bad = copy.deepcopy(recs)
    ok = [i for i in idx if recs[i]["status"] == "Success"]
    assert ok, [r["status"] for r in recs]
    bad[ok[0]]["consensus"] = bad[ok[0]]["consensus"][:-1]
    bad[ok[-1]]["qvs"] = [q + 2 for q in bad[ok[-1]]["qvs"]]
    _, par = bench.sampled_cpu_baseline(_args(cpu_sample=3), settings, zs, bad, idx)
    assert not par["ok"] and ok[0] in par["mismatched_zmws"] and ok[-1] in par["mismatched_zmws"]
    costs = [bench.zmw_cost(z) for z in zs]
    cb, par = bench.sampled_cpu_baseline(_args(cpu_sample=3), settings, zs, recs, idx, costs)
    ex = cb["extrapolated"]
    assert par["ok"] and abs(cb["value"] - 2 / ex["core_s_per_zmw"]) < 0.02 * cb["value"]


def test_occupancy_report_from_wave_stamps():
    """roofline.occupancy: resident waves = wave-seconds / wall; the VGPR share uses the build's resource table
    (allocation rounded up to 8 registers) over 1024 SIMDs x 512."""
    import json
    import os
    import bench
    table = os.path.join(bench.ROOT, "pbccs_amd", "_lib", "kernel_resources.json")
    if not os.path.exists(table):
        pytest.skip("library not built")
    res = json.load(open(table))
    fill = [v for k, v in res.items() if "k_fill_coopILi16E" in k][0]
    alloc = (fill["vgprs"] + fill["agprs"] + 7) // 8 * 8
    occ = bench.occupancy_report({"k_fill": {"wave_s": 2048.0, "launches": 4}}, 2.0)
    assert bench.occupancy_report({"k_fill": {"wave_s": 0.0, "launches": 4}}, 2.0) is None
    assert occ["resident_waves"] == 1024.0 and occ["waves_per_simd"] == 1.0
    assert occ["families"]["k_fill"]["vgprs_per_lane"] == alloc
    assert abs(occ["vgpr_file_frac"] - round(1024 * alloc / (1024 * 512), 4)) < 1e-9
    assert occ["wave_slot_frac"] == round(1 / 8, 4)


def test_cpu_leg_sample_is_stratified_and_the_power_law_recovers_its_exponent():
    """the heterogeneous workloads' CPU leg samples one ZMW per cost stratum of the eligible
    range (not a simple random sample that clusters on the cheap ZMWs), and the extrapolation fits CPU time as a
    power of the cost model instead of scaling linearly."""
    sys.path.insert(0, ROOT)
    import random
    import types
    import bench
    rng = random.Random(3)
    costs = [10 ** rng.uniform(6, 10) for _ in range(2000)]
    args = types.SimpleNamespace(cpu_sample=32, seed=3)
    idx = bench.sample_indices(args, len(costs), costs)
    assert len(idx) == 32 and len(set(idx)) == 32
    assert all(costs[i] <= bench.SAMPLE_COST_CAP for i in idx)
    elig = sorted(c for c in costs if c <= bench.SAMPLE_COST_CAP)
    picked = sorted(costs[i] for i in idx)
    # one per stratum: the k-th smallest pick lies in the k-th 1/32 of the eligible ZMWs by cost
    for k, c in enumerate(picked):
        lo, hi = len(elig) * k // 32, len(elig) * (k + 1) // 32
        assert elig[lo] <= c <= elig[hi - 1]
    secs = [2e-9 * costs[i] ** 1.3 for i in idx]
    a, alpha = bench.power_law_fit([costs[i] for i in idx], secs)
    assert abs(alpha - 1.3) < 1e-9
    assert bench.power_law_fit([1.0, 1.0, 1.0], [1.0, 2.0, 3.0]) is None
