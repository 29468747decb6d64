"""bench.py host logic on CPU: the driver parses the bench's stdout as its one JSON line, so a multi-rank run
must keep library chatter (gloo's connection report) off fd 1 -- quiet_stdout() points fd 1 at stderr and
emit() writes the line to the saved stdout."""
import json
import os
import subprocess
import sys

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
