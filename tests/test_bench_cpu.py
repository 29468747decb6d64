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
