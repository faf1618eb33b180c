"""bench.py host logic that needs no GPU: the deadline guard of the optional
sharded pass in N > 1 runs (the headline line must still be printed, once,
and every rank must leave with status 0 when that pass hangs)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(code):
    return subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=60)


def test_guard_expiry_prints_line_once_and_exits_zero():
    p = _run("import bench, time\n"
             "line = {'metric': 'm', 'value': 1.0, 'sharded_c4': None}\n"
             "g = bench._LineGuard(line, 0.3)\n"
             "line['sharded_c4'] = {'phases': 'half done'}\n"
             "time.sleep(20)\n"
             "print('not reached')\n")
    assert p.returncode == 0, p.stderr
    out = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(out) == 1, p.stdout
    rec = json.loads(out[0])
    assert rec["value"] == 1.0
    assert "unfinished" in rec["sharded_c4"]["error"]
    assert rec["sharded_c4"]["partial"] == {"phases": "half done"}


def test_guard_other_ranks_exit_silently():
    p = _run("import bench, time\n"
             "g = bench._LineGuard(None, 0.3)\n"
             "time.sleep(20)\n")
    assert p.returncode == 0 and p.stdout.strip() == ""


def test_guard_finish_cancels():
    p = _run("import bench, time\n"
             "g = bench._LineGuard({'value': 2}, 0.5)\n"
             "g.finish()\n"
             "time.sleep(1.0)\n"
             "print('done')\n")
    assert p.returncode == 0 and p.stdout.strip() == "done"
