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


def test_roofline_models_and_newest_profile():
    """The issue model and the measured compute core of the c2 kernels, and
    the choice of the newest committed PMC run by round tag (r02y < r02aa)."""
    sys.path.insert(0, ROOT)
    import bench
    m = bench.issue_model("encrypt", 1 << 20, 500, 1, 256, 1.0, 2.0)
    assert m["ceiling_cycles_per_simd"] > m["measured_core"]["cycles_per_simd"] > m["floor_cycles_per_simd"] > 0
    assert abs(m["measured_core"]["frac"] - m["measured_core"]["ms"] / 1.0) < 1e-12
    assert "pmc" not in m
    # issued slots from a PMC summary: VALU - dual-issue pairs + LDS, per SIMD
    pmc = {"SQ_INSTS_VALU": 4.2e8, "SQ_ACTIVE_INST_VALU2": 3.6e7, "SQ_INSTS_LDS": 1.2e8, "GRBM_GUI_ACTIVE": 1.6e7}
    p = bench.issue_model("encrypt", 1 << 20, 500, 1, 256, 1.0, 2.0, pmc)["pmc"]
    assert abs(p["issued_slots_per_simd"] - (4.2e8 - 3.6e7 + 1.2e8) / 1024) < 1e-6
    assert abs(p["dual_issued_frac_of_valu"] - 2 * 3.6e7 / 4.2e8) < 1e-12
    assert bench.issue_model("encrypt", 1 << 20, 100, 1, 256, 1.0, 2.0) is None   # c2 shape only
    path, d = bench._newest_pmc("encrypt", 1 << 20, 500, 1)
    assert path is not None and "encrypt" in d
    import glob
    import re
    cands = []
    for p in glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")):
        t = re.match(r"r(\d+)([a-z]+)_pmc\.json$", os.path.basename(p))
        with open(p) as f:
            w = json.load(f).get("_workload", {})
        if t and (w.get("packets"), w.get("length"), w.get("keys")) == (1 << 20, 500, 1):
            cands.append(((int(t.group(1)), len(t.group(2)), t.group(2)), p))
    assert path == max(cands)[1]


def test_cpu_openssl_row_without_library(tmp_path, monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))     # no tools/libcpu_openssl.so there
    assert bench.cpu_openssl(1.0, 1, 500) is None
    assert bench.cpu_openssl(0.0, 1, 500) is None
