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


def _cpu_phase_worker(rank, world, port, q):
    import argparse
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    import bench
    import time
    line = {"value": 1.0, "cpu_baseline": None, "cpu_openssl": None}
    t0 = time.perf_counter()
    bench._cpu_phase(line, argparse.Namespace(cpu_seconds=0.5, cpu_workers=2), 500, rank)
    q.put((rank, line["cpu_baseline"], time.perf_counter() - t0))
    dist.destroy_process_group()


def test_cpu_baseline_phase_at_n_gt_1():
    """at N > 1 rank 0 times the CPU baseline after the
    GPU phases while the other ranks wait on the rendezvous store; every
    rank leaves only when rank 0 is done, and the line carries the baseline."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_cpu_phase_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = {r: (cpu, dt) for r, cpu, dt in (q.get() for _ in range(2))}
    cpu0 = got[0][0]
    assert cpu0["kind"] == "port" and cpu0["value"] > 0 and cpu0["cores"] == 2 and "rank 0" in cpu0["note"]
    assert got[1][0] is None and got[1][1] >= 0.5          # rank 1 waited for rank 0's timed phase


def test_guard_names_its_phase():
    """The host-origin pass of an N > 1 run has its own deadline: on expiry
    the line carries the error under e2e_pcie, the headline intact."""
    p = _run("import bench, time\n"
             "line = {'metric': 'm', 'value': 3.0, 'e2e_pcie': None, 'sharded_c4': None}\n"
             "g = bench._LineGuard(line, 0.3, field='e2e_pcie', what='host-origin pass')\n"
             "time.sleep(20)\n")
    assert p.returncode == 0, p.stderr
    rec = json.loads(p.stdout.strip())
    assert rec["value"] == 3.0 and rec["sharded_c4"] is None
    assert rec["e2e_pcie"]["error"] == "host-origin pass unfinished after 0.3 s"


def test_committed_n_gt_1_lines_carry_every_north_star_number():
    """VERDICT r02 next #2, checked on the committed rehearsal lines of
    bench.py's N > 1 path (RNSTOK_BENCH_REHEARSE=1: every rank on one GPU over
    gloo, 2 and 4 ranks; not measurements): the weak-scaling headline, the
    node's host-origin aggregate, the CPU baseline timed in the same run, and
    the sharded c4 pass with its serial legs and the pipelined pass, whose
    output equals the serial pass's."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r03*_rehearse_n*_gloo.json")))
    assert len(paths) >= 2
    for p in paths:
        with open(p) as f:
            rec = json.loads(f.read().strip().splitlines()[-1])
        n = rec["n_gpus"]
        assert n >= 2 and rec["value"] > 0 and rec["scaling"] == "weak"
        agg = rec["e2e_pcie"]["aggregate"]
        assert agg["ranks"] == n
        legs = ("serial", "pipelined") + (("pipelined_copy_engine",) if "pipelined_copy_engine" in agg else ())
        for leg in legs:
            assert agg[leg]["ok_all"] is True and agg[leg]["encrypt_packets_s"] > 0 and agg[leg]["decrypt_packets_s"] > 0
        cpu = rec["cpu_baseline"]
        assert cpu["kind"] == "port" and cpu["value"] > 0 and cpu["cores"] >= 1
        sc = rec["sharded_c4"]
        assert sc["ok"] is True and sc["n_gpus"] == n
        # from round 3's r03m on, c4 runs both directions
        names = ["encrypt"] + (["decrypt"] if "decrypt" in sc["config"]["workload"] else [])
        for name in names:
            ph = sc["phases"][name]
            assert min(ph["scatter_ms"], ph["compute_ms"], ph["gather_ms"], ph["pipelined_ms"]) > 0
            assert ph["pipelined_equals_serial"] is True and ph["pipelined_chunks"] >= 1


def test_ceiling_fracs_and_calibrated_traffic():
    """Round 6: the bench line's ceiling fractions (canonical lane-ops over the
    ISA slot floor at two wave64 instructions per slot) and the decrypt's
    traffic from FETCH_SIZE scaled by its own read pattern's calibration."""
    sys.path.insert(0, ROOT)
    import bench
    c = bench.ceiling_fracs("decrypt", 500, 1, 0.40)
    ops = 64 * bench.ops_dec(500)
    floor = bench.SLOTS_PER_WAVE_PACKET_500B["decrypt"]["floor"]
    assert abs(c["ceiling_frac"] - ops / (floor * 128)) < 1e-12
    assert 0.45 < c["ceiling_frac"] < 0.52 and 0.6 < c["ceiling_frac_valu_only"] < 0.72
    assert abs(c["frac_over_ceiling"] - 0.40 / c["ceiling_frac"]) < 1e-12
    assert bench.ceiling_fracs("decrypt", 383, 1, 0.4)["ceiling_frac"] is None        # c2 shape only
    t = bench.traffic_from_profiles("decrypt", 1 << 20, 500, 1, "rows")
    k, _ = bench.FETCH_CALIBRATION[("decrypt", "rows")]
    path, d = bench._newest_pmc("decrypt", 1 << 20, 500, 1)
    m = d["decrypt"]
    assert abs(t["bytes_calibrated"] - (k * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024) < 1.0
    assert t["bytes_calibrated"] < t["bytes_with_x2_fetch_correction"]
    assert bench.traffic_from_profiles("encrypt", 1 << 20, 500, 1, "rows")["bytes_calibrated"] is None
