"""bench.py's own code paths on one GPU, at small sizes: the headline step's
correctness gate runs inside bench.main at full size on every bench run; here
the sharded configs (c4, c5: shard.sharded_call's per-rank work on the device)
run end to end at world size 1 and must report a verified round trip."""
import argparse

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg, packets", [("c4", 1000), ("c5", 20_000)])
def test_sharded_config_world1(cfg, packets):
    import bench
    args = argparse.Namespace(packets=packets)
    rep = bench.sharded_bench(cfg, args, world=1, rank=0, local=0, reps=1)
    assert rep["ok"] is True
    assert rep["config"]["packets"] == packets
    assert set(rep["phases"]) == {"encrypt", "decrypt"}
    # c4: every segment encrypted, then its token decrypted;
    # c5: half and half
    per = packets if cfg == "c4" else packets // 2
    assert rep["phases"]["encrypt"]["packets"] == per
    assert rep["phases"]["decrypt"]["packets"] == packets - (0 if cfg == "c4" else per)
    assert rep["value"] > 0 and rep["compute_ms"] > 0
    assert rep["roofline"]["bound"] == "valu" and 0 < rep["roofline"]["frac"] < 1


def test_c3_key_setup_times():
    """the per-key setup timed apart from the steps, from a
    host table and from a table already in HBM."""
    import numpy as np
    import torch
    import bench
    keys = np.random.default_rng(3).integers(0, 256, (4096, 64), dtype=np.uint8)
    r = bench.key_setup_times(keys, 0, torch.device("cuda", 0), reps=2)
    assert r["keys"] == 4096 and r["host_ms"] > 0 and r["device_ms"] > 0 and r["keys_per_s_device"] > 0


def test_node_rate_small():
    """bench.node_rate (the composed interface path in the bench line) at a
    small size: both directions timed, every packet back."""
    import torch
    import bench
    r = bench.node_rate(torch.device("cuda", 0), steps=3, n=4096)
    assert r["ok"] is True and r["packets"] == 4096
    assert r["outbound"]["ms"] > 0 and r["inbound"]["ms"] > 0 and r["stream_bytes"] > 4096 * 467


def test_shard_rate_small():
    """bench.shard_rate (the c4 8-GPU per-rank shape in the bench line) at a
    small per-CU count: long-token kernels, every token back."""
    import torch
    import bench
    r = bench.shard_rate(torch.device("cuda", 0), 8, steps=3, L=4096, per_cu=16)
    assert r["ok"] is True and r["tokens"] == 128
    assert r["encrypt"]["ms"] > 0 and r["decrypt"]["ms"] > 0 and 0 < r["encrypt"]["frac_of_valu_peak"] < 1


def test_c3_rate_small():
    """bench.c3_rate (the per-key c3 leg of the bench line) at a small size:
    both directions timed, every packet back."""
    import torch
    import bench
    r = bench.c3_rate(torch.device("cuda", 0), 8, n=8192, n_keys=97, steps=3)
    assert r["ok"] is True and r["packets"] == 8192
    assert r["encrypt"]["ms"] > 0 and r["decrypt"]["ms"] > 0 and r["round_trips_s"] > 0


def test_node_host_rate_small():
    """bench.node_host_rate (the composed interface path host-origin, in the
    bench line) at a small size: both directions timed through pinned host
    buffers, every slice's stream, every status and a sample of plaintexts
    checked on the host copies."""
    import torch
    import bench
    r = bench.node_host_rate(torch.device("cuda", 0), n=8192, slices=4, reps=1)
    assert r["ok"] is True and r["packets"] == 8192
    assert r["outbound"]["ms"] > 0 and r["inbound"]["ms"] > 0
