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
    assert set(rep["phases"]) == ({"encrypt"} if cfg == "c4" else {"encrypt", "decrypt"})
    assert rep["value"] > 0 and rep["compute_ms"] > 0
