"""RCCL on the one GPU a box has: tests/rccl_one_rank.py runs reticulum_amd.shard's
device-tensor branches in a one-rank "nccl" process group (init with
device_id, a key-table broadcast from HBM, the pipelined sharded call, a
grouped self send/recv of device tensors through shard._Posted).  The tokens it
made through the broadcast key set are checked against the C oracle here."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from oracle import ctoken

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_one_rank_rccl_broadcast_pipeline_and_self_p2p():
    import torch
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_one_rank.py")], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["backend"] == "nccl"
    assert res["table_equal"] and res["pipelined_equal"]
    # the same seeded inputs as the child: its tokens through the broadcast key set are the oracle's
    g = torch.Generator().manual_seed(11)
    keys = torch.randint(0, 256, (300, 64), dtype=torch.uint8, generator=g).numpy()
    n, L = 1000, 200
    pt = torch.randint(0, 256, (n, L), dtype=torch.uint8, generator=g).numpy()
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, generator=g).numpy()
    kidx = torch.randint(0, 300, (n,), dtype=torch.int32, generator=g).numpy()
    tl = 16 + 16 * (L // 16 + 1) + 32
    tok = np.frombuffer(bytes.fromhex(res["tokens"]), np.uint8).reshape(n, tl)
    for i in range(0, n, 7):
        assert tok[i].tobytes() == ctoken.encrypt(keys[kidx[i]].tobytes(), iv[i].tobytes(), pt[i].tobytes()), i
    # a self send/recv may be refused by torch/RCCL; anything else is a failure
    assert res["self_p2p"] == "ok" or res["self_p2p"].startswith("refused"), res["self_p2p"]
    print("self send/recv:", res["self_p2p"])
