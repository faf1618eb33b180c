"""Sharding across ranks (one process per GPU in production): partition,
scatter, per-rank compute, gather — exercised with the gloo backend on CPU at
world_size 2 and 3.  The per-rank compute here is the C oracle (the checker);
on GPUs it is the HIP kernel (bench.py, test_token_gpu.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from reticulum_amd import shard


def test_partition_by_count():
    assert shard.partition(10, 3) == [(0, 4), (4, 7), (7, 10)]
    assert shard.partition(2, 4) == [(0, 1), (1, 2), (2, 2), (2, 2)]


def test_partition_by_work_is_balanced_and_covers():
    rng = np.random.Generator(np.random.PCG64(5))
    lens = torch.from_numpy(rng.integers(64, 4097, 10000).astype(np.int32))
    b = shard.partition(10000, 8, lens)
    assert b[0][0] == 0 and b[-1][1] == 10000
    assert all(b[i][1] == b[i + 1][0] for i in range(7))
    w = shard.work_per_packet(lens)
    loads = [int(w[lo:hi].sum()) for lo, hi in b]
    assert max(loads) / (sum(loads) / 8) < 1.01


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, result_q):
    import torch.distributed as dist
    from oracle import ctoken
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    key = bytes(range(64))
    if rank == 0:
        rng = np.random.Generator(np.random.PCG64(77))
        lens = rng.integers(0, 700, 301).astype(np.int32)
        off = np.zeros(301, np.int64)
        off[1:] = np.cumsum(lens[:-1])
        buf = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
        ivs = rng.integers(0, 256, (301, 16), dtype=np.uint8)
        tb, to, tl = torch.from_numpy(buf), torch.from_numpy(off), torch.from_numpy(lens)
        bounds = shard.partition(301, world, tl)
    else:
        tb = to = tl = None
        bounds = None
    obj = [bounds]
    dist.broadcast_object_list(obj, 0)
    bounds = obj[0]
    b, o, l = shard.scatter_packed(tb, to, tl, bounds)
    # per-rank compute: one token per packet (IV = packet index bytes, deterministic)
    lo, hi = bounds[rank]
    toks = []
    for i in range(len(o)):
        pt = b[int(o[i]):int(o[i]) + int(l[i])].numpy().tobytes()
        iv = (lo + i).to_bytes(16, "little")
        toks.append(ctoken.encrypt(key, iv, pt))
    lens_out = torch.tensor([len(t) for t in toks], dtype=torch.int32)
    offs_out = torch.zeros(len(toks), dtype=torch.int64)
    if len(toks) > 1:
        offs_out[1:] = torch.cumsum(lens_out[:-1].to(torch.int64), 0)
    bout = torch.from_numpy(np.frombuffer(b"".join(toks), np.uint8).copy()) if toks else torch.zeros(0, dtype=torch.uint8)
    g = shard.gather_packed(bout, offs_out, lens_out)
    if rank == 0:
        gb, go, gl = g
        ok = len(gl) == 301
        for i in range(301):
            pt = buf[off[i]:off[i] + lens[i]].tobytes()
            ref = ctoken.encrypt(key, i.to_bytes(16, "little"), pt)
            got = gb[int(go[i]):int(go[i]) + int(gl[i])].numpy().tobytes()
            ok = ok and got == ref
        result_q.put(ok)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_scatter_compute_gather_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get() is True
