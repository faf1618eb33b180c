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
    b, o, l, _ = shard.scatter_packed(tb, to, tl, bounds)
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
        gb, go, gl, _ = g
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


def _oracle_work(key):
    """Per-rank stand-in for the device kernels with sharded_call's contract:
    encrypt every packet of the shard under its IV row."""
    from oracle import ctoken

    def work(b, o, l, rows):
        (ivs,) = rows
        toks = [ctoken.encrypt(key, ivs[i].numpy().tobytes(), b[int(o[i]):int(o[i]) + int(l[i])].numpy().tobytes())
                for i in range(len(o))]
        lens = torch.tensor([len(t) for t in toks], dtype=torch.int32)
        offs = torch.zeros(len(toks), dtype=torch.int64)
        if len(toks) > 1:
            offs[1:] = torch.cumsum(lens[:-1].to(torch.int64), 0)
        out = torch.from_numpy(np.frombuffer(b"".join(toks), np.uint8).copy()) if toks else torch.zeros(0, torch.uint8)
        return out, offs, lens, [torch.zeros(len(toks), dtype=torch.int32)]
    return work


def _sharded_worker(rank, world, port, result_q):
    import torch.distributed as dist
    from oracle import ctoken
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    key = bytes(range(64))
    n = 257
    if rank == 0:
        rng = np.random.Generator(np.random.PCG64(78))
        lens = rng.integers(0, 2000, n).astype(np.uint32)          # numpy Packed dtypes: uint32 lengths ...
        off = np.zeros(n, np.uint64)                                 # ... and uint64 offsets
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
        buf = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
        ivs = rng.integers(0, 256, (n, 16), dtype=np.uint8)
        args = (torch.from_numpy(buf), torch.from_numpy(off.astype(np.int64)), torch.from_numpy(lens.astype(np.int64)))
        rows = [torch.from_numpy(ivs)]
    else:
        args, rows = (None, None, None), ()
    res, times = shard.sharded_call(_oracle_work(key), *args, rows=rows, row_specs=[(torch.uint8, 16)],
                                    balance=True)
    assert set(times) == {"scatter_s", "compute_s", "gather_s"}
    if rank == 0:
        gb, go, gl, (gst,) = res
        ok = len(gl) == n and gst.numel() == n and gl.dtype == torch.int32 and go.dtype == torch.int64
        for i in range(n):
            ref = ctoken.encrypt(key, ivs[i].tobytes(), buf[int(off[i]):int(off[i]) + int(lens[i])].tobytes())
            ok = ok and gb[int(go[i]):int(go[i]) + int(gl[i])].numpy().tobytes() == ref
        result_q.put(ok)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_call_gloo_world2():
    """shard.sharded_call — the entry bench.py's sharded configs (c4, c5) run
    over RCCL — end to end at world size 2 on gloo, the oracle standing in
    for the per-rank kernels: work-balanced partition, scatter of bytes +
    IV rows, gather of tokens + status rows, every token bit-exact."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get() is True


def test_slice_handles_unordered_offsets():
    buf = torch.arange(20, dtype=torch.uint8)
    off = torch.tensor([10, 0, 5], dtype=torch.int64)
    ln = torch.tensor([3, 4, 2], dtype=torch.int64)
    b, o, l = shard._slice(buf, off, ln, 0, 3)
    assert l.dtype == torch.int32 and o.dtype == torch.int64
    for i in range(3):
        assert b[int(o[i]):int(o[i]) + int(l[i])].tolist() == buf[int(off[i]):int(off[i]) + int(ln[i])].tolist()


def _keys_worker(rank, world, port, result_q):
    import torch.distributed as dist
    from oracle import ctoken
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    table = torch.from_numpy(np.random.Generator(np.random.PCG64(9)).integers(0, 256, (1000, 64), dtype=np.uint8))
    got = shard.broadcast_keys(table if rank == 0 else None, src=0)
    # every rank holds rank 0's table and its tokens under key 999 match the oracle's
    ok = got.dtype == torch.uint8 and tuple(got.shape) == (1000, 64) and torch.equal(got, table)
    iv = bytes(16)
    ok = ok and ctoken.encrypt(got[999].numpy().tobytes(), iv, b"x" * 33) == \
        ctoken.encrypt(table[999].numpy().tobytes(), iv, b"x" * 33)
    flags = torch.tensor([int(ok)], dtype=torch.int32)
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    if rank == 0:
        result_q.put(bool(flags[0]))
    dist.barrier()
    dist.destroy_process_group()


def test_broadcast_keys_gloo_world2():
    """The c3/c5 key table held by rank 0 reaches every rank (SURVEY §8(e):
    broadcast, then a per-rank key setup; device.keyset builds that on GPUs)."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_keys_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get() is True


def test_broadcast_keys_rejects_bad_tables():
    """A table that is not (n, 64 or 32) uint8 is refused on the source
    before any collective runs (world size 1, gloo)."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        for bad in (torch.zeros((4, 48), dtype=torch.uint8), torch.zeros((4, 64), dtype=torch.int32),
                    torch.zeros((0, 64), dtype=torch.uint8), torch.zeros(64, dtype=torch.uint8)):
            with pytest.raises(ValueError):
                shard.broadcast_keys(bad, src=0)
        assert torch.equal(shard.broadcast_keys(torch.ones((3, 32), dtype=torch.uint8), src=0),
                           torch.ones((3, 32), dtype=torch.uint8))
    finally:
        dist.destroy_process_group()


def _token_cap(lens):
    return 16 + 16 * (lens // 16 + 1) + 32


def _pipelined_worker(rank, world, port, result_q, chunks, balance):
    import torch.distributed as dist
    from oracle import ctoken
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    key = bytes(range(64))
    n = 203
    if rank == 0:
        rng = np.random.Generator(np.random.PCG64(79))
        lens = rng.integers(0, 1500, n).astype(np.int64)
        lens[5:9] = 0                                            # empty packets inside a chunk
        off = np.zeros(n, np.int64)
        off[1:] = np.cumsum(lens[:-1])
        buf = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
        ivs = rng.integers(0, 256, (n, 16), dtype=np.uint8)
        args = (torch.from_numpy(buf), torch.from_numpy(off), torch.from_numpy(lens))
        rows = [torch.from_numpy(ivs)]
    else:
        args, rows = (None, None, None), ()
    work = _oracle_work(key)
    serial, _ = shard.sharded_call(work, *args, rows=rows, row_specs=[(torch.uint8, 16)], balance=balance)
    piped, times = shard.sharded_call_pipelined(work, *args, rows=rows, row_specs=[(torch.uint8, 16)],
                                                out_cap=_token_cap, out_row_specs=[(torch.int32, 0)],
                                                chunks=chunks, balance=balance)
    assert set(times) == {"total_s", "chunks"} and times["chunks"] == chunks
    if rank == 0:
        sb, so, sl, (sst,) = serial
        pb, po, pl, (pst,) = piped
        ok = torch.equal(sb, pb) and torch.equal(so, po) and torch.equal(sl, pl) and torch.equal(sst, pst)
        ok = ok and pl.dtype == torch.int32 and po.dtype == torch.int64 and pl.numel() == n
        for i in range(n):
            ref = ctoken.encrypt(key, ivs[i].tobytes(), buf[int(off[i]):int(off[i]) + int(lens[i])].tobytes())
            ok = ok and pb[int(po[i]):int(po[i]) + int(pl[i])].numpy().tobytes() == ref
        result_q.put(ok)
    else:
        assert piped is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,chunks,balance", [(2, 4, True), (2, 1, False), (3, 5, False), (3, 3, True)])
def test_sharded_call_pipelined_equals_serial_gloo(world, chunks, balance):
    """the chunk-pipelined scatter -> compute -> gather
     returns exactly what the serial sharded_call returns, and
    every token is the oracle's, at world sizes 2 and 3, with more chunks
    than some ranks have packets' worth of work and empty packets."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_pipelined_worker, args=(r, world, port, q, chunks, balance)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get() is True


def test_slice_compacts_gapped_offsets():
    """a range whose byte span holds other packets' bytes (or
    gaps) sends only its own packets' bytes, compacted in packet order."""
    buf = torch.arange(100, dtype=torch.uint8)
    off = torch.tensor([80, 0, 40], dtype=torch.int64)
    ln = torch.tensor([5, 3, 0], dtype=torch.int64)
    b, o, l = shard._slice(buf, off, ln, 0, 3)
    assert b.numel() == 8 and o.tolist() == [0, 5, 8] and l.tolist() == [5, 3, 0]
    assert b.tolist() == list(range(80, 85)) + [0, 1, 2]
    # contiguous ranges stay views of the caller's buffer
    b2, o2, _ = shard._slice(buf, torch.tensor([10, 13]), torch.tensor([3, 4]), 0, 2)
    assert b2.data_ptr() == buf[10:].data_ptr() and o2.tolist() == [0, 3]


def _refuse_worker(rank, world, port, result_q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shard.broadcast_keys(torch.zeros((4, 48), dtype=torch.uint8) if rank == 0 else None, src=0)
        result_q.put((rank, "no error"))
    except ValueError as e:
        result_q.put((rank, str(e)))
    dist.destroy_process_group()


def test_broadcast_keys_refusal_raises_on_every_rank():
    """a table refused on the source makes every rank raise
    (no rank is left waiting in the next broadcast)."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_refuse_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = dict(q.get() for _ in range(2))
    assert "uint8 table" in got[0] and "refused" in got[1]
