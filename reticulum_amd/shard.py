"""One-process-per-GPU sharding of token batches.

Packets are independent, so a batch splits into contiguous packet ranges, one
per rank, with no exchange during compute.  The collective layer is used only
to move inputs and outputs:

* ``partition``      — contiguous ranges balanced by packet count, or by the
                       per-packet work (AES blocks + SHA-256 compressions) for
                       mixed-length batches (config c5);
* ``scatter_packed`` — root -> ranks: each rank receives its packets' bytes,
                       offsets (rebased) and lengths;
* ``gather_packed``  — the mirror: ranks -> root, reassembled in order.

With the ``nccl`` backend (RCCL on ROCm) the tensors live on each rank's GPU
and move over xGMI peer links as grouped point-to-point sends (RCCL has no
scatter primitive); with ``gloo`` the same code runs on CPU tensors, which is
how the multi-process tests exercise it.
"""
import torch
import torch.distributed as dist


def work_per_packet(lengths):
    """Relative cost of a packet of L bytes: AES blocks + SHA-256 compressions
    (352 and 1464 VALU ops each in the canonical model, bench.py)."""
    L = lengths.to(torch.int64)
    blocks = L // 16 + 1
    sha = (89 + 16 * blocks + 63) // 64
    return 352 * blocks + 1464 * sha


def partition(n, world, lengths=None):
    """Contiguous [lo, hi) packet ranges for each rank.  With ``lengths``,
    ranges are balanced by work_per_packet (prefix-sum split)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    if lengths is None:
        per, rem = divmod(n, world)
        bounds, lo = [], 0
        for r in range(world):
            hi = lo + per + (1 if r < rem else 0)
            bounds.append((lo, hi))
            lo = hi
        return bounds
    w = work_per_packet(torch.as_tensor(lengths).cpu())
    if w.numel() != n:
        raise ValueError("lengths must have n entries")
    csum = torch.cumsum(w, 0)
    total = int(csum[-1]) if n else 0
    cuts = [0]
    for r in range(1, world):
        target = total * r // world
        cuts.append(int(torch.searchsorted(csum, torch.tensor(target), right=True)))
    cuts.append(n)
    cuts = [min(max(c, cuts[i - 1] if i else 0), n) for i, c in enumerate(cuts)]
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def _slice(buf, off, length, lo, hi):
    """Bytes, rebased offsets and lengths of packets [lo, hi) of a packed
    batch.  Offsets need not ascend.  When the packets' bytes lie contiguous
    in the range's span (the usual packed batch) the slice is a view of that
    span; when the span holds more than the packets' own bytes (offsets out of
    order, gaps, other packets in between) the packets are gathered into a
    compact buffer, so only their own bytes cross the link."""
    if hi <= lo:
        return buf.new_zeros(0), off.new_zeros(0).to(torch.int64), length.new_zeros(0).to(torch.int32)
    o = off[lo:hi].to(torch.int64)
    ln = length[lo:hi].to(torch.int64)
    start = int(o.min())
    end = int((o + ln).max())
    total = int(ln.sum())
    if end - start <= total:
        return buf[start:end], o - start, ln.to(torch.int32)
    dst = torch.cumsum(ln, 0) - ln                         # compact offsets, packet order
    idx = torch.repeat_interleave(o - dst, ln) + torch.arange(total, device=o.device)
    return buf[idx.to(buf.device)], dst, ln.to(torch.int32)


def _staged(group):
    """gloo moves host tensors only: device tensors go through host copies
    (the one-GPU rehearsal of bench.py's N > 1 path).  RCCL/NCCL moves them
    directly over xGMI."""
    return dist.get_backend(group) == "gloo"


def _wait(ops, group=None):
    """Post (kind, tensor, peer) transfers as one grouped batch and wait."""
    if not ops:
        return
    stage = _staged(group)
    posted, copy_back = [], []
    for kind, t, peer in ops:
        if stage and t.is_cuda:
            h = t.cpu() if kind == "send" else torch.empty(t.shape, dtype=t.dtype)
            if kind == "recv":
                copy_back.append((t, h))
            t = h
        posted.append(dist.P2POp(dist.isend if kind == "send" else dist.irecv, t, peer, group))
    for req in dist.batch_isend_irecv(posted):
        req.wait()
    for t, h in copy_back:
        t.copy_(h)


def _default_device(group):
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def broadcast_keys(keys, src=0, group=None, device=None):
    """The key table (n_keys, 64 or 32) uint8 held on ``src`` (ignored, may be
    None, elsewhere), on every rank (per-packet key tables are
    broadcast, each rank expands its own copy; 65 536 x 64 B = 4 MiB, one
    RCCL broadcast over xGMI).  Returns the contiguous table on ``device``."""
    rank = dist.get_rank(group)
    dev = device if device is not None else (keys.device if keys is not None else _default_device(group))
    if rank == src:
        k = torch.as_tensor(keys)
        bad = k.dtype != torch.uint8 or k.dim() != 2 or k.shape[1] not in (32, 64) or k.shape[0] < 1
        # a refused table still completes the shape broadcast (as [-1, -1]) so
        # that every rank raises instead of the others waiting forever
        shape = torch.tensor([-1, -1] if bad else [k.shape[0], k.shape[1]], dtype=torch.int64, device=dev)
    else:
        shape = torch.empty(2, dtype=torch.int64, device=dev)
    if dist.get_world_size(group) > 1:
        dist.broadcast(shape, src, group=group)
    n, klen = (int(x) for x in shape)
    if n < 0:
        raise ValueError("keys must be a (n_keys, 64 or 32) uint8 table" if rank == src else
                         f"rank {src} refused its key table (not a (n_keys, 64 or 32) uint8 table)")
    out = k.contiguous().to(dev) if rank == src else torch.empty((n, klen), dtype=torch.uint8, device=dev)
    if _staged(group) and out.is_cuda:          # gloo: through a host copy
        h = out.cpu()
        dist.broadcast(h, src, group=group)
        out.copy_(h)
    else:
        dist.broadcast(out, src, group=group)
    return out


def broadcast_keyset(keys, src=0, group=None, device=None, stream=None):
    """broadcast_keys, then a device KeySet of the table on every rank
    (device.keyset: expanded on the GPU, no host round trip)."""
    from . import device as _device
    return _device.keyset(broadcast_keys(keys, src, group, device), stream=stream)


def scatter_packed(buf, off, length, bounds, src=0, group=None, device=None, rows=()):
    """Send each rank its packet range of a packed batch held on ``src``.

    On the source, ``buf`` (uint8), ``off`` (any integer dtype, sent as
    int64) and ``length`` (sent as int32) describe the whole batch, and each
    tensor of ``rows`` holds one fixed-width record per packet (e.g. IVs
    (n, 16) uint8, key indices (n,) int32); elsewhere they are ignored (may
    be None; ``rows`` must then be ``(dtype, width)`` pairs so receivers can
    size their buffers).  Returns this rank's (buf, off, length, rows) with
    offsets rebased to 0.
    """
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = device if device is not None else (buf.device if buf is not None else _default_device(group))
    if rank == src:
        parts = [_slice(buf, off, length, lo, hi) for lo, hi in bounds]
        sizes = torch.tensor([[p[0].numel(), p[1].numel()] for p in parts], dtype=torch.int64, device=dev)
    else:
        sizes = torch.empty((world, 2), dtype=torch.int64, device=dev)
    dist.broadcast(sizes, src, group=group)
    nb, npk = (int(x) for x in sizes[rank])
    if rank == src:
        ops = []
        for r in range(world):
            if r == src:
                continue
            lo, hi = bounds[r]
            for t in (*parts[r], *(x[lo:hi] for x in rows)):
                if t.numel():
                    ops.append(("send", t.contiguous().to(dev), r))
        _wait(ops, group)
        lo, hi = bounds[src]
        b, o, l = parts[src]
        return b.to(dev), o.to(dev), l.to(dev), [x[lo:hi].to(dev) for x in rows]
    rb = torch.empty(nb, dtype=torch.uint8, device=dev)
    ro = torch.empty(npk, dtype=torch.int64, device=dev)
    rl = torch.empty(npk, dtype=torch.int32, device=dev)
    rr = [torch.empty((npk, *w) if isinstance(w, tuple) else ((npk, w) if w else (npk,)), dtype=dt, device=dev)
          for dt, w in rows]
    _wait([("recv", t, src) for t in (rb, ro, rl, *rr) if t.numel()], group)
    return rb, ro, rl, rr


def gather_packed(buf, off, length, dst=0, group=None, rows=()):
    """Mirror of scatter_packed: every rank sends its packed output range
    (and its fixed-width ``rows``) to ``dst``, which returns the concatenated
    batch (offsets rebased per rank onto one buffer, packet order = rank
    order) and the concatenated rows.  Other ranks return None."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = buf.device
    off = off.to(torch.int64)
    length = length.to(torch.int32)
    mine = torch.tensor([buf.numel(), off.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.empty(2, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, mine, group=group)
    sizes = [(int(s[0]), int(s[1])) for s in sizes]
    if rank != dst:
        _wait([("send", t.contiguous(), dst) for t in (buf, off, length, *rows) if t.numel()], group)
        return None
    bufs, offs, lens, rws, ops = [], [], [], [[] for _ in rows], []
    for r in range(world):
        nb, npk = sizes[r]
        if r == dst:
            b, o, l, rr = buf, off, length, list(rows)
        else:
            b = torch.empty(nb, dtype=torch.uint8, device=dev)
            o = torch.empty(npk, dtype=torch.int64, device=dev)
            l = torch.empty(npk, dtype=torch.int32, device=dev)
            rr = [torch.empty((npk, *x.shape[1:]), dtype=x.dtype, device=dev) for x in rows]
            ops += [("recv", t, r) for t in (b, o, l, *rr) if t.numel()]
        bufs.append(b)
        offs.append(o)
        lens.append(l)
        for j, t in enumerate(rr):
            rws[j].append(t)
    _wait(ops, group)
    base, out_off = 0, []
    for r in range(world):
        out_off.append(offs[r] + base)
        base += sizes[r][0]
    return torch.cat(bufs), torch.cat(out_off), torch.cat(lens), [torch.cat(x) for x in rws]


def sharded_call(work, buf, off, length, rows=(), row_specs=(), balance=False, src=0, group=None, device=None,
                 sync=None):
    """One batch held on ``src``, processed by every rank: partition (by
    count, or by work_per_packet with ``balance``), scatter, ``work`` on each
    rank's shard, gather back to ``src``.

    ``work(buf, off, length, rows) -> (out_buf, out_off, out_len, out_rows)``
    runs the per-rank kernels (reticulum_amd.device on a GPU; any stand-in
    with the same contract in tests).  ``row_specs`` gives receivers the
    (dtype, width) of each of ``rows``.  ``sync()`` (e.g.
    torch.cuda.synchronize) separates the phases for timing.

    Returns ``(result, times)``: on ``src`` result is the gathered
    (buf, off, length, rows), elsewhere None; times = {"scatter_s",
    "compute_s", "gather_s"} measured on this rank between barriers.
    """
    import time
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    sync = sync or (lambda: None)
    if rank == src:
        n = off.numel()
        bounds = partition(n, world, length if balance else None)
    else:
        bounds = None
    times = {}
    dist.barrier(group=group)
    t0 = time.perf_counter()
    b, o, l, rr = scatter_packed(buf, off, length, bounds, src=src, group=group, device=device,
                                 rows=rows if rank == src else row_specs)
    sync()
    dist.barrier(group=group)
    t1 = time.perf_counter()
    ob, oo, ol, orows = work(b, o, l, rr)
    sync()
    dist.barrier(group=group)
    t2 = time.perf_counter()
    res = gather_packed(ob, oo, ol, dst=src, group=group, rows=orows)
    sync()
    dist.barrier(group=group)
    t3 = time.perf_counter()
    times["scatter_s"], times["compute_s"], times["gather_s"] = t1 - t0, t2 - t1, t3 - t2
    return res, times


class _Posted:
    """Transfers posted as one grouped batch.  wait(): with RCCL the current
    stream waits for them (the host does not block); with gloo the host
    blocks.  Device tensors under gloo (the one-GPU rehearsal) are staged
    through host copies synchronously at posting time."""

    def __init__(self, ops, group):
        self.works, self.copy_back = [], []
        if not ops:
            return
        if _staged(group) and any(t.is_cuda for _, t, _ in ops):
            _wait(ops, group)
            return
        posted = [dist.P2POp(dist.isend if kind == "send" else dist.irecv, t, peer, group) for kind, t, peer in ops]
        self.works = dist.batch_isend_irecv(posted)

    def wait(self):
        for w in self.works:
            w.wait()
        self.works = []


def _chunks(lo, hi, chunks, lengths=None):
    """[lo, hi) cut into `chunks` contiguous sub-ranges (by count, or by
    work_per_packet with ``lengths``)."""
    sub = partition(hi - lo, chunks, None if lengths is None else lengths[lo:hi])
    return [(lo + a, lo + b) for a, b in sub]


def sharded_call_pipelined(work, buf, off, length, rows=(), row_specs=(), out_cap=None, out_row_specs=(),
                           chunks=4, balance=False, src=0, group=None, device=None, sync=None):
    """sharded_call with the three legs overlapped ("or
    overlapped via chunked pipelining").  Each rank's share is cut into
    ``chunks`` sub-ranges; at step k one grouped batch of point-to-point
    transfers carries the inputs of chunk k (src -> ranks) AND the outputs of
    chunk k-2 (ranks -> src), both directions of every xGMI link at once,
    while the compute stream runs chunk k-1.  With RCCL nothing blocks the
    host inside the pipeline: the batch of step k is posted after the work of
    chunk k-2 was enqueued (the collective stream waits for it), and the work
    of chunk k-1 is enqueued after its own inputs' batch (the compute stream
    waits for that one only).

    ``out_cap(lengths) -> per-packet output capacity`` (int64 tensor, e.g.
    the token length of each plaintext) fixes the output layout: ``work``
    must place packet i's output at the prefix sum of the capacities of the
    packets before it in its chunk (as reticulum_amd.device's packed entries
    do) and return at least that many bytes; ``out_row_specs`` gives the
    (dtype, width) of each output row tensor.  Every size is known on ``src``
    before the first transfer, so one size table is broadcast up front and
    no rank synchronises with the host again until the end.

    Returns ``(result, times)`` like sharded_call: on ``src`` the gathered
    (buf, off, length, rows) in packet order, with off = prefix sums of the
    capacities and length = the capacities; times = {"total_s", "chunks"},
    the overlapped wall time between barriers.
    """
    import time
    if out_cap is None:
        raise ValueError("sharded_call_pipelined needs out_cap (the per-packet output capacity)")
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    sync = sync or (lambda: None)
    chunks = max(1, int(chunks))
    dev = device if device is not None else (buf.device if buf is not None else _default_device(group))

    def rows_alloc(specs, npk):
        return [torch.empty((npk, *w) if isinstance(w, tuple) else ((npk, w) if w else (npk,)), dtype=dt, device=dev)
                for dt, w in specs]

    dist.barrier(group=group)
    t0 = time.perf_counter()
    # size table: per (rank, chunk) [packets, input bytes, output bytes, first packet]
    if rank == src:
        n = off.numel()
        lens64 = length.to(torch.int64)
        cap = out_cap(lens64).to(torch.int64)
        bounds = partition(n, world, lens64 if balance else None)
        cut = [_chunks(lo, hi, chunks, lens64 if balance else None) for lo, hi in bounds]
        pieces = [[_slice(buf, off, length, a, b) for a, b in cut[r]] for r in range(world)]
        cap_cs = torch.cumsum(cap, 0) - cap if n else cap
        cap_cs_host = cap_cs.cpu().tolist()         # gather destinations, no host sync inside the pipeline
        table = torch.tensor([[[b - a, pieces[r][c][0].numel(), int(cap[a:b].sum()) if b > a else 0, a]
                               for c, (a, b) in enumerate(cut[r])] for r in range(world)], dtype=torch.int64)
    else:
        table = torch.empty((world, chunks, 4), dtype=torch.int64)
    if world > 1:
        tt = table.to(dev) if dist.get_backend(group) == "nccl" else table
        dist.broadcast(tt, src, group=group)
        table = tt.cpu()
    tab = table.tolist()

    if rank == src:
        total_out = int(cap.sum()) if n else 0
        out_buf = torch.empty(max(total_out, 1), dtype=torch.uint8, device=dev)[:total_out]
        out_rows = rows_alloc(out_row_specs, n)
    inputs = {}     # chunk -> (b, o, l, rows) on this rank
    outputs = {}    # chunk -> (out bytes, out rows) awaiting the gather

    def scatter_ops(c):
        ops = []
        if rank == src:
            for r in range(world):
                npk, nb, _, first = tab[r][c]
                b, o, l = pieces[r][c]
                rr = [x[first:first + npk] for x in rows]
                if r == src:
                    inputs[c] = (b.to(dev), o.to(dev), l.to(dev), [x.to(dev) for x in rr])
                    continue
                for t in (b, o, l, *rr):
                    if t.numel():
                        ops.append(("send", t.contiguous().to(dev), r))
        else:
            npk, nb, _, _ = tab[rank][c]
            rb = torch.empty(nb, dtype=torch.uint8, device=dev)
            ro = torch.empty(npk, dtype=torch.int64, device=dev)
            rl = torch.empty(npk, dtype=torch.int32, device=dev)
            rr = rows_alloc(row_specs, npk)
            inputs[c] = (rb, ro, rl, rr)
            ops += [("recv", t, src) for t in (rb, ro, rl, *rr) if t.numel()]
        return ops

    def gather_ops(c):
        ops = []
        if rank == src:
            for r in range(world):
                npk, _, ob, first = tab[r][c]
                if npk == 0:
                    continue
                base = cap_cs_host[first] if first < n else total_out
                dst = [out_buf[base:base + ob]] + [x[first:first + npk] for x in out_rows]
                if r == src:
                    mb, mrows = outputs.pop(c)
                    for d, s_ in zip(dst, [mb[:ob]] + list(mrows)):
                        d.copy_(s_)
                    continue
                ops += [("recv", t, r) for t in dst if t.numel()]
        elif c in outputs:
            npk, _, ob, _ = tab[rank][c]
            mb, mrows = outputs.pop(c)
            ops += [("send", t.contiguous(), src) for t in [mb[:ob], *mrows] if t.numel()]
        return ops

    def compute(c):
        npk = tab[rank][c][0]
        if npk == 0:
            return
        b, o, l, rr = inputs.pop(c)
        ob, _, _, orows = work(b, o, l, rr)
        outputs[c] = (ob, list(orows))

    pending = {}
    for k in range(chunks + 2):
        ops = (scatter_ops(k) if k < chunks else []) + (gather_ops(k - 2) if k >= 2 else [])
        pending[k] = _Posted(ops, group)
        if 1 <= k <= chunks:
            pending.pop(k - 1).wait()           # inputs of chunk k-1 (and the gathers of k-3)
            compute(k - 1)
    for p in pending.values():
        p.wait()
    sync()
    dist.barrier(group=group)
    times = {"total_s": time.perf_counter() - t0, "chunks": chunks}
    if rank != src:
        return None, times
    out_off = cap_cs if n else cap
    return (out_buf, out_off.to(dev), cap.to(torch.int32).to(dev), out_rows), times
