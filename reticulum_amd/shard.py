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
    """Bytes, rebased offsets and lengths of packets [lo, hi) of a packed batch."""
    if hi <= lo:
        return buf.new_zeros(0), off.new_zeros(0), length.new_zeros(0)
    start = int(off[lo])
    end = int((off[lo:hi] + length[lo:hi].to(off.dtype)).max())
    return buf[start:end], off[lo:hi] - start, length[lo:hi]


def scatter_packed(buf, off, length, bounds, src=0, group=None, device=None):
    """Send each rank its packet range of a packed batch held on ``src``.

    On the source, ``buf`` (uint8), ``off`` (int64) and ``length`` (int32)
    describe the whole batch; elsewhere they are ignored (may be None).
    Returns this rank's (buf, off, length) with offsets rebased to 0.
    """
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = device if device is not None else (buf.device if buf is not None else torch.device("cpu"))
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
            b, o, l = parts[r]
            for t in (b, o, l):
                if t.numel():
                    ops.append(dist.P2POp(dist.isend, t.contiguous().to(dev), r, group))
        for req in (dist.batch_isend_irecv(ops) if ops else []):
            req.wait()
        b, o, l = parts[src]
        return b.to(dev), o.to(dev), l.to(dev)
    rb = torch.empty(nb, dtype=torch.uint8, device=dev)
    ro = torch.empty(npk, dtype=torch.int64, device=dev)
    rl = torch.empty(npk, dtype=torch.int32, device=dev)
    ops = [dist.P2POp(dist.irecv, t, src, group) for t in (rb, ro, rl) if t.numel()]
    for req in (dist.batch_isend_irecv(ops) if ops else []):
        req.wait()
    return rb, ro, rl


def gather_packed(buf, off, length, dst=0, group=None):
    """Mirror of scatter_packed: every rank sends its packed output range to
    ``dst``, which returns the concatenated batch (offsets rebased per rank
    onto one buffer, packet order = rank order).  Other ranks return None."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = buf.device
    mine = torch.tensor([buf.numel(), off.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.empty(2, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, mine, group=group)
    sizes = [(int(s[0]), int(s[1])) for s in sizes]
    if rank != dst:
        ops = [dist.P2POp(dist.isend, t.contiguous(), dst, group) for t in (buf, off, length) if t.numel()]
        for req in (dist.batch_isend_irecv(ops) if ops else []):
            req.wait()
        return None
    bufs, offs, lens, ops = [], [], [], []
    for r in range(world):
        nb, npk = sizes[r]
        if r == dst:
            b, o, l = buf, off, length
        else:
            b = torch.empty(nb, dtype=torch.uint8, device=dev)
            o = torch.empty(npk, dtype=torch.int64, device=dev)
            l = torch.empty(npk, dtype=torch.int32, device=dev)
            ops += [dist.P2POp(dist.irecv, t, r, group) for t in (b, o, l) if t.numel()]
        bufs.append(b)
        offs.append(o)
        lens.append(l)
    for req in (dist.batch_isend_irecv(ops) if ops else []):
        req.wait()
    base, out_off = 0, []
    for r in range(world):
        out_off.append(offs[r] + base)
        base += sizes[r][0]
    return torch.cat(bufs), torch.cat(out_off), torch.cat(lens)
