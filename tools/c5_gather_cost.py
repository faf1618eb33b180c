"""What a coalescing pass would cost at c5's per-rank share (VERDICT r03 next
#1: "have the bucketing pass also gather each bucket into the unit-interleaved
layout, timed inside the step").

The encrypt half of one rank's c5 share is 2^19 packets of 64-4096 B (1.09
GB of plaintext) in packed rows.  A tile layout (64 length-ordered packets per
tile, 16-B unit u of the tile's lane l at tile_base + 16 (64 u + l)) makes every
wave's loads one contiguous KiB, but somebody has to write it: on the device,
a gather of every plaintext unit (and, for outputs a caller wants as byte
strings, a scatter back).  This times that gather as a bare copy (torch
index_select of 16-B units through the permutation, no crypto), i.e. a lower
bound of any gather pass, beside the encrypt kernel it would feed.

  python tools/c5_gather_cost.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    dev = torch.device("cuda", 0)
    kg = torch.Generator().manual_seed(55)
    n = 1 << 19
    lens = torch.randint(64, 4097, (n,), dtype=torch.int32, generator=kg)
    units = (lens + 15) // 16                      # plaintext units per packet (the pad block is made in-kernel)
    order = torch.argsort(units, descending=True, stable=True)
    u_sorted = units[order]
    n_tiles = (n + 63) // 64
    pad = n_tiles * 64 - n
    u_t = torch.cat([u_sorted, torch.zeros(pad, dtype=u_sorted.dtype)]).view(n_tiles, 64)
    tile_units = u_t.max(dim=1).values             # a tile is as long as its longest packet
    tile_base = torch.zeros(n_tiles, dtype=torch.int64)
    tile_base[1:] = torch.cumsum(64 * tile_units[:-1].to(torch.int64), 0)
    total_units = int(64 * tile_units.to(torch.int64).sum())
    off_units = torch.zeros(n, dtype=torch.int64)
    off_units[1:] = torch.cumsum(units[:-1].to(torch.int64), 0)
    # destination unit index of source unit j of packet order[k]
    src = torch.full((total_units,), -1, dtype=torch.int64)
    pos = torch.arange(n, dtype=torch.int64)
    tile, lane = pos // 64, pos % 64
    for u in range(int(units.max())):
        has = u_sorted > u
        k = pos[has]
        dst = tile_base[tile[has]] + 64 * u + lane[has]
        src[dst] = off_units[order[k]] + u
    src = src.clamp(min=0).to(dev)
    pt = torch.randint(0, 256, (int(units.sum()) * 16,), dtype=torch.uint8, device=dev).view(-1, 16)
    out = torch.empty((total_units, 16), dtype=torch.uint8, device=dev)

    def gather():
        torch.index_select(pt, 0, src, out=out)

    stream = torch.cuda.current_stream()
    bench.warmup(gather, stream, 4, 0.3)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
    for a, b in ev:
        a.record()
        gather()
        b.record()
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev)[5]
    moved = pt.numel() + out.numel()
    res = {"packets": n, "plaintext_bytes": int(lens.sum()), "tile_bytes": out.numel(),
           "tile_padding": out.numel() / (16 * int(units.sum())) - 1, "gather_ms": ms,
           "gather_gb_s": moved / (ms * 1e-3) / 1e9,
           "note": "bare 16-B-unit gather rows -> length-ordered 64-packet tiles (torch index_select), the lower "
                   "bound of a coalescing pass over c5's per-rank encrypt half; the encrypt kernel it would feed "
                   "runs ~1.7 ms (bench c5_rank_share_8gpu), so a pass inside the step costs this much before any "
                   "gain in the kernel (and as much again to scatter tokens back to byte strings)"}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
