"""c5's encrypt half with coalesced plaintext reads, against packed rows
("have the bucketing pass gather each bucket into the
unit-interleaved layout ... A/B it in one process").

  tools/build_variant.sh base
  tools/build_variant.sh tile -DRNSTOK_SPLIT_TILE=1
  python tools/c5_tile_ab.py build_exp/base/librnstok.so build_exp/tile/librnstok.so

One rank's c5 encrypt half: 2^19 packets of 64-4096 B, 65 536 keys, ordered
longest first (as RT_F_SORT_BY_LENGTH orders them), on the split kernel's
packed path (k_encrypt_split, GEN).  The base build reads each packet's
plaintext from its byte string; the tile build reads it from 64-packet tiles
(unit u of lane l at tile + 16 (64 u + l), each tile as long as its longest
packet), so every wave's plaintext load is one contiguous KiB.  Tokens are
byte strings in both and must be identical.  The tiles are built before
timing; the gather that would build them inside a step is timed apart (a
device gather of 16-B units, the same bytes).  Prints one JSON line.
"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    libs = sys.argv[1:3]
    import numpy as np
    import torch
    from reticulum_amd import _native
    _native._share_hip_runtime_with_torch()
    torch.cuda.init()
    dev = torch.device("cuda", 0)
    n, nk = 1 << 19, 65536
    kg = torch.Generator().manual_seed(55)
    g = torch.Generator(device=dev).manual_seed(5)
    lens = torch.randint(64, 4097, (n,), dtype=torch.int32, generator=kg)
    keys = torch.randint(0, 256, (nk, 64), dtype=torch.uint8, generator=kg).numpy()
    lens, _ = torch.sort(lens, descending=True, stable=True)
    lens_d = lens.to(dev)
    L64 = lens.to(torch.int64)
    off = torch.zeros(n, dtype=torch.int64)
    off[1:] = torch.cumsum(L64[:-1], 0)
    total = int(L64.sum())
    rows = torch.zeros(total + 16, dtype=torch.uint8, device=dev)
    rows[:total] = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device=dev, generator=g)
    kidx = torch.randint(0, nk, (n,), dtype=torch.int32, device=dev, generator=g)
    # tiles: 64 consecutive packets of the order, unit u of lane l at 16 (base + 64 u + l)
    units = (L64 + 15) // 16
    t_units = units.view(-1, 64).max(dim=1).values
    t_base = torch.zeros(n // 64, dtype=torch.int64)
    t_base[1:] = torch.cumsum(64 * t_units[:-1], 0)
    tile_units = int(64 * t_units.sum())
    pos = torch.arange(n, dtype=torch.int64)
    lane, tile = pos % 64, pos // 64
    toff_tile = 16 * (t_base[tile] + lane)                # unit 0 of each packet in the tile buffer
    tiles = torch.zeros(tile_units * 16 + 16, dtype=torch.uint8, device=dev)
    src_units, dst_units = [], []
    ar16 = torch.arange(16, device=dev)
    off_d, toff_tile_d, units_d = off.to(dev), toff_tile.to(dev), units.to(dev)
    for u in range(int(units.max())):
        k = torch.nonzero(units_d > u).squeeze(1)
        src = (off_d[k] + 16 * u)[:, None] + ar16
        keep = (16 * u + ar16)[None, :] < lens_d[k].to(torch.int64)[:, None]
        dst = (toff_tile_d[k] + 1024 * u)[:, None] + ar16
        tiles[dst[keep]] = rows[src[keep]]
        src_units.append(off_d[k] + 16 * u)
        dst_units.append(toff_tile_d[k] + 1024 * u)
    torch.cuda.synchronize()
    tl = (16 + 16 * (lens // 16 + 1) + 32).to(torch.int64)
    tok_off = torch.zeros(n, dtype=torch.int64)
    tok_off[1:] = torch.cumsum(tl[:-1], 0)
    tok_bytes = int(tl.sum())
    tok_off_d = tok_off.to(dev)
    off_rows_d = off_d

    variants = []
    for path, pt_buf, pt_off in ((libs[0], rows, off_rows_d), (libs[1], tiles, toff_tile_d)):
        lib = ctypes.CDLL(os.path.abspath(path))
        for name, res, argt in _native.SIGNATURES:
            if hasattr(lib, name):
                f = getattr(lib, name)
                f.restype, f.argtypes = res, argt
        ctx = lib.rt_create(0)
        ks = lib.rt_keyset_create(ctx, keys.ctypes.data_as(ctypes.c_void_p), 64, nk)
        assert ctx and ks, lib.rt_last_error()
        tok = torch.zeros(tok_bytes, dtype=torch.uint8, device=dev)
        variants.append(dict(path=path, lib=lib, ks=ks, pt=pt_buf, off=pt_off, tok=tok, ms=[]))
    s = torch.cuda.current_stream()

    def run(v):
        rc = v["lib"].rt_encrypt(v["ks"], v["pt"].data_ptr(), v["off"].data_ptr(), lens_d.data_ptr(),
                                 kidx.data_ptr(), iv.data_ptr(), v["tok"].data_ptr(), tok_off_d.data_ptr(), n,
                                 s.cuda_stream)
        assert rc == 0, v["lib"].rt_last_error()

    for v in variants:
        run(v)
        run(v)
    torch.cuda.synchronize()
    same = torch.equal(variants[0]["tok"], variants[1]["tok"])
    for r in range(20):
        for v in (variants if r % 2 == 0 else variants[::-1]):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            run(v)
            b.record(s)
            torch.cuda.synchronize()
            v["ms"].append(a.elapsed_time(b))
    # the gather that would build the tiles inside a step: every 16-B unit
    # (row units may straddle; a copy of 16-B units through an index is the
    # lower bound of any such pass)
    src_u = torch.cat(src_units)
    dst_u = torch.cat(dst_units)
    r16 = rows.unfold(0, 16, 1)                          # 16-B window at every byte offset (a view)
    out16 = tiles[:tile_units * 16].view(-1, 16)
    gms = []
    for r in range(10):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        out16.index_copy_(0, dst_u // 16, r16.index_select(0, src_u))
        b.record(s)
        torch.cuda.synchronize()
        gms.append(a.elapsed_time(b))
    res = {"packets": n, "keys": nk, "plaintext_bytes": total, "tile_bytes": tile_units * 16,
           "tokens_identical": same,
           "rows_ms": statistics.median(variants[0]["ms"]), "tile_ms": statistics.median(variants[1]["ms"]),
           "gather_ms": statistics.median(gms),
           "note": "c5 encrypt half, longest first, per-key split kernel (GEN, static batches); tile build reads "
                   "plaintext from 64-packet tiles (coalesced 1-KiB wave loads), tokens stay byte strings; "
                   "gather_ms = torch gather of the tiles' 16-B units (index_select + index_copy), untuned"}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
