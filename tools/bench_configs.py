"""Device-resident timings of the non-headline BASELINE configs on one GPU.

  python tools/bench_configs.py [--config c3|c4|c4s8|c5] [--steps K]

c3  : 2^20 x 500 B, 65 536 per-packet keys (uniform random key_idx)
c4  : 262 144 x 16 KiB, one key (Resource-sized tokens, whole batch on 1 GPU)
c4s8: 32 768 x 16 KiB, one key (the per-GPU shard of c4 at 8 GPUs)
ident: 2^20 x 500 B with a fresh HKDF-derived key per packet (Identity.encrypt
      keying, Identity.py:837-846): times rt_hkdf (32 B shared key, 16 B
      salt -> 64 B), the derived keyset (HKDF + key setup, incl. allocation)
      and encrypt / decrypt with key_idx = packet index
ratchet: Identity.decrypt's ratchet trial loop: 2^16 x 500 B tokens x 16
      candidate keys (first opening key per token), then the decrypt
resource: Resource hashmaps: 1024 resources x 1024 parts
      x 464 B, map hashes with and without the 224-part collision guard
wire: the interface path around the token, 2^20 raw
      500-B packets on the device: HDLC framing into one stream, deframing
      that stream (the read loop), IFAC mask and unmask (16-B IFACs, 64-B
      key), Packet.unpack + packet hash; one line with every stage
node: the interface path composed (reticulum_amd.pipeline), 2^20 DATA packets
      of 383 B plaintext (a 432-B token, 451-B packet, 467 B with a 16-B
      IFAC): outbound token encrypt -> header pack -> IFAC mask -> HDLC
      framing into one stream, and inbound deframing -> IFAC unmask -> unpack
      -> token decrypt of that stream; every plaintext checked
c5  : 2^20 packets (the per-GPU share of 8 M at 8 GPUs), lengths uniform in
      64..4096 B, 65 536 keys, 50/50 encrypt / decrypt (decrypt inputs are
      valid tokens produced by the encrypt kernel beforehand)

Prints one JSON line per config.  Used for DESIGN.md §5; bench.py is the
headline (c2).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def warm(fn, seconds=0.3):
    """Steady clocks before timing: `fn` back to back for `seconds` (the GPU's
    clocks ramp up over ~50 ms of work after an idle spell, bench.warmup)."""
    import torch
    import bench
    bench.warmup(fn, torch.cuda.current_stream(), 2, seconds)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--sort", type=int, default=1, help="c5: bucket packets by length before launch")
    args = ap.parse_args()
    import torch
    import reticulum_amd as rt
    from reticulum_amd import device

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    cfg = args.config
    res = {"config": cfg}
    if cfg in ("c3", "c4", "c4s8"):
        n, L, nk = {"c3": (1 << 20, 500, 65536), "c4": (262144, 16384, 1), "c4s8": (32768, 16384, 1)}[cfg]
        tl = rt.token_len(L)
        pt = torch.randint(0, 256, (n, L), dtype=torch.uint8, device=dev, generator=g)
        iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device=dev, generator=g)
        keys = torch.randint(0, 256, (nk, 64), dtype=torch.uint8).numpy()
        ks = rt.KeySet(keys)
        kidx = torch.randint(0, nk, (n,), dtype=torch.int32, device=dev, generator=g) if nk > 1 else None
        tok = torch.empty((n, tl), dtype=torch.uint8, device=dev)
        back = torch.empty((n, tl - 48), dtype=torch.uint8, device=dev)
        ol = torch.empty(n, dtype=torch.int32, device=dev)
        st = torch.empty(n, dtype=torch.int32, device=dev)

        def enc():
            device.encrypt_uniform(ks, pt, L, iv, tok, key_idx=kidx)

        def dec():
            device.decrypt_uniform(ks, tok, tl, back, ol, st, key_idx=kidx)

        bytes_pt = n * L
        n_enc = n_dec = n
        check = lambda: bool((st == 0).all()) and torch.equal(back[:, :L], pt)  # noqa: E731
    elif cfg == "ident":
        n, L = 1 << 20, 500
        tl = rt.token_len(L)
        ikm = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device=dev, generator=g)
        salt = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device=dev, generator=g)
        okm = torch.empty((n, 64), dtype=torch.uint8, device=dev)
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        hk, dk = [], []
        warm(lambda: (device.hkdf(ikm, okm, salt), device.derive_keyset(ikm, salt)))
        for _ in range(5):
            e0.record()
            device.hkdf(ikm, okm, salt)
            e1.record()
            ks = device.derive_keyset(ikm, salt)
            e2.record()
            torch.cuda.synchronize()
            hk.append(e0.elapsed_time(e1))
            dk.append(e1.elapsed_time(e2))
        res["hkdf_ms"] = sorted(hk)[2]
        res["derive_keyset_ms"] = sorted(dk)[2]
        res["hkdf_keys_s"] = n / (res["hkdf_ms"] * 1e-3)
        # one salt row for the whole batch (salt_stride 0): packets to one identity
        shared = salt[:1].expand(n, 16)
        okm2 = torch.empty_like(okm)
        hs, ds = [], []
        for _ in range(5):
            e0.record()
            device.hkdf(ikm, okm2, shared)
            e1.record()
            device.derive_keyset(ikm, shared)
            e2.record()
            torch.cuda.synchronize()
            hs.append(e0.elapsed_time(e1))
            ds.append(e1.elapsed_time(e2))
        res["hkdf_shared_salt_ms"] = sorted(hs)[2]
        res["derive_keyset_shared_salt_ms"] = sorted(ds)[2]
        pt = torch.randint(0, 256, (n, L), dtype=torch.uint8, device=dev, generator=g)
        iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device=dev, generator=g)
        kidx = torch.arange(n, dtype=torch.int32, device=dev)
        tok = torch.empty((n, tl), dtype=torch.uint8, device=dev)
        back = torch.empty((n, tl - 48), dtype=torch.uint8, device=dev)
        ol = torch.empty(n, dtype=torch.int32, device=dev)
        st = torch.empty(n, dtype=torch.int32, device=dev)

        def enc():
            device.encrypt_uniform(ks, pt, L, iv, tok, key_idx=kidx)

        def dec():
            device.decrypt_uniform(ks, tok, tl, back, ol, st, key_idx=kidx)

        bytes_pt = n * L
        n_enc = n_dec = n
        check = lambda: bool((st == 0).all()) and torch.equal(back[:, :L], pt)  # noqa: E731
    elif cfg == "c5":
        n, nk = 1 << 20, 65536
        lens = torch.randint(64, 4097, (n,), dtype=torch.int32, device=dev, generator=g)
        is_enc = torch.rand(n, device=dev, generator=g) < 0.5
        keys = torch.randint(0, 256, (nk, 64), dtype=torch.uint8).numpy()
        ks = rt.KeySet(keys)
        kidx = torch.randint(0, nk, (n,), dtype=torch.int32, device=dev, generator=g)
        tl = (16 + 16 * (lens // 16 + 1) + 32).to(torch.int32)
        pt_off = torch.zeros(n, dtype=torch.int64, device=dev)
        pt_off[1:] = torch.cumsum(lens[:-1].to(torch.int64), 0)
        tok_off = torch.zeros(n, dtype=torch.int64, device=dev)
        tok_off[1:] = torch.cumsum(tl[:-1].to(torch.int64), 0)
        pt = torch.randint(0, 256, (int(lens.sum()),), dtype=torch.uint8, device=dev, generator=g)
        iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device=dev, generator=g)
        tok = torch.zeros(int(tl.sum()), dtype=torch.uint8, device=dev)
        cap_off = torch.zeros(n, dtype=torch.int64, device=dev)        # decrypt writes tok_len-48 bytes each
        cap_off[1:] = torch.cumsum((tl[:-1] - 48).to(torch.int64), 0)
        back = torch.zeros(int((tl - 48).sum()), dtype=torch.uint8, device=dev)
        ol = torch.empty(n, dtype=torch.int32, device=dev)
        st = torch.empty(n, dtype=torch.int32, device=dev)
        # all tokens first (decrypt inputs), then split 50/50
        device.encrypt(ks, pt, pt_off, lens, iv, tok, tok_off, key_idx=kidx)
        e_idx = torch.nonzero(is_enc).flatten()
        d_idx = torch.nonzero(~is_enc).flatten()
        # the timed encrypt writes its half into a zeroed buffer of its own;
        # the check compares it with the tokens of the one unsorted launch
        # above (and the decrypt half's plaintexts with the inputs)
        tok_e = torch.zeros_like(tok)
        e_args = [pt, pt_off[e_idx].contiguous(), lens[e_idx].contiguous(), iv[e_idx].contiguous(), tok_e,
                  tok_off[e_idx].contiguous()]
        e_k = kidx[e_idx].contiguous()
        d_args = [tok, tok_off[d_idx].contiguous(), tl[d_idx].contiguous(), back, cap_off[d_idx].contiguous(),
                  ol[: len(d_idx)], st[: len(d_idx)]]
        d_k = kidx[d_idx].contiguous()

        def enc():
            device.encrypt(ks, *e_args, key_idx=e_k, sort=bool(args.sort))

        def dec():
            device.decrypt(ks, *d_args, key_idx=d_k, sort=bool(args.sort))

        bytes_pt = int(lens.sum())
        n_enc, n_dec = len(e_idx), len(d_idx)
        def check():
            # byte mask of the encrypt half's tokens (2.2 G bytes: repeat_interleave
            # and mask indexing past 2^31 elements fail on ROCm, so marks + cumsum)
            marks = torch.zeros(tok.numel() + 1, dtype=torch.int32, device=dev)
            e_off = tok_off[e_idx]
            marks.index_add_(0, e_off, torch.ones_like(e_off, dtype=torch.int32))
            marks.index_add_(0, e_off + tl[e_idx].to(torch.int64), -torch.ones_like(e_off, dtype=torch.int32))
            emask = torch.cumsum(marks, 0, dtype=torch.int32)[:-1] > 0
            # elementwise, no boolean-mask compaction (> 2^31 elements)
            ok = torch.equal(tok_e, torch.where(emask, tok, torch.zeros((), dtype=tok.dtype, device=dev)))
            ok = ok and bool((st[: len(d_idx)] == 0).all()) and torch.equal(ol[: len(d_idx)], lens[d_idx])
            for j in range(0, len(d_idx), 4099):
                i = int(d_idx[j])
                a, c, m = int(pt_off[i]), int(cap_off[i]), int(lens[i])
                ok = ok and torch.equal(back[c:c + m], pt[a:a + m])
            return ok
    elif cfg == "wire":
        print(json.dumps(wire_config(dev, g, args.steps)))
        return
    elif cfg == "resource":
        print(json.dumps(resource_config(dev, g, args.steps)))
        return
    elif cfg == "node":
        print(json.dumps(node_config(dev, g, args.steps)))
        return
    elif cfg == "ratchet":
        print(json.dumps(ratchet_config(dev, g, args.steps)))
        return
    else:
        raise SystemExit("unknown config " + cfg)

    for _ in range(2):
        enc()
        dec()
    torch.cuda.synchronize()
    ok = check()
    warm(lambda: (enc(), dec()))
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    t0 = time.perf_counter()
    for e in ev:
        e[0].record()
        enc()
        e[1].record()
        dec()
        e[2].record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    em = sorted(a.elapsed_time(b) for a, b, _ in ev)[len(ev) // 2]
    dm = sorted(b.elapsed_time(c) for _, b, c in ev)[len(ev) // 2]
    res.update({"ok": ok, "encrypt_ms": em, "decrypt_ms": dm, "step_ms": wall / args.steps * 1e3,
                "packets_per_step": (n_enc + n_dec) if cfg == "c5" else n,
                "encrypt_packets_s": n_enc / (em * 1e-3), "decrypt_packets_s": n_dec / (dm * 1e-3),
                "plaintext_gib_per_step": bytes_pt / 2**30,
                "gib_s": (bytes_pt if cfg == "c5" else 2 * bytes_pt) / ((em + dm) * 1e-3) / 2**30})
    print(json.dumps(res))


def ratchet_config(dev, g, steps):
    """Identity.decrypt's ratchet loop (Identity.py:865-878) at batch scale:
    2^16 tokens of 500 B, each tried against 16 candidate keys (out of 65 536
    derived keys) with the opening key at a uniform random rank: the trial
    pass (1 M HMAC verifications) and the decrypt of the opened tokens with
    their keys."""
    import torch
    import reticulum_amd as rt
    from reticulum_amd import device
    n, L, nk, per = 1 << 16, 500, 65536, 16
    tl = rt.token_len(L)
    ks = rt.KeySet(torch.randint(0, 256, (nk, 64), dtype=torch.uint8).numpy())
    kidx = torch.randint(0, nk, (n,), dtype=torch.int32, device=dev, generator=g)
    pt = torch.randint(0, 256, (n, L), dtype=torch.uint8, device=dev, generator=g)
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device=dev, generator=g)
    tok = torch.empty((n, tl), dtype=torch.uint8, device=dev)
    device.encrypt_uniform(ks, pt, L, iv, tok, key_idx=kidx)
    cand = torch.randint(0, nk, (n, per), dtype=torch.int32, device=dev, generator=g)
    rank = torch.randint(0, per, (n,), dtype=torch.int64, device=dev, generator=g)
    cand[torch.arange(n, device=dev), rank] = kidx
    pair_off = torch.arange(0, n * per + 1, per, dtype=torch.int32, device=dev)
    tok_off = torch.arange(n, dtype=torch.int64, device=dev) * tl
    tok_len = torch.full((n,), tl, dtype=torch.int32, device=dev)
    first = torch.empty(n, dtype=torch.int32, device=dev)
    flat, pairs = tok.reshape(-1), cand.reshape(-1)
    back = torch.empty((n, tl - 48), dtype=torch.uint8, device=dev)
    ol = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)

    def trial():
        device.verify_trials(ks, flat, tok_off, tok_len, pair_off, pairs, first)

    def opened():
        key = cand.gather(1, first.clamp(min=0).long().unsqueeze(1)).squeeze(1).contiguous()
        device.decrypt_uniform(ks, tok, tl, back, ol, st, key_idx=key)

    times = {}
    for name, fn in (("verify_trials", trial), ("decrypt_opened", opened)):
        warm(fn)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        for a, b in ev:
            a.record()
            fn()
            b.record()
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in ev)[steps // 2]
        times[name] = {"ms": ms}
    times["verify_trials"]["trials_s"] = n * per / (times["verify_trials"]["ms"] * 1e-3)
    times["decrypt_opened"]["packets_s"] = n / (times["decrypt_opened"]["ms"] * 1e-3)
    # the opening rank is the first occurrence of the token's key among its
    # candidates (a random candidate can repeat it earlier)
    expect = (cand == kidx.unsqueeze(1)).int().argmax(dim=1)
    ok = torch.equal(first.long(), expect.long()) and bool((st == 0).all()) and torch.equal(back[:, :L], pt)
    return {"config": "ratchet", "tokens": n, "candidates_per_token": per, "keys": nk, "payload": L, "ok": ok,
            "stages": times}


def resource_config(dev, g, steps):
    """Resource hashmaps (Resource.py:426-468, 505-506) for 1024 resources of
    1024 parts x 464 B (SDU) each, one launch: map hash = SHA-256(part ||
    random_hash)[:4] per part (8 compressions for 464 + 4 B), and the
    collision guard over the previous 224 parts of the same resource."""
    import torch
    from reticulum_amd import device
    n_res, per, sdu, guard = 1024, 1024, 464, 224
    n = n_res * per
    data = torch.randint(0, 256, (n * sdu,), dtype=torch.uint8, device=dev, generator=g)
    salts = torch.randint(0, 256, (n_res, 4), dtype=torch.uint8, device=dev, generator=g)
    off = torch.arange(n, dtype=torch.int64, device=dev) * sdu
    ln = torch.full((n,), sdu, dtype=torch.int32, device=dev)
    res = torch.arange(n, dtype=torch.int32, device=dev) // per
    out = torch.empty(n * 4, dtype=torch.uint8, device=dev)
    first = torch.empty(n_res, dtype=torch.int32, device=dev)
    times = {}
    for name, gd in (("map_hashes", 0), ("map_hashes+collision_guard", guard)):
        warm(lambda: device.map_hashes(data, out, salts, off, ln, res, sdu=sdu, guard=gd, first_collision=first))
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        for a, b in ev:
            a.record()
            device.map_hashes(data, out, salts, off, ln, res, sdu=sdu, guard=gd, first_collision=first)
            b.record()
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in ev)[steps // 2]
        times[name] = {"ms": ms, "parts_s": n / (ms * 1e-3), "input_gb_s": n * sdu / (ms * 1e-3) / 1e9}
    # size-independent check: a part equal to another part of the same resource
    # hashes equally, so one repeat planted inside the guard window is found
    # (first_collision holds global part indices); its neighbour stays clean
    rows = data.view(n, sdu)
    rows[5 * per + 100] = rows[5 * per + 40]
    device.map_hashes(data, out, salts, off, ln, res, sdu=sdu, guard=guard, first_collision=first)
    torch.cuda.synchronize()
    f = first.cpu()
    h = out.view(n, 4)
    ok = int(f[5]) == 5 * per + 100 and int(f[4]) == -1 and torch.equal(h[5 * per + 100], h[5 * per + 40])
    return {"config": "resource", "resources": n_res, "parts_per_resource": per, "sdu": sdu, "guard": guard,
            "ok": ok, "stages": times}


def node_config(dev, g, steps):
    import bench
    return bench.node_rate(dev, steps, g)


def wire_config(dev, g, steps):
    import torch
    from reticulum_amd import device
    n, L, isz = 1 << 20, 500, 16
    raw = torch.randint(0, 256, (n, L), dtype=torch.uint8, device=dev, generator=g)
    raw[:, 1] &= 0x7F                                       # hops < PATHFINDER_M: every packet unpacks
    flat = raw.reshape(-1)
    off = torch.arange(n, dtype=torch.int64, device=dev) * L
    ln = torch.full((n,), L, dtype=torch.int32, device=dev)
    framed = torch.empty(n * (2 * L + 2), dtype=torch.uint8, device=dev)
    foff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    device.hdlc_frame(flat, off, ln, framed, foff)
    torch.cuda.synchronize()
    total = int(foff[-1])
    stream_buf = framed[:total].clone()
    pairs = 2 * n                                            # frames and the empty gaps 7E|7E between them
    dout = torch.empty(total, dtype=torch.uint8, device=dev)
    d_off = torch.empty(pairs, dtype=torch.int64, device=dev)
    d_len = torch.empty(pairs, dtype=torch.int32, device=dev)
    d_st = torch.empty(pairs, dtype=torch.int32, device=dev)
    cnt = torch.empty(2, dtype=torch.int64, device=dev)
    ifac = torch.randint(0, 256, (n, isz), dtype=torch.uint8, device=dev, generator=g)
    key = torch.randint(0, 256, (64,), dtype=torch.uint8, device=dev, generator=g)
    ml = L + isz
    masked = torch.empty(n * ml, dtype=torch.uint8, device=dev)
    m_off = torch.arange(n, dtype=torch.int64, device=dev) * ml
    m_len = torch.full((n,), ml, dtype=torch.int32, device=dev)
    un = torch.empty(n * ml, dtype=torch.uint8, device=dev)
    ifac_out = torch.empty((n, isz), dtype=torch.uint8, device=dev)
    u_st = torch.empty(n, dtype=torch.int32, device=dev)
    fields = torch.empty((n, 96), dtype=torch.uint8, device=dev)
    stages = {
        "hdlc_frame": (lambda: device.hdlc_frame(flat, off, ln, framed, foff), n * L),
        "hdlc_deframe": (lambda: device.hdlc_deframe(stream_buf, dout, d_off, d_len, d_st, cnt), total),
        "ifac_mask": (lambda: device.ifac_mask(flat, off, ln, ifac, key, masked, m_off), n * L),
        "ifac_unmask": (lambda: device.ifac_unmask(masked, m_off, m_len, key, ifac_out, un, m_off, u_st), n * ml),
        "packet_unpack": (lambda: device.packet_unpack(flat, off, ln, fields), n * L),
    }
    for f, _ in stages.values():
        f()
    torch.cuda.synchronize()
    # size-independent checks: deframing returns every packet, unmasking inverts masking
    rows = torch.randint(0, n, (4096,), device=dev, generator=g)
    ok_frames = (int(cnt[0]) == pairs - 1 and int((d_st[0::2] == 0).sum()) == n and bool((d_len[0::2] == L).all()))
    idx = d_off[0::2][rows].unsqueeze(1) + torch.arange(L, device=dev)
    ok_frames = ok_frames and torch.equal(dout[idx], raw[rows])
    back = un.view(n, ml)[:, :L]
    ok_ifac = bool((u_st == 0).all()) and torch.equal(ifac_out, ifac) and torch.equal(back[:, 1:], raw[:, 1:]) and \
        torch.equal(back[:, 0], raw[:, 0] & 0x7F)
    ok_unpack = bool((fields[:, 0] == 1).all())
    res = {"config": "wire", "packets": n, "packet_bytes": L, "ifac_size": isz,
           "ok": bool(ok_frames and ok_ifac and ok_unpack), "stages": {}}
    for name, (f, nbytes) in stages.items():
        warm(f)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        for a, b in ev:
            a.record()
            f()
            b.record()
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in ev)[steps // 2]
        res["stages"][name] = {"ms": ms, "packets_s": n / (ms * 1e-3), "input_gb_s": nbytes / (ms * 1e-3) / 1e9}
    return res


if __name__ == "__main__":
    main()
