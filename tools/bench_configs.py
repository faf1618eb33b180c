"""Device-resident timings of the non-headline BASELINE configs on one GPU.

  python tools/bench_configs.py [--config c3|c4|c4s8|c5] [--steps K]

c3  : 2^20 x 500 B, 65 536 per-packet keys (uniform random key_idx)
c4  : 262 144 x 16 KiB, one key (Resource-sized tokens, whole batch on 1 GPU)
c4s8: 32 768 x 16 KiB, one key (the per-GPU shard of c4 at 8 GPUs)
ident: 2^20 x 500 B with a fresh HKDF-derived key per packet (Identity.encrypt
      keying, Identity.py:837-846): times rt_hkdf (32 B shared key, 16 B
      salt -> 64 B), the derived keyset (HKDF + key setup, incl. allocation)
      and encrypt / decrypt with key_idx = packet index
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
        e_args = [pt, pt_off[e_idx].contiguous(), lens[e_idx].contiguous(), iv[e_idx].contiguous(), tok,
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
        check = lambda: bool((st[: len(d_idx)] == 0).all())  # noqa: E731
    else:
        raise SystemExit("unknown config " + cfg)

    for _ in range(2):
        enc()
        dec()
    torch.cuda.synchronize()
    ok = check()
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


if __name__ == "__main__":
    main()
