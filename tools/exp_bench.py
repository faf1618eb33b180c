"""A/B timing of librnstok variants in ONE process, interleaved rounds.

  python tools/exp_bench.py build_exp/a/librnstok.so build_exp/b/librnstok.so [--packets N] [--length L]

Each variant is loaded with its own ctypes handle (RTLD_LOCAL), gets its own
context and key set, and encrypts/decrypts the same device-resident batch;
outputs are cross-checked between variants.  Prints median / min kernel ms.
"""
import argparse
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--packets", type=int, default=1 << 20)
    ap.add_argument("--length", type=int, default=500)
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--keys", type=int, default=1)
    ap.add_argument("--probe", action="store_true", help="timing probes: skip the round-trip assertion")
    ap.add_argument("--kidx", choices=["random", "zero", "seq", "sorted"], default="random",
                    help="per-packet key pattern (with --keys > 1)")
    ap.add_argument("--ilv", action="store_true", help="the unit-interleaved layout (rt_encrypt_interleaved)")
    ap.add_argument("--packed", type=int, default=-1,
                    help="variable lengths drawn from [PACKED, length] through rt_encrypt/rt_decrypt (packed entry)")
    args = ap.parse_args()

    import torch
    from reticulum_amd import _native
    _native._share_hip_runtime_with_torch()
    torch.cuda.init()

    n, L = args.packets, args.length
    tl = 16 + 16 * (L // 16 + 1) + 32
    g = torch.Generator(device="cuda").manual_seed(1)
    # the plaintext rows sit in a buffer padded to 16-B units per packet, so
    # a variant that reads whole 16-B units of every packet (e.g. a
    # block-interleaved layout experiment) stays inside the allocation
    pt_buf = torch.zeros(max(n * ((L + 15) // 16 * 16), 16), dtype=torch.uint8, device="cuda")
    pt = pt_buf[: n * L].view(n, L)
    pt.copy_(torch.randint(0, 256, (n, L), dtype=torch.uint8, device="cuda", generator=g))
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    keys = torch.randint(0, 256, (args.keys, 64), dtype=torch.uint8).numpy()
    kidx = torch.randint(0, args.keys, (n,), dtype=torch.int32, device="cuda", generator=g) if args.keys > 1 else None
    if kidx is not None and args.kidx == "zero":
        kidx.zero_()
    elif kidx is not None and args.kidx == "seq":
        kidx = (torch.arange(n, device="cuda", dtype=torch.int32) % args.keys).contiguous()
    elif kidx is not None and args.kidx == "sorted":
        kidx = kidx.sort().values.contiguous()
    variants = []
    for path in args.libs:
        lib = ctypes.CDLL(os.path.abspath(path))
        for name, res, argt in _native.SIGNATURES:
            if not hasattr(lib, name):        # an older build of the library: entry points added since
                continue
            f = getattr(lib, name)
            f.restype, f.argtypes = res, argt
        ctx = lib.rt_create(0)
        assert ctx, lib.rt_last_error()
        ks = lib.rt_keyset_create(ctx, keys.ctypes.data_as(ctypes.c_void_p), 64, args.keys)
        assert ks, lib.rt_last_error()
        tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
        back = torch.empty((n, tl - 48), dtype=torch.uint8, device="cuda")
        ol = torch.empty(n, dtype=torch.int32, device="cuda")
        st = torch.empty(n, dtype=torch.int32, device="cuda")
        variants.append(dict(path=path, lib=lib, ks=ks, tok=tok, back=back, ol=ol, st=st, enc=[], dec=[]))
    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    kp = kidx.data_ptr() if kidx is not None else None
    packed = args.packed >= 0
    if packed:
        lens = torch.randint(args.packed, L + 1, (n,), dtype=torch.int32, device="cuda", generator=g)
        rows = torch.arange(n, dtype=torch.int64, device="cuda")
        p_off, t_off, b_off = rows * L, rows * tl, rows * (tl - 48)
        t_len = (16 + 16 * (lens // 16 + 1) + 32).to(torch.int32)

    if args.ilv:
        from reticulum_amd import device as _dev
        pt_u = _dev.interleave(pt, L)

    def run(v, ev=None):
        if ev:
            ev[0].record(s)
        if args.ilv:
            rc = v["lib"].rt_encrypt_interleaved(v["ks"], pt_u.data_ptr(), L, kp, iv.data_ptr(), v["tok"].data_ptr(),
                                                 n, sp)
        elif packed:
            rc = v["lib"].rt_encrypt(v["ks"], pt_buf.data_ptr(), p_off.data_ptr(), lens.data_ptr(), kp, iv.data_ptr(),
                                     v["tok"].data_ptr(), t_off.data_ptr(), n, sp)
        else:
            rc = v["lib"].rt_encrypt_uniform(v["ks"], pt.data_ptr(), L, L, kp, iv.data_ptr(), v["tok"].data_ptr(), tl,
                                             n, sp)
        assert rc == 0
        if ev:
            ev[1].record(s)
        if args.ilv:
            rc = v["lib"].rt_decrypt_interleaved(v["ks"], v["tok"].data_ptr(), tl, kp, v["back"].data_ptr(),
                                                 v["ol"].data_ptr(), v["st"].data_ptr(), n, sp)
        elif packed:
            rc = v["lib"].rt_decrypt(v["ks"], v["tok"].data_ptr(), t_off.data_ptr(), t_len.data_ptr(), kp,
                                     v["back"].data_ptr(), b_off.data_ptr(), v["ol"].data_ptr(), v["st"].data_ptr(), n, sp)
        else:
            rc = v["lib"].rt_decrypt_uniform(v["ks"], v["tok"].data_ptr(), tl, tl, kp, v["back"].data_ptr(), tl - 48,
                                             v["ol"].data_ptr(), v["st"].data_ptr(), n, sp)
        assert rc == 0
        if ev:
            ev[2].record(s)

    for v in variants:
        run(v)
        run(v)
    torch.cuda.synchronize()
    for v in variants:
        if packed:
            ok = bool((v["st"] == 0).all()) and torch.equal(v["ol"], lens)
            for i in range(0, n, max(1, n // 64)):
                ok = ok and torch.equal(v["back"][i, :int(lens[i])], pt[i, :int(lens[i])])
        elif args.ilv:
            back = _dev.deinterleave(v["back"].view((tl - 48) // 16, n, 16), tl - 48)
            ok = bool((v["st"] == 0).all()) and torch.equal(back[:, :L], pt)
        else:
            ok = bool((v["st"] == 0).all()) and torch.equal(v["back"][:, :L], pt)
        if packed:     # token bytes only (rows are wider than their tokens)
            same = all(torch.equal(v["tok"][i, :int(t_len[i])], variants[0]["tok"][i, :int(t_len[i])])
                       for i in range(0, n, max(1, n // 256)))
        else:
            same = torch.equal(v["tok"], variants[0]["tok"])
        print(f"{v['path']}: round-trip ok={ok} tokens==variant0: {same}")
    for r in range(args.rounds):
        for v in (variants if r % 2 == 0 else variants[::-1]):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            run(v, ev)
            torch.cuda.synchronize()
            v["enc"].append(ev[0].elapsed_time(ev[1]))
            v["dec"].append(ev[1].elapsed_time(ev[2]))
    for v in variants:
        e, d = statistics.median(v["enc"]), statistics.median(v["dec"])
        print(f"{v['path']:40s} enc {e:.4f} ms (min {min(v['enc']):.4f}) {n / e / 1e6:.3f} Gpkt/s | "
              f"dec {d:.4f} ms (min {min(v['dec']):.4f}) {n / d / 1e6:.3f} Gpkt/s")


if __name__ == "__main__":
    main()
