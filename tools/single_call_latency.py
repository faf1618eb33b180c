"""Per-call latency of the drop-in Token surface (one packet per call, as
Identity/Link call it): Token(key).encrypt / decrypt of 500-B plaintexts
through the library's host path (H2D, kernel, D2H, synchronous), with a
breakdown:

  token_*      Token(key).encrypt / decrypt (the drop-in, Python + C + GPU)
  host_abi_*   rt_encrypt_host / rt_decrypt_host on prebuilt numpy arrays
               (the C host path alone: copies, launch, sync)
  device_*     rt_encrypt_uniform / rt_decrypt_uniform on resident tensors
               + synchronize (launch + kernel + sync, no copies)
  sync_only    a one-element torch op + synchronize (the floor of any
               synchronous GPU call)

  python tools/single_call_latency.py [--calls N] [--length B]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def per_call(fn, calls):
    for _ in range(20):
        fn()
    t0 = time.perf_counter()
    for _ in range(calls):
        fn()
    return (time.perf_counter() - t0) / calls * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=2000)
    ap.add_argument("--length", type=int, default=500)
    args = ap.parse_args()
    import numpy as np
    import torch
    import reticulum_amd as rt
    from reticulum_amd import device as dev
    from reticulum_amd.token import token_len

    L = args.length
    tok = rt.Token(os.urandom(64))
    pt = os.urandom(L)
    for _ in range(50):
        assert tok.decrypt(tok.encrypt(pt)) == pt
    res = {"calls": args.calls, "length": L}
    t0 = time.perf_counter()
    toks = [tok.encrypt(pt) for _ in range(args.calls)]
    t1 = time.perf_counter()
    outs = [tok.decrypt(t) for t in toks]
    t2 = time.perf_counter()
    assert all(o == pt for o in outs)
    res["token_encrypt_us"] = (t1 - t0) / args.calls * 1e6
    res["token_decrypt_us"] = (t2 - t1) / args.calls * 1e6

    ks = tok.keyset
    lib = ks._lib
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    TL = token_len(L)
    h_pt = np.frombuffer(pt, dtype=np.uint8).copy()
    h_off = np.zeros(1, np.uint64)
    h_len = np.array([L], np.uint32)
    h_iv = np.frombuffer(os.urandom(16), dtype=np.uint8).copy()
    h_tok = np.zeros(TL, np.uint8)
    h_tlen = np.array([TL], np.uint32)
    h_out = np.zeros(TL, np.uint8)
    h_olen = np.zeros(1, np.uint32)
    h_st = np.zeros(1, np.int32)
    a_enc = (ks.handle, p(h_pt), p(h_off), p(h_len), None, p(h_iv), p(h_tok), p(h_off), 1)
    a_dec = (ks.handle, p(h_tok), p(h_off), p(h_tlen), None, p(h_out), p(h_off), p(h_olen), p(h_st), 1)
    res["host_abi_encrypt_us"] = per_call(lambda: lib.rt_encrypt_host(*a_enc), args.calls)
    res["host_abi_decrypt_us"] = per_call(lambda: lib.rt_decrypt_host(*a_dec), args.calls)
    assert h_st[0] == 0 and h_out[:L].tobytes() == pt

    d_pt = torch.from_numpy(h_pt).cuda().view(1, L)
    d_iv = torch.from_numpy(h_iv).cuda().view(1, 16)
    d_tok = torch.zeros(1, TL, dtype=torch.uint8, device="cuda")
    d_out = torch.zeros(1, TL, dtype=torch.uint8, device="cuda")
    d_olen = torch.zeros(1, dtype=torch.int32, device="cuda")
    d_st = torch.zeros(1, dtype=torch.int32, device="cuda")

    def enc():
        dev.encrypt_uniform(ks, d_pt, L, d_iv, d_tok)
        torch.cuda.synchronize()

    def dec():
        dev.decrypt_uniform(ks, d_tok, TL, d_out, d_olen, d_st)
        torch.cuda.synchronize()

    res["device_encrypt_us"] = per_call(enc, args.calls)
    res["device_decrypt_us"] = per_call(dec, args.calls)
    assert int(d_st[0]) == 0 and bytes(d_out[0, :L].cpu().numpy()) == pt
    x = torch.zeros(1, device="cuda")

    def sync_only():
        x.add_(1)
        torch.cuda.synchronize()

    res["sync_only_us"] = per_call(sync_only, args.calls)
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
