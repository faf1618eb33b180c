"""Where k_encrypt_split's waves wait (probe build: -DRNSTOK_SPLIT_PROBE).

  tools/build_variant.sh splitprobe -DRNSTOK_SPLIT_PROBE
  RNSTOK_LIB=build_exp/splitprobe/librnstok.so python tools/split_wait_probe.py [--length L] [--ilv]

Per role (AES waves / hashing waves): the share of each wave's cycles (table
fill to exit) spent polling the other role's counter, and how many quads
found the counter not yet there.  The probe adds s_memtime reads around each
wait; timings are of the probe build, not the product's.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--length", type=int, default=500)
    ap.add_argument("--packets", type=int, default=1 << 20)
    ap.add_argument("--keys", type=int, default=1)
    ap.add_argument("--ilv", action="store_true")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import torch
    import reticulum_amd as rt
    from reticulum_amd import _native, device
    lib = _native.load()
    fn = lib.rt_split_probe_read
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    fn.restype = ctypes.c_int
    n, L = args.packets, args.length
    g = torch.Generator(device="cuda").manual_seed(3)
    keys = np.random.default_rng(3).integers(0, 256, (args.keys, 64), dtype=np.uint8)
    ks = rt.KeySet(keys if args.keys > 1 else keys[0].tobytes())
    kidx = torch.randint(0, args.keys, (n,), dtype=torch.int32, device="cuda", generator=g) if args.keys > 1 else None
    pt = torch.randint(0, 256, (n, L), dtype=torch.uint8, device="cuda", generator=g)
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    tl = rt.token_len(L)
    if args.ilv:
        pu = device.interleave(pt, L)
        tu = torch.empty((tl // 16, n, 16), dtype=torch.uint8, device="cuda")
        run = lambda: device.encrypt_interleaved(ks, pu, L, iv, tu, key_idx=kidx)     # noqa: E731
    else:
        tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
        run = lambda: device.encrypt_uniform(ks, pt, L, iv, tok, key_idx=kidx)        # noqa: E731
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 8)()
    fn(buf)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(args.reps):
        run()
    ev1.record()
    torch.cuda.synchronize()
    assert fn(buf) == 0
    v = list(buf)
    res = {"length": L, "packets": n, "keys": args.keys, "layout": "interleaved" if args.ilv else "rows",
           "ms_per_launch": ev0.elapsed_time(ev1) / args.reps}
    for r, name in ((0, "aes_waves"), (1, "hash_waves")):
        waves = v[6 + r] or 1
        res[name] = {"waves": waves // args.reps, "wait_share": v[r] / max(v[4 + r], 1),
                     "waits_per_wave": v[2 + r] / waves, "cycles_per_wave": v[4 + r] / waves,
                     "wait_cycles_per_wait": v[r] / max(v[2 + r], 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
