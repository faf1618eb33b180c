"""Throughput of the library's host-buffer entry points (rt_encrypt_host /
rt_decrypt_host through KeySet.encrypt_batch / decrypt_batch): packed numpy
(pageable) buffers of 2^20 x 500 B in, host buffers out, synchronous.  The
Python packing of bytes objects is excluded (the batch is built as Packed).

  python tools/host_path_bench.py [--packets N] [--length L] [--reps R]
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
    ap.add_argument("--packets", type=int, default=1 << 20)
    ap.add_argument("--length", type=int, default=500)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import numpy as np
    import reticulum_amd as rt
    from reticulum_amd.token import Packed
    n, L = args.packets, args.length
    rng = np.random.Generator(np.random.PCG64(7))
    pts = Packed(rng.integers(0, 256, n * L, dtype=np.uint8), np.arange(n, dtype=np.uint64) * L,
                 np.full(n, L, np.uint32))
    ivs = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    ks = rt.KeySet(bytes(range(64)))
    ks.encrypt_batch(Packed(pts.buf[:64 * L], pts.off[:64], pts.length[:64]), ivs=ivs[:64])   # warm-up
    te = td = float("inf")
    for _ in range(args.reps):
        t0 = time.perf_counter()
        toks = ks.encrypt_batch(pts, ivs=ivs)
        t1 = time.perf_counter()
        back, st = ks.decrypt_batch(toks)
        t2 = time.perf_counter()
        te, td = min(te, t1 - t0), min(td, t2 - t1)
    ok = bool((st == 0).all()) and np.array_equal(back.buf[:n * L].reshape(n, L) if False else back.buf.reshape(n, -1)[:, :L],
                                                  pts.buf.reshape(n, L))
    print(json.dumps({"packets": n, "length": L, "ok": ok, "encrypt_s": te, "decrypt_s": td,
                      "encrypt_packets_s": n / te, "decrypt_packets_s": n / td,
                      "encrypt_gib_s": n * L / te / 2**30, "decrypt_gib_s": n * L / td / 2**30}))


if __name__ == "__main__":
    main()
