"""Soak of tests/test_threads_gpu.py's mix: more host threads and iterations
than the test (one process, one context), every result checked against the
oracle.  python tools/soak_threads.py [--threads 12] [--iters 600]"""
import argparse
import os
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=12)
    ap.add_argument("--iters", type=int, default=600)
    args = ap.parse_args()
    import reticulum_amd as rt
    from reticulum_amd import _native
    from oracle import ctoken as oracle
    import test_threads_gpu as T
    _native.context(0)
    T.ITERS = args.iters
    key = bytes(range(100, 164))
    tok = rt.Token(key)
    oracle.decrypt(key, oracle.encrypt(key, bytes(16), b""))
    stop = threading.Event()
    t0 = time.perf_counter()
    with ThreadPoolExecutor(args.threads + 1) as ex:
        dev = ex.submit(T._device_worker, rt, stop)
        try:
            futs = [ex.submit(T._worker, rt, 100 + t, key, tok) for t in range(args.threads)]
            counts = [f.result(timeout=600) for f in futs]
        finally:
            stop.set()
        rounds, bad = dev.result(timeout=120)
    dt = time.perf_counter() - t0
    ok = counts == [args.iters] * args.threads and bad == 0
    print({"ok": ok, "threads": args.threads, "iters": args.iters, "host_ops": sum(counts), "device_rounds": rounds,
           "device_mismatches": bad, "seconds": round(dt, 1)})
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
