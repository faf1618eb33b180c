"""Per-call vs batched use of the drop-in: where the GPU path pays.

  python tools/crossover.py [--out profiles/r06_crossover.json] [--seconds 0.6]

The reference calls Token once per packet, synchronously, from interface
reader threads and application threads (RNS/Link.py:1161-1182,
RNS/Identity.py:829-845).  For 383-B (a Link MDU-sized payload) and 500-B
plaintexts this measures round trips/s (encrypt, then decrypt of the token)
from host buffers, copies included:

* gpu_token_call:   reticulum_amd.Token.encrypt/decrypt, one packet per call;
* gpu_batch[B]:     KeySet.encrypt_batch / decrypt_batch over B packets per call
                    (lists of bytes in, Packed out: the Python surface's costs
                    included), B = 1, 8, 64, 512, 4096;
* cpu_openssl:      OpenSSL libcrypto (AES-NI + SHA-NI, key schedule and HMAC
                    pads hoisted), the strong-CPU context (tools/cpu_openssl.c);
* cpu_reference_est: oracle/cpuref.py (the reference's work shape in pure
                    Python) divided by its measured speed ratio to the
                    reference (tools/calibrate_cpuref.py: enc 1.64, dec 1.95),
                    i.e. the reference's own Token on one core.

each from 1 thread and from 16 threads (16 processes for the CPU rows, one
key per thread).  The crossover is the smallest B at which gpu_batch beats a
CPU row at the same thread count.
"""
import argparse
import ctypes
import json
import multiprocessing as mp
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BATCHES = (1, 8, 64, 512, 4096)
CPUREF_RATIO = {"enc": 1.64, "dec": 1.95}   # cpuref speed / reference speed


def _threads_rate(n_threads, seconds, setup, body):
    """round trips/s over n_threads threads, each running body(state) (which
    returns the round trips it made) until the deadline."""
    states = [setup(i) for i in range(n_threads)]
    for s in states:
        body(s)                                  # warm: key sets built, kernels loaded
    done = [0] * n_threads
    bad = []
    barrier = threading.Barrier(n_threads + 1)

    def work(i):
        barrier.wait()
        end = time.perf_counter() + seconds
        while time.perf_counter() < end:
            k = body(states[i])
            if k < 0:
                bad.append(i)
                return
            done[i] += k

    th = [threading.Thread(target=work, args=(i,)) for i in range(n_threads)]
    for t in th:
        t.start()
    barrier.wait()
    t0 = time.perf_counter()
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    return {"round_trips_s": sum(done) / el, "threads": n_threads, "seconds": el, "ok": not bad}


def gpu_token_call(L, n_threads, seconds):
    import reticulum_amd as rt

    def setup(i):
        return rt.Token(os.urandom(64)), os.urandom(L)

    def body(s):
        t, p = s
        return 1 if t.decrypt(t.encrypt(p)) == p else -1
    return _threads_rate(n_threads, seconds, setup, body)


def gpu_batch(L, B, n_threads, seconds):
    import reticulum_amd as rt

    def setup(i):
        return rt.KeySet(os.urandom(64)), [os.urandom(L) for _ in range(B)]

    def body(s):
        ks, pts = s
        toks = ks.encrypt_batch(pts)
        back, st = ks.decrypt_batch(toks)
        if not (st == 0).all() or back[B - 1] != pts[B - 1] or back[0] != pts[0]:
            return -1
        return B
    return _threads_rate(n_threads, seconds, setup, body)


def cpu_openssl(L, n_threads, seconds):
    path = os.path.join(ROOT, "tools", "libcpu_openssl.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.cpu_openssl_run.restype = ctypes.c_double
    lib.cpu_openssl_run.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
    done = ctypes.c_uint64()
    r = lib.cpu_openssl_run(n_threads, seconds, L, ctypes.byref(done))
    return {"round_trips_s": r, "threads": n_threads, "ok": r > 0}


def _cpuref_proc(L, seconds, q):
    from oracle import cpuref
    key, iv, p = os.urandom(64), os.urandom(16), os.urandom(L)
    n, te, td = 0, 0.0, 0.0
    end = time.perf_counter() + seconds
    while time.perf_counter() < end:
        t0 = time.perf_counter()
        tok = cpuref.encrypt(key, iv, p)
        t1 = time.perf_counter()
        ok = cpuref.decrypt(key, tok)
        t2 = time.perf_counter()
        te, td, n = te + t1 - t0, td + t2 - t1, n + 1
    q.put((n, te, td))


def cpu_reference_est(L, n_procs, seconds):
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    ps = [ctx.Process(target=_cpuref_proc, args=(L, seconds, q)) for _ in range(n_procs)]
    for p in ps:
        p.start()
    res = [q.get() for _ in ps]
    for p in ps:
        p.join()
    # per process: reference time per round trip = cpuref enc time x 1.64 + dec time x 1.95
    rate = sum(n / (te * CPUREF_RATIO["enc"] + td * CPUREF_RATIO["dec"]) for n, te, td in res)
    raw = sum(n / (te + td) for n, te, td in res)
    return {"round_trips_s": rate, "cpuref_round_trips_s": raw, "threads": n_procs, "ok": True}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06_crossover.json"))
    ap.add_argument("--seconds", type=float, default=0.6)
    ap.add_argument("--lengths", default="383,500")
    ap.add_argument("--threads", default="1,16")
    args = ap.parse_args()
    out = {"batches": list(BATCHES), "rows": []}
    combos = [(int(L), int(nt)) for L in args.lengths.split(",") for nt in args.threads.split(",")]
    # CPU rows first: their worker processes are forked before this process
    # touches the GPU
    cpu_rows = {(L, nt): {"cpu_reference_est": cpu_reference_est(L, nt, max(2.0, 3 * args.seconds)),
                          "cpu_openssl": cpu_openssl(L, nt, max(1.0, args.seconds))} for L, nt in combos}
    for L, nt in combos:
        row = {"plaintext_bytes": L, "threads": nt, **cpu_rows[(L, nt)]}
        row["gpu_token_call"] = gpu_token_call(L, nt, args.seconds)
        row["gpu_batch"] = {str(B): gpu_batch(L, B, nt, args.seconds) for B in BATCHES}
        for name in ("cpu_reference_est", "cpu_openssl", "gpu_token_call"):
            if row[name] is None:
                continue
            cpu = row[name]["round_trips_s"]
            win = [B for B in BATCHES if row["gpu_batch"][str(B)]["round_trips_s"] > cpu]
            row.setdefault("crossover_batch", {})[name] = win[0] if win else None
        print(json.dumps({"L": L, "threads": nt,
                          "ref": round(row["cpu_reference_est"]["round_trips_s"]),
                          "openssl": round((row["cpu_openssl"] or {}).get("round_trips_s", 0)),
                          "token_call": round(row["gpu_token_call"]["round_trips_s"]),
                          "batch": {B: round(v["round_trips_s"]) for B, v in row["gpu_batch"].items()},
                          "crossover": row.get("crossover_batch")}), flush=True)
        out["rows"].append(row)
    out["note"] = __doc__
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
