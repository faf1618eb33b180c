"""Calibrate oracle/cpuref.py against the reference on the same core.

Runs ONLY in the build container (imports /root/reference).  Prints
ratio = cpuref_rate / reference_rate for 500 B encrypt and decrypt
(BASELINE.md §3 step 3); the result is recorded in DESIGN.md.
"""
import os
import sys
import time

sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(1, "/root/reference")

import RNS.Cryptography  # noqa: E402
from oracle import cpuref  # noqa: E402

Token = sys.modules["RNS.Cryptography.Token"].Token


def rate(fn, secs=4.0):
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < secs:
        fn()
        n += 1
    return n / (time.perf_counter() - t0)


def main():
    key, pt, iv = os.urandom(64), os.urandom(500), os.urandom(16)
    tok_ref = Token(key).encrypt(pt)
    tok_cpu = cpuref.encrypt(key, iv, pt)
    r_enc = rate(lambda: Token(key).encrypt(pt))
    c_enc = rate(lambda: cpuref.encrypt(key, iv, pt))
    r_dec = rate(lambda: Token(key).decrypt(tok_ref))
    c_dec = rate(lambda: cpuref.decrypt(key, tok_cpu))
    print(f"reference enc {r_enc:.1f} pkt/s dec {r_dec:.1f} pkt/s (backend {RNS.Cryptography.backend()})")
    print(f"cpuref    enc {c_enc:.1f} pkt/s dec {c_dec:.1f} pkt/s")
    print(f"ratio enc {c_enc / r_enc:.3f} dec {c_dec / r_dec:.3f}")


if __name__ == "__main__":
    main()
