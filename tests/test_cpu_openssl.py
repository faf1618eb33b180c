"""Pin the "strong CPU" baseline (tools/cpu_openssl.c, OpenSSL libcrypto; not
the reference path) to the golden vectors generated
from the reference, so the row bench.py reports times the same token."""
import ctypes
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tools", "libcpu_openssl.so")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.skip("tools/libcpu_openssl.so not built (__graft_entry__.build)")
    lib = ctypes.CDLL(LIB)
    lib.cpu_openssl_token.restype = ctypes.c_int
    lib.cpu_openssl_token.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                      ctypes.c_char_p]
    lib.cpu_openssl_run.restype = ctypes.c_double
    lib.cpu_openssl_run.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
    return lib


def test_openssl_token_matches_golden_vectors(lib, golden):
    n = 0
    for v in golden["encrypt"]:
        key, iv, pt = (bytes.fromhex(v[k]) for k in ("key", "iv", "pt"))
        if len(key) != 64:          # the baseline covers the AES-256 token only
            continue
        out = ctypes.create_string_buffer(16 + 16 * (len(pt) // 16 + 1) + 32)
        r = lib.cpu_openssl_token(key, iv, pt, len(pt), out)
        assert r == len(out) and out.raw.hex() == v["token"]
        n += 1
    assert n >= 80


def test_openssl_round_trip_run(lib):
    done = ctypes.c_uint64()
    rate = lib.cpu_openssl_run(2, 0.2, 500, ctypes.byref(done))
    assert rate > 0 and done.value > 0
