"""One packet per host call, the shape of every Token.encrypt / Token.decrypt
(Token.py:87-114, called per packet from Link.py:1161-1182): rt_encrypt_host /
rt_decrypt_host with n = 1 run the token kernel on the staging lane's mapped
pinned buffer itself, with no copy kernel in and no store kernel out
(RNSTOK_HOST_DIRECT, csrc/token_capi.hip).

Bit-exact against the C oracle over a length sweep on one key set (each call's
inputs replace the previous call's in the same staging buffer, so stale data
would show), at nonzero offsets inside caller buffers whose other bytes must
survive, with per-packet keys and AES-128 keys, and on tampered, truncated and
malformed tokens.
"""
import ctypes

import numpy as np
import pytest

from oracle import ctoken as oracle

pytestmark = pytest.mark.gpu

LENGTHS = [0, 1, 15, 16, 17, 63, 64, 100, 383, 500, 1000, 4096, 16384]


@pytest.fixture(scope="module")
def rt():
    import reticulum_amd
    from reticulum_amd import _native
    lib = _native.load()
    assert lib.rt_device_count() >= 1, "no HIP device visible"
    _native.context(0)
    return reticulum_amd


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _check(rc):
    from reticulum_amd import _native
    _native.check(rc)


def _encrypt_one(ks, pt_buf, pt_off, L, iv, tok_buf, tok_off, kidx=None):
    po, pl, to = np.array([pt_off], np.uint64), np.array([L], np.uint32), np.array([tok_off], np.uint64)
    ki = None if kidx is None else np.array([kidx], np.uint32)
    _check(ks._lib.rt_encrypt_host(ks.handle, _p(pt_buf), _p(po), _p(pl), None if ki is None else _p(ki), _p(iv),
                                   _p(tok_buf), _p(to), 1))


def _decrypt_one(ks, tok_buf, tok_off, T, out, out_off, kidx=None):
    to, tl, oo = np.array([tok_off], np.uint64), np.array([T], np.uint32), np.array([out_off], np.uint64)
    ol, st = np.full(1, 0xFFFFFFFF, np.uint32), np.full(1, -7, np.int32)
    ki = None if kidx is None else np.array([kidx], np.uint32)
    _check(ks._lib.rt_decrypt_host(ks.handle, _p(tok_buf), _p(to), _p(tl), None if ki is None else _p(ki), _p(out),
                                   _p(oo), _p(ol), _p(st), 1))
    return int(st[0]), int(ol[0])


def _oracle_decrypt_one(keys, tok_buf, tok_off, T, cap, kidx=None):
    want = np.zeros(max(cap, 1), np.uint8)
    wl, ws = np.zeros(1, np.uint32), np.zeros(1, np.int32)
    oracle.decrypt_batch(keys, tok_buf, np.array([tok_off], np.uint64), np.array([T], np.uint32),
                         None if kidx is None else np.array([kidx], np.uint32), want, np.zeros(1, np.uint64), wl, ws,
                         threads=1)
    return int(ws[0]), int(wl[0]), want


@pytest.mark.parametrize("klen,n_keys", [(64, 1), (32, 1), (64, 5)])
def test_one_packet_calls_sweep_vs_oracle(rt, klen, n_keys):
    rng = np.random.Generator(np.random.PCG64(4100 + klen + n_keys))
    keys = rng.integers(0, 256, (n_keys, klen), dtype=np.uint8)
    ks = rt.KeySet(keys if n_keys > 1 else keys[0].tobytes())
    for rep in range(2):
        for L in LENGTHS:
            kidx = int(rng.integers(0, n_keys)) if n_keys > 1 else None
            T = rt.token_len(L)
            po, to, oo = (int(x) for x in rng.integers(0, 40, 3))
            pt_buf = rng.integers(0, 256, po + L + 7, dtype=np.uint8)
            iv = rng.integers(0, 256, 16, dtype=np.uint8)
            tok = np.full(to + T + 9, 0x5A, np.uint8)
            ref = tok.copy()
            oracle.encrypt_batch(keys, pt_buf, np.array([po], np.uint64), np.array([L], np.uint32),
                                 None if kidx is None else np.array([kidx], np.uint32), iv.reshape(1, 16), ref,
                                 np.array([to], np.uint64), threads=1)
            _encrypt_one(ks, pt_buf, po, L, iv, tok, to, kidx)
            assert np.array_equal(tok, ref), (klen, n_keys, L, rep)

            out = np.full(oo + (T - 48) + 5, 0xC3, np.uint8)
            st, ol = _decrypt_one(ks, tok, to, T, out, oo, kidx)
            assert (st, ol) == (rt.RT_ST_OK, L), (klen, n_keys, L, rep)
            assert np.array_equal(out[oo:oo + L], pt_buf[po:po + L])
            assert (out[:oo] == 0xC3).all() and (out[oo + T - 48:] == 0xC3).all()


def test_one_packet_bad_tokens_vs_oracle(rt):
    """Tampered, truncated and malformed single tokens: the oracle's status;
    the caller's region (tok_len - 48 bytes) zeroed, the bytes around it kept."""
    rng = np.random.Generator(np.random.PCG64(4200))
    key = rng.integers(0, 256, 64, dtype=np.uint8)
    ks = rt.KeySet(key.tobytes())
    tok = ks.encrypt_batch([rng.integers(0, 256, 383, dtype=np.uint8).tobytes()])[0]
    cases = []
    for pos in (0, 17, len(tok) - 40, len(tok) - 1):              # iv, ciphertext, last block, tag
        b = bytearray(tok)
        b[pos] ^= 0x10
        cases.append(bytes(b))
    cases += [tok[:k] for k in (0, 20, 32, 33, 48, 63, 64, 70, len(tok) - 16)]
    seen = set()
    for t in cases:
        T = len(t)
        to, oo = (int(x) for x in rng.integers(0, 40, 2))
        tok_buf = np.zeros(to + max(T, 1) + 3, np.uint8)
        tok_buf[to:to + T] = np.frombuffer(t, np.uint8)
        cap = max(T - 48, 0)
        want_st, want_len, _ = _oracle_decrypt_one(key.reshape(1, 64), tok_buf, to, T, cap)
        out = np.full(oo + cap + 5, 0xC3, np.uint8)
        st, ol = _decrypt_one(ks, tok_buf, to, T, out, oo)
        assert st == want_st, (T, st, want_st)
        seen.add(st)
        if st != rt.RT_ST_BAD_PAD:
            assert ol == (want_len if st == rt.RT_ST_OK else 0), (T, ol)
        if st != rt.RT_ST_OK:
            assert (out[oo:oo + cap] == 0).all(), T
        assert (out[:oo] == 0xC3).all() and (out[oo + cap:] == 0xC3).all(), T
    assert rt.RT_ST_BAD_HMAC in seen and len(seen) >= 2
