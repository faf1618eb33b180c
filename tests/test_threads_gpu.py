"""Concurrency: the reference calls Token from interface reader threads and
application threads at once (SURVEY §8(b) Threading; TCPInterface.py:175,294
-> Transport.inbound -> Link.receive, plus Resource/Channel threads), with one
cached Token per link shared between them (Link.py:1163-1164,1177).

Eight Python threads (ctypes releases the GIL inside every librnstok call)
mix every host entry point on one context: per-packet Tokens created and
dropped, one shared Token, KeySet batches with per-packet keys, verify,
HKDF and device-derived key sets, while a ninth thread keeps the device API
busy on its own torch stream.  Every result is checked against the C oracle
(bit-exact); any exception or mismatch in any thread fails the test.
"""
import hashlib
import hmac
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from oracle import ctoken as oracle

pytestmark = pytest.mark.gpu

N_THREADS = 8
ITERS = 120


@pytest.fixture(scope="module")
def rt():
    import reticulum_amd
    from reticulum_amd import _native
    _native.context(0)        # raises loudly if the HIP path is unusable
    return reticulum_amd


def _worker(rt, tid, shared_key, shared_token):
    rng = np.random.Generator(np.random.PCG64(4242 + tid))
    rb = lambda k: rng.integers(0, 256, k, dtype=np.uint8).tobytes()  # noqa: E731
    done = 0
    for it in range(ITERS):
        op = (it + tid) % 7
        if op == 0:                                   # Identity.encrypt-style: one Token per packet
            key, msg = rb(64 if it % 2 else 32), rb(int(rng.integers(0, 700)))
            tok = rt.Token(key).encrypt(msg)
            assert oracle.decrypt(key, tok) == (0, msg)
        elif op == 1:                                 # decrypt of an oracle token
            key, msg, iv = rb(64), rb(int(rng.integers(0, 1500))), rb(16)
            assert rt.Token(key).decrypt(oracle.encrypt(key, iv, msg)) == msg
        elif op == 2:                                 # the link's cached Token, shared by all threads
            msg = rb(int(rng.integers(0, 500)))
            tok = shared_token.encrypt(msg)
            assert shared_token.decrypt(tok) == msg
            assert oracle.decrypt(shared_key, tok) == (0, msg)
        elif op == 3:                                 # a batch with per-packet keys
            nk, n = int(rng.integers(1, 50)), int(rng.integers(1, 200))
            keys = rng.integers(0, 256, (nk, 64), dtype=np.uint8)
            kidx = rng.integers(0, nk, n).astype(np.uint32)
            msgs = [rb(int(rng.integers(0, 2000))) for _ in range(n)]
            ks = rt.KeySet(keys)
            toks = ks.encrypt_batch(msgs, key_idx=kidx)
            back, st = ks.decrypt_batch(toks, key_idx=kidx)
            assert (st == 0).all() and back.to_list() == msgs
            j = int(rng.integers(0, n))
            assert oracle.decrypt(keys[kidx[j]].tobytes(), toks[j]) == (0, msgs[j])
        elif op == 4:                                 # verify_hmac, valid and tampered
            key, msg = rb(64), rb(int(rng.integers(0, 300)))
            t = rt.Token(key)
            tok = bytearray(oracle.encrypt(key, rb(16), msg))
            assert t.verify_hmac(bytes(tok))
            tok[int(rng.integers(0, len(tok)))] ^= 0x10
            assert not t.verify_hmac(bytes(tok))
        elif op == 5:                                 # HKDF (Identity key derivation)
            ikm, salt = rb(32), rb(16)
            assert rt.hkdf(64, ikm, salt) == oracle.hkdf(64, ikm, salt)
        else:                                         # device-derived per-packet key set
            n = int(rng.integers(1, 300))
            ikm = rng.integers(0, 256, (n, 32), dtype=np.uint8)
            salt = rb(16)
            ks = rt.derive_keyset(ikm, salt)
            msgs = [rb(int(rng.integers(0, 400))) for _ in range(n)]
            kidx = np.arange(n, dtype=np.uint32)
            toks = ks.encrypt_batch(msgs, key_idx=kidx)
            j = int(rng.integers(0, n))
            key = oracle.hkdf(64, ikm[j].tobytes(), salt)
            assert oracle.decrypt(key, toks[j]) == (0, msgs[j])
            tag = hmac.new(key[:32], toks[j][:-32], hashlib.sha256).digest()
            assert tag == toks[j][-32:]
        done += 1
    return done


def _device_worker(rt, stop):
    """c2-shaped launches on a private stream until the host threads finish."""
    import torch
    from reticulum_amd import device
    n, L = 1 << 16, 500
    tl = rt.token_len(L)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        g = torch.Generator(device="cuda").manual_seed(3)
        pt = torch.randint(0, 256, (n, L), dtype=torch.uint8, device="cuda", generator=g)
        iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
        ks = rt.KeySet(bytes(range(64)))
        ref = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
        device.encrypt_uniform(ks, pt, L, iv, ref, stream=s)
        out = torch.empty_like(ref)
        back = torch.empty((n, tl - 48), dtype=torch.uint8, device="cuda")
        ol = torch.empty(n, dtype=torch.int32, device="cuda")
        st = torch.empty(n, dtype=torch.int32, device="cuda")
        rounds = 0
        bad = torch.zeros((), dtype=torch.int64, device="cuda")
        while not stop.is_set() or rounds < 5:
            device.encrypt_uniform(ks, pt, L, iv, out, stream=s)
            device.decrypt_uniform(ks, out, tl, back, ol, st, stream=s)
            bad += (out != ref).any(dim=1).sum() + (back[:, :L] != pt).any(dim=1).sum() + st.abs().sum()
            rounds += 1
            if rounds % 8 == 0:
                s.synchronize()
        s.synchronize()
    # the first token against the oracle, so the reference itself is checked
    t0 = ref[0].cpu().numpy().tobytes()
    assert oracle.decrypt(bytes(range(64)), t0) == (0, pt[0].cpu().numpy().tobytes())
    return rounds, int(bad)


def test_threads_share_one_context(rt):
    shared_key = bytes(range(100, 164))
    shared_token = rt.Token(shared_key)
    oracle.decrypt(shared_key, oracle.encrypt(shared_key, bytes(16), b""))   # oracle tables built once
    stop = threading.Event()
    with ThreadPoolExecutor(N_THREADS + 1) as ex:
        dev = ex.submit(_device_worker, rt, stop)
        try:
            futs = [ex.submit(_worker, rt, t, shared_key, shared_token) for t in range(N_THREADS)]
            counts = [f.result(timeout=100) for f in futs]
        finally:
            stop.set()
        rounds, bad = dev.result(timeout=60)
    assert counts == [ITERS] * N_THREADS
    assert rounds >= 5 and bad == 0
