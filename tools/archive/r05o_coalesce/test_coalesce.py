"""Group-committed Token calls (reticulum_amd.coalesce.CoalescingToken):
many threads calling encrypt / decrypt / verify_hmac on tokens of different
keys (AES-256 and AES-128) get exactly Token's results and exceptions
(Token.py:77-114), checked against the C oracle; an uncontended call is a
batch of one; under contention the calls share batches.  CPU suite: the
library is stood in for by tests/fake_native.py (the oracle behind the same
entry points); tests/test_coalesce_gpu.py runs the same on the kernels."""
import os
import threading

import numpy as np
import pytest

from oracle import ctoken

import fake_native


def _check_thread(tok_cls, key, seed, n, errors, barrier=None):
    import reticulum_amd as rt
    rng = np.random.Generator(np.random.PCG64(seed))
    t = tok_cls(key)
    if barrier is not None:
        barrier.wait()
    try:
        for i in range(n):
            L = int(rng.integers(0, 700))
            pt = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
            tok = t.encrypt(pt)
            assert len(tok) == rt.token_len(L)
            s, p = ctoken.decrypt(key, tok)                     # the oracle opens it
            assert s == 0 and p == pt
            assert t.decrypt(tok) == pt
            assert t.verify_hmac(tok) is True
            bad = bytearray(tok)
            bad[int(rng.integers(0, len(bad)))] ^= 1 << int(rng.integers(0, 8))
            with pytest.raises(ValueError, match="Token HMAC was invalid"):
                t.decrypt(bytes(bad))
            assert t.verify_hmac(bytes(bad)) is False
            with pytest.raises(ValueError, match="Cannot verify HMAC on token of only 20 bytes"):
                t.decrypt(bytes(20))
            with pytest.raises(TypeError):
                t.encrypt(bytearray(pt))
    except BaseException as exc:                                # noqa: BLE001 (reported to the main thread)
        errors.append(exc)


def _run_threads(tok_cls, n_threads, n_each):
    keys = [os.urandom(64 if i % 3 else 32) for i in range(n_threads)]
    errors = []
    barrier = threading.Barrier(n_threads)
    th = [threading.Thread(target=_check_thread, args=(tok_cls, keys[i], 500 + i, n_each, errors, barrier))
          for i in range(n_threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    if errors:
        raise errors[0]


def test_coalesced_calls_from_many_threads_match_token(monkeypatch):
    fake_native.install(monkeypatch)
    from reticulum_amd import coalesce
    monkeypatch.setattr(coalesce, "_coalescers", {})
    _run_threads(coalesce.CoalescingToken, 12, 15)
    st = coalesce.coalescer().stats
    assert st["calls"] == 12 * 15 * 5                           # encrypt, decrypt, verify, bad decrypt, bad verify
    assert st["batches"] <= st["calls"]


def test_uncontended_call_is_a_batch_of_one(monkeypatch):
    fake = fake_native.install(monkeypatch)
    from reticulum_amd import coalesce
    monkeypatch.setattr(coalesce, "_coalescers", {})
    key = os.urandom(64)
    t = coalesce.CoalescingToken(key)
    tok = t.encrypt(b"hello")
    assert t.decrypt(tok) == b"hello"
    st = coalesce.coalescer().stats
    assert (st["calls"], st["batches"], st["key_tables"]) == (2, 2, 0)      # the plain Token calls
    assert [c for c in fake.calls if c[0] in ("encrypt", "decrypt")] == [("encrypt", 1), ("decrypt", 1)]


def test_queued_calls_share_one_batch(monkeypatch):
    """Calls queued while a leader's batch runs go into the next leader's
    batch together (group commit)."""
    fake = fake_native.install(monkeypatch)
    from reticulum_amd import coalesce
    c = coalesce.Coalescer(leaders=1)
    gate, entered = threading.Event(), threading.Event()
    orig = fake.rt_encrypt_host

    def slow(*a):
        entered.set()
        gate.wait(10)
        return orig(*a)
    monkeypatch.setattr(fake, "rt_encrypt_host", slow)
    key = os.urandom(64)
    tok = coalesce.CoalescingToken(key)
    out = {}
    first = threading.Thread(target=lambda: out.setdefault("first", c.run(coalesce._ENC, coalesce.CoalescingToken(key), b"a")))
    first.start()
    assert entered.wait(10)
    rest = [threading.Thread(target=lambda i=i: out.setdefault(i, c.run(coalesce._ENC, tok, bytes([i]) * i)))
            for i in range(1, 9)]
    for x in rest:
        x.start()
    while len(c._queue) < 8:                                     # all eight queued behind the leader
        threading.Event().wait(0.01)
    gate.set()
    first.join()
    for x in rest:
        x.join()
    assert (c.stats["calls"], c.stats["batches"]) == (9, 2)
    assert [n for op, n in fake.calls if op == "encrypt"] == [1, 8]
    for i in range(1, 9):
        s, p = ctoken.decrypt(key, out[i])
        assert s == 0 and p == bytes([i]) * i


def test_key_table_is_rebuilt_only_for_new_keys(monkeypatch):
    fake_native.install(monkeypatch)
    from reticulum_amd import coalesce
    c = coalesce.Coalescer(max_keys=3)
    keys = [os.urandom(64) for _ in range(5)]
    toks = [coalesce.CoalescingToken(k) for k in keys]
    for a, b in ((0, 1), (1, 2), (2, 0)):                        # batches of two (a batch of one is the plain call)
        c._execute([coalesce._Call(coalesce._ENC, toks[a], b"x"), coalesce._Call(coalesce._ENC, toks[b], b"x")])
    assert c.stats["key_tables"] == 2                            # built for keys 0, 1; rebuilt for key 2
    calls = [coalesce._Call(coalesce._ENC, toks[i % 3], b"y") for i in range(6)]
    c._execute(calls)
    for i, cl in enumerate(calls):
        assert ctoken.decrypt(keys[i % 3], cl.result) == (0, b"y")
    assert c.stats["key_tables"] == 2                            # known keys: no rebuild
    c._execute([coalesce._Call(coalesce._ENC, toks[3], b"z"), coalesce._Call(coalesce._ENC, toks[4], b"z")])
    assert c.stats["key_tables"] == 3 and list(c._tables[64][1]) == [keys[3], keys[4]]   # past max_keys: restart


def test_type_and_key_errors_as_token():
    from reticulum_amd.coalesce import CoalescingToken
    with pytest.raises(ValueError, match="Token key cannot be None"):
        CoalescingToken(None)
    with pytest.raises(ValueError, match="Token key must be 128 or 256 bits, not 384"):
        CoalescingToken(bytes(48))
