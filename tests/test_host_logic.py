"""Host-layer tests of reticulum_amd.Token / KeySet / Packed on CPU.

The HIP library is replaced by tests/fake_native.py (C oracle behind the same
entry points) so that argument marshalling, the key split, the exception
classes and messages of RNS/Cryptography/Token.py:58-114 are checked without
a GPU.  The same assertions run against the real kernels in test_token_gpu.py.
"""
import numpy as np
import pytest

import reticulum_amd as rt
from tests_helpers import b, trial_case


@pytest.fixture
def fake(monkeypatch):
    import fake_native
    return fake_native.install(monkeypatch)


def test_token_constants_and_generate_key():
    assert rt.Token.TOKEN_OVERHEAD == 48
    assert len(rt.Token.generate_key()) == 64
    assert len(rt.Token.generate_key(rt.AES_128_CBC)) == 32
    with pytest.raises(TypeError):
        rt.Token.generate_key("bogus")


def test_key_errors_match_reference(golden):
    for e in golden["kat"]["key_errors"]:
        key = None if e["key_len"] is None else bytes(e["key_len"])
        with pytest.raises({"ValueError": ValueError, "TypeError": TypeError}[e["exc"]]) as ex:
            rt.Token(key)
        assert str(ex.value) == e["msg"]
    with pytest.raises(TypeError):
        rt.Token(bytes(64), mode="AES_9")


def test_key_split(fake):
    t = rt.Token(bytes(range(64)))
    assert t.mode is rt.AES_256_CBC and t._signing_key == bytes(range(32)) and t._encryption_key == bytes(range(32, 64))
    t = rt.Token(bytes(range(32)))
    assert t.mode is rt.AES_128_CBC and t._signing_key == bytes(range(16))


def test_type_errors_match_reference(golden, fake):
    t = rt.Token(bytes(64))
    for e in golden["kat"]["type_errors"]:
        arg = bytearray(b"x") if e["arg_type"] == "bytearray" else "str"
        with pytest.raises(TypeError) as ex:
            getattr(t, e["method"])(arg)
        assert str(ex.value) == e["msg"]
    assert fake.calls == []          # rejected before reaching the library


def test_golden_through_host_layer(golden, fake):
    for v in golden["encrypt"][:60]:
        ks = rt.KeySet(b(v["key"]))
        toks = ks.encrypt_batch([b(v["pt"])], ivs=np.frombuffer(b(v["iv"]), np.uint8))
        assert toks[0].hex() == v["token"]


def test_decrypt_messages_through_host_layer(golden, fake):
    for c in golden["decrypt"]:
        t = rt.Token(b(c["key"]))
        if c["status"] == 0:
            assert t.decrypt(b(c["token"])).hex() == c["pt"]
        else:
            with pytest.raises(ValueError) as ex:
                t.decrypt(b(c["token"]))
            assert str(ex.value) == c["msg"], c["name"]


def test_verify_hmac(golden, fake):
    k = golden["kat"]["fixed_token"]
    t = rt.Token(b(k["derived_key"]))
    tok = b(k["token"])
    assert t.verify_hmac(tok)
    assert not t.verify_hmac(tok[:-1] + bytes([tok[-1] ^ 1]))
    with pytest.raises(ValueError):
        t.verify_hmac(bytes(32))


def test_packed_layout_roundtrip(fake):
    items = [b"", b"a", bytes(range(200)), b"z" * 17]
    p = rt.Packed.from_list(items)
    assert p.to_list() == items and list(p.off) == [0, 0, 1, 201]
    ks = rt.KeySet([bytes(64), bytes(range(64))])
    toks = ks.encrypt_batch(items, key_idx=[1, 0, 1, 0])
    assert list(toks.length) == [rt.token_len(len(x)) for x in items]
    back, st = ks.decrypt_batch(toks, key_idx=[1, 0, 1, 0])
    assert list(st) == [0] * 4 and back.to_list() == items
    _, st = ks.decrypt_batch(toks, key_idx=[0, 1, 0, 1])
    assert list(st) == [rt.RT_ST_BAD_HMAC] * 4


def test_batch_argument_validation(fake):
    ks = rt.KeySet(bytes(64))
    with pytest.raises(ValueError):
        ks.encrypt_batch([b"x"], ivs=np.zeros(8, np.uint8))
    with pytest.raises(ValueError):
        ks.encrypt_batch([b"x"], key_idx=[3])
    with pytest.raises(ValueError):
        rt.KeySet([bytes(64), bytes(32)])
    with pytest.raises(ValueError):
        rt.KeySet(bytes(48))


def test_fresh_iv_per_token(fake):
    t = rt.Token(bytes(64))
    a, c = t.encrypt(b"same"), t.encrypt(b"same")
    assert a[:16] != c[:16] and t.decrypt(a) == t.decrypt(c) == b"same"


def test_verify_trials_host_layer(fake):
    """KeySet.verify_trials / decrypt_trials: the CSR the library receives and
    the first-opening key it returns, per the reference's ratchet loop
    (Identity.py:865-878); a token under none of its candidates stays closed."""
    keys, toks, cands, expect = trial_case(5)
    ks = rt.KeySet(keys)
    got = ks.verify_trials(toks, cands)
    assert got.tolist() == expect.tolist()
    pts, st, used = ks.decrypt_trials(toks, cands)
    assert used.tolist() == [e if s == rt.RT_ST_OK else -1 for e, s in zip(expect.tolist(), st.tolist())]
    assert all(st[i] == rt.RT_ST_BAD_HMAC for i in range(len(toks)) if expect[i] < 0)
    assert ks.verify_trials([], []).size == 0
    with pytest.raises(ValueError):
        ks.verify_trials(toks[:2], cands[:1])
    with pytest.raises(ValueError):
        ks.verify_trials(toks[:1], [[len(keys)]])


def test_verify_hmac_goldens_host_layer(golden, fake):
    """verify_hmac runs the verify-only entry point (rt_verify_host, no
    decrypt): True wherever the reference's tag check passes, including
    tokens decrypt rejects afterwards (len40_validtag, ct_not_mult16)."""
    for c in golden["decrypt"]:
        t = rt.Token(b(c["key"]))
        if c["status"] == 1:
            with pytest.raises(ValueError):
                t.verify_hmac(b(c["token"]))
        else:
            assert t.verify_hmac(b(c["token"])) is (c["status"] != 2), c["name"]
    assert any(call[0] == "verify" for call in fake.calls)
    assert not any(call[0] == "decrypt" for call in fake.calls)
    ks = rt.KeySet(b(golden["decrypt"][0]["key"]))
    st = ks.verify_batch([b(c["token"]) for c in golden["decrypt"] if c["key"] == golden["decrypt"][0]["key"]])
    assert st.dtype == np.int32 and set(st.tolist()) <= {0, 1, 2}


def test_device_api_validates_before_launch():
    """reticulum_amd.device rejects rows narrower than the packet/token and
    length/status/key arrays of the wrong dtype or size before any launch
    (ADVICE r01): the kernels would otherwise write past a row or read int64
    words as pairs of int32."""
    import torch
    from reticulum_amd import device
    n, L = 4, 100
    tl = rt.token_len(L)
    ks = object()
    pt = torch.zeros((n, L), dtype=torch.uint8)
    iv = torch.zeros((n, 16), dtype=torch.uint8)
    with pytest.raises(ValueError, match="tok rows"):
        device.encrypt_uniform(ks, pt, L, iv, torch.zeros((n, tl - 1), dtype=torch.uint8))
    with pytest.raises(ValueError, match="pt rows"):
        device.encrypt_uniform(ks, pt[:, :50], L, iv, torch.zeros((n, tl), dtype=torch.uint8))
    with pytest.raises(ValueError, match="tok rows"):
        device.encrypt_uniform(ks, pt[:1], L, iv[:1], torch.zeros((1, 16), dtype=torch.uint8))
    with pytest.raises(ValueError, match="key_idx"):
        device.encrypt_uniform(ks, pt, L, iv, torch.zeros((n, tl), dtype=torch.uint8),
                               key_idx=torch.zeros(n, dtype=torch.int64))
    tok = torch.zeros((n, tl), dtype=torch.uint8)
    ok32 = torch.zeros(n, dtype=torch.int32)
    with pytest.raises(ValueError, match="pt rows"):
        device.decrypt_uniform(ks, tok, tl, torch.zeros((n, tl - 49), dtype=torch.uint8), ok32, ok32)
    with pytest.raises(ValueError, match="status"):
        device.decrypt_uniform(ks, tok, tl, torch.zeros((n, tl - 48), dtype=torch.uint8), ok32,
                               torch.zeros(n, dtype=torch.int64))
    with pytest.raises(ValueError, match="key_idx"):
        device.decrypt_uniform(ks, tok, tl, torch.zeros((n, tl - 48), dtype=torch.uint8), ok32, ok32,
                               key_idx=torch.zeros(n + 1, dtype=torch.int32))
    with pytest.raises(ValueError, match="pt_off"):
        device.encrypt(ks, pt.reshape(-1), torch.zeros(n, dtype=torch.int32), ok32, iv, tok.reshape(-1),
                       torch.zeros(n, dtype=torch.int64))
    with pytest.raises(ValueError, match="tok_len"):
        device.verify(ks, tok.reshape(-1), torch.zeros(n, dtype=torch.int64), torch.zeros(n, dtype=torch.int64),
                      ok32)
