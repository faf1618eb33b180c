"""Pin the oracle: the C restatement and the pure-Python restatement against
the golden vectors generated from the reference (tests/golden/gen_golden.py),
the reference's own token KAT (tests/identity.py:11-19,148-158) and the
SHA-256 KATs of tests/hashes.py:12-30."""
import hashlib

import numpy as np
import pytest

from oracle import cpuref
from oracle import ctoken


def b(h):
    return bytes.fromhex(h)


def test_c_oracle_encrypt_vectors(golden):
    for v in golden["encrypt"]:
        tok = ctoken.encrypt(b(v["key"]), b(v["iv"]), b(v["pt"]))
        assert tok.hex() == v["token"]
        st, pt = ctoken.decrypt(b(v["key"]), tok)
        assert st == 0 and pt.hex() == v["pt"]


def test_c_oracle_decrypt_cases(golden):
    for c in golden["decrypt"]:
        st, pt = ctoken.decrypt(b(c["key"]), b(c["token"]))
        assert st == c["status"], c["name"]
        assert (pt.hex() if pt is not None else None) == c["pt"], c["name"]


def test_c_oracle_reference_kat(golden):
    k = golden["kat"]["fixed_token"]
    st, pt = ctoken.decrypt(b(k["derived_key"]), b(k["token"]))
    assert st == 0 and pt.hex() == k["pt"]


def test_c_oracle_sha_hmac_kats(golden):
    for v in golden["kat"]["sha256"]:
        msg = b(v["msg_repeat"][0]) * v["msg_repeat"][1] if "msg_repeat" in v else b(v["msg"])
        assert ctoken.sha256(msg).hex() == v["digest"]
    for v in golden["kat"]["hmac_sha256"]:
        assert ctoken.hmac_sha256(b(v["key"]), b(v["msg"])).hex() == v["mac"]


def test_c_oracle_batch_matches_single(golden):
    rng = np.random.Generator(np.random.PCG64(9))
    n = 200
    keys = rng.integers(0, 256, (5, 64), dtype=np.uint8)
    lens = rng.integers(0, 700, n).astype(np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    buf = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    ivs = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    kidx = rng.integers(0, 5, n).astype(np.uint32)
    tl = (16 + 16 * (lens // 16 + 1) + 32).astype(np.uint32)
    toff = np.zeros(n, np.uint64)
    toff[1:] = np.cumsum(tl[:-1].astype(np.uint64))
    tok = np.zeros(int(tl.sum()), np.uint8)
    ctoken.encrypt_batch(keys, buf, off, lens, kidx, ivs, tok, toff, threads=4)
    for i in range(n):
        one = ctoken.encrypt(keys[kidx[i]].tobytes(), ivs[i].tobytes(), buf[off[i]:off[i] + lens[i]].tobytes())
        assert tok[toff[i]:toff[i] + tl[i]].tobytes() == one
    pt = np.zeros(int(tl.sum()), np.uint8)
    plen = np.zeros(n, np.uint32)
    st = np.zeros(n, np.int32)
    poff = toff.copy()
    ctoken.decrypt_batch(keys, tok, toff, tl, kidx, pt, poff, plen, st, threads=4)
    assert (st == 0).all() and np.array_equal(plen, lens)


def test_cpuref_vectors(golden):
    for v in golden["encrypt"]:
        if len(v["pt"]) > 2 * 5000:
            continue           # keep the pure-Python check fast
        tok = cpuref.encrypt(b(v["key"]), b(v["iv"]), b(v["pt"]))
        assert tok.hex() == v["token"]
        st, pt = cpuref.decrypt(b(v["key"]), tok)
        assert st == 0 and pt.hex() == v["pt"]
    for c in golden["decrypt"]:
        st, pt = cpuref.decrypt(b(c["key"]), b(c["token"]))
        assert st == c["status"], c["name"]
        assert (pt.hex() if pt is not None else None) == c["pt"]


def test_cpuref_hmac_matches_hashlib(golden):
    for v in golden["kat"]["hmac_sha256"]:
        assert cpuref.hmac_sha256(b(v["key"]), b(v["msg"])).hex() == v["mac"]
    assert hashlib.sha256(b"abc").hexdigest() == golden["kat"]["sha256"][1]["digest"]


def test_cpuref_sbox_is_derived_and_matches_c():
    assert bytes(cpuref.SBOX) == ctoken.sbox()
    assert cpuref.SBOX[0] == 0x63 and cpuref.SBOX[0x53] == 0xED   # FIPS-197 §5.1.1 example


@pytest.mark.parametrize("klen", [32, 64])
def test_oracles_agree_random(klen):
    rng = np.random.Generator(np.random.PCG64(klen))
    for L in list(range(0, 40)) + [100, 255, 256, 500, 1000]:
        key = rng.integers(0, 256, klen, dtype=np.uint8).tobytes()
        iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        pt = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        assert ctoken.encrypt(key, iv, pt) == cpuref.encrypt(key, iv, pt)
