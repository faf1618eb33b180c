"""Seeded fuzz of the device entry points against the C oracle.

Each case draws its own batch shape: a mixture of lengths (empty, every tail
shape, c2-sized, long-token sized), one key or many, AES-256 or AES-128
keys, packets placed in shuffled order with gaps in the buffer (offsets not
ascending), sorted or unsorted launches, and a decrypt batch that mixes
valid tokens with bit-flipped ones, truncated ones (< 48 B and ragged
lengths) and crafted tokens whose HMAC is valid but whose body is not
(ciphertext length not a multiple of 16, bad PKCS7 padding).  Tokens,
statuses, output lengths and plaintexts must equal the oracle's
(oracle_encrypt_batch / oracle_decrypt_batch, which follow Token.py:86-130),
and rt_verify must agree with the oracle's status on the tag check.
Bit-exact throughout.
"""
import hashlib
import hmac

import numpy as np
import pytest

from oracle import ctoken as oracle

pytestmark = pytest.mark.gpu

N_CASES = 48


@pytest.fixture(scope="module")
def rt():
    import reticulum_amd
    from reticulum_amd import _native
    _native.context(0)        # raises loudly if the HIP path is unusable
    return reticulum_amd


def _lengths(rng, n):
    kind = rng.integers(0, 4, n)
    lens = np.where(kind == 0, rng.integers(0, 48, n),
                    np.where(kind == 1, rng.integers(48, 700, n),
                             np.where(kind == 2, 500, rng.integers(700, 4200, n))))
    n_long = int(rng.integers(0, 4))                  # a few long-token-mode packets
    if n_long:
        lens[rng.choice(n, n_long, replace=False)] = rng.integers(1000, 17000, n_long)
    return lens.astype(np.int32)


def _place(rng, lens):
    """Offsets of len(lens) regions placed in a random order with random gaps."""
    n = len(lens)
    order = rng.permutation(n)
    gaps = rng.integers(0, 40, n)
    off = np.zeros(n, np.int64)
    pos = 0
    for i in order:
        pos += int(gaps[i])
        off[i] = pos
        pos += int(lens[i])
    return off, pos + 1


def _craft(rng, key, body_len):
    """A token with a valid tag over iv || body of body_len random bytes."""
    half = len(key) // 2
    iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
    body = rng.integers(0, 256, body_len, dtype=np.uint8).tobytes()
    tag = hmac.new(key[:half], iv + body, hashlib.sha256).digest()
    return iv + body + tag


@pytest.mark.parametrize("case", range(N_CASES))
def test_fuzz_encrypt_decrypt_verify_vs_oracle(rt, case):
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(9000 + case))
    n = int(rng.integers(1, 2500))
    klen = 64 if case % 3 else 32
    nk = 1 if case % 4 == 0 else int(rng.integers(2, 3000))
    sort = bool(case % 2)
    keys = rng.integers(0, 256, (nk, klen), dtype=np.uint8)
    kidx = rng.integers(0, nk, n).astype(np.int32)
    ks = rt.KeySet(keys)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731

    # -- encrypt: shuffled, gapped placement of plaintexts and tokens
    lens = _lengths(rng, n)
    off, size = _place(rng, lens)
    buf = rng.integers(0, 256, size, dtype=np.uint8)
    ivs = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    tl = (16 + 16 * (lens // 16 + 1) + 32).astype(np.int32)
    toff, tsize = _place(rng, tl)
    ref = np.zeros(tsize, np.uint8)
    oracle.encrypt_batch(keys, buf, off.astype(np.uint64), lens.astype(np.uint32),
                         kidx.astype(np.uint32) if nk > 1 else None, ivs, ref, toff.astype(np.uint64), threads=8)
    d_tok = torch.zeros(tsize, dtype=torch.uint8, device="cuda")
    device.encrypt(ks, cu(buf), cu(off), cu(lens), cu(ivs), d_tok, cu(toff),
                   key_idx=cu(kidx) if nk > 1 else None, sort=sort)
    torch.cuda.synchronize()
    tok = d_tok.cpu().numpy()
    assert np.array_equal(tok, ref), "case %d: tokens differ from the oracle" % case

    # -- decrypt batch: the tokens above, corrupted and crafted ones, shuffled
    toks = [tok[toff[i]:toff[i] + tl[i]].tobytes() for i in range(n)]
    dk = list(kidx)
    for i in np.nonzero(rng.random(n) < 0.03)[0]:            # bit flips
        b = bytearray(toks[i])
        b[int(rng.integers(0, len(b)))] ^= 1 << int(rng.integers(0, 8))
        toks[i] = bytes(b)
    for i in np.nonzero(rng.random(n) < 0.02)[0]:            # truncations, incl. < 48 B
        toks[i] = toks[i][:int(rng.integers(0, len(toks[i])))]
    for _ in range(int(rng.integers(1, 12))):                 # valid tag, bad body
        k = int(rng.integers(0, nk))
        blen = int(rng.choice([0, 5, 16 * int(rng.integers(1, 40)), 16 * int(rng.integers(1, 40)) + 7]))
        toks.append(_craft(rng, keys[k].tobytes(), blen))
        dk.append(k)
    m = len(toks)
    perm = rng.permutation(m)
    toks = [toks[j] for j in perm]
    dk = np.asarray(dk, np.int32)[perm]
    tlen = np.asarray([len(t) for t in toks], np.int32)
    doff, dsize = _place(rng, tlen)
    dbuf = np.zeros(dsize, np.uint8)
    for i, t in enumerate(toks):
        dbuf[doff[i]:doff[i] + len(t)] = np.frombuffer(t, np.uint8)
    cap = np.maximum(tlen - 48, 0).astype(np.int32)
    poff, psize = _place(rng, cap)
    want_pt = np.zeros(psize, np.uint8)
    want_len = np.zeros(m, np.uint32)
    want_st = np.zeros(m, np.int32)
    oracle.decrypt_batch(keys, dbuf, doff.astype(np.uint64), tlen.astype(np.uint32),
                         dk.astype(np.uint32) if nk > 1 else None, want_pt, poff.astype(np.uint64), want_len,
                         want_st, threads=8)
    d_kidx = cu(dk) if nk > 1 else None
    d_out = torch.full((psize,), 0xA5, dtype=torch.uint8, device="cuda")
    d_len = torch.full((m,), -7, dtype=torch.int32, device="cuda")
    d_st = torch.full((m,), -7, dtype=torch.int32, device="cuda")
    d_dbuf, d_doff, d_tlen = cu(dbuf), cu(doff), cu(tlen)
    device.decrypt(ks, d_dbuf, d_doff, d_tlen, d_out, cu(poff), d_len, d_st, key_idx=d_kidx, sort=sort)
    d_vst = torch.full((m,), -7, dtype=torch.int32, device="cuda")
    device.verify(ks, d_dbuf, d_doff, d_tlen, d_vst, key_idx=d_kidx)
    torch.cuda.synchronize()
    st, olen, vst = d_st.cpu().numpy(), d_len.cpu().numpy(), d_vst.cpu().numpy()
    assert np.array_equal(st, want_st), "case %d: statuses differ" % case
    # pt_len carries the offending pad byte on BAD_PAD (include/rnstok.h); the
    # oracle leaves the decrypted body in place, so that byte is its last one
    want_len = want_len.astype(np.int32)
    for i in np.nonzero(want_st == rt.RT_ST_BAD_PAD)[0]:
        want_len[i] = want_pt[poff[i] + cap[i] - 1]
    assert np.array_equal(olen, want_len), "case %d: output lengths differ" % case
    assert {int(s) for s in st} >= {rt.RT_ST_OK, rt.RT_ST_BAD_HMAC}
    out = d_out.cpu().numpy()
    for i in range(m):              # whole body (pad included) on OK, zeroed region otherwise
        got = out[poff[i]:poff[i] + cap[i]]
        if st[i] == rt.RT_ST_OK:
            assert np.array_equal(got, want_pt[poff[i]:poff[i] + cap[i]]), (case, i)
        else:
            assert not got.any(), (case, i, int(st[i]))
    # the tag check alone: OK wherever the oracle got past the HMAC
    tag_ok = (want_st == rt.RT_ST_OK) | (want_st == rt.RT_ST_BAD_CT_LEN) | (want_st == rt.RT_ST_BAD_PAD)
    assert np.array_equal(vst == rt.RT_ST_OK, tag_ok), "case %d: verify disagrees" % case
    assert np.array_equal(vst == rt.RT_ST_TOO_SHORT, want_st == rt.RT_ST_TOO_SHORT)


@pytest.mark.parametrize("case", range(20))
def test_fuzz_uniform_row_views_vs_oracle(rt, case):
    """Fixed-length batches through rt_encrypt_uniform / rt_decrypt_uniform
    with rows taken from wider buffers (row stride > row length)."""
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(7000 + case))
    n = int(rng.integers(1, 40000))
    L = int(rng.choice([0, 1, 15, 16, 17, 31, 32, 100, 255, 256, 500, 511, 1000, 1500]))
    klen = 64 if case % 3 else 32
    nk = 1 if case % 2 else int(rng.integers(2, 5000))
    keys = rng.integers(0, 256, (nk, klen), dtype=np.uint8)
    kidx = rng.integers(0, nk, n).astype(np.int32)
    T = rt.token_len(L)
    pt_stride, tok_stride = L + 1 + int(rng.integers(0, 9)), T + int(rng.integers(0, 9))
    pt_rows = rng.integers(0, 256, (n, pt_stride), dtype=np.uint8)
    ivs = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    ks = rt.KeySet(keys)
    d_pt = torch.from_numpy(pt_rows).cuda()
    d_tok = torch.zeros((n, tok_stride), dtype=torch.uint8, device="cuda")
    d_k = torch.from_numpy(kidx).cuda() if nk > 1 else None
    device.encrypt_uniform(ks, d_pt[:, :L], L, torch.from_numpy(ivs).cuda(), d_tok[:, :T], key_idx=d_k)
    d_back = torch.zeros((n, T - 48 + 3), dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    device.decrypt_uniform(ks, d_tok[:, :T], T, d_back[:, :T - 48], ol, st, key_idx=d_k)
    torch.cuda.synchronize()
    tok = d_tok.cpu().numpy()
    assert not tok[:, T:].any(), "bytes past the token row were written"
    sample = np.unique(np.concatenate([rng.integers(0, n, 300), [0, n - 1]]))
    lens = np.full(sample.size, L, np.uint32)
    off = (np.arange(sample.size, dtype=np.uint64) * np.uint64(max(L, 1)))
    buf = np.ascontiguousarray(pt_rows[sample, :L]).reshape(-1)
    ref = np.zeros(sample.size * T, np.uint8)
    oracle.encrypt_batch(keys, buf if buf.size else np.zeros(1, np.uint8), off, lens,
                         kidx[sample].astype(np.uint32) if nk > 1 else None, ivs[sample], ref,
                         np.arange(sample.size, dtype=np.uint64) * np.uint64(T), threads=8)
    assert np.array_equal(tok[sample, :T].reshape(-1), ref), "case %d: tokens differ" % case
    assert (st.cpu().numpy() == 0).all() and (ol.cpu().numpy() == L).all()
    back = d_back.cpu().numpy()
    assert np.array_equal(back[:, :L], pt_rows[:, :L])
