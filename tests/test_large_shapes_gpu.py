"""Large uniform batches on the multi-pass kernels (more than 1 024 tokens per
CU: the 768-thread single-key decrypt with paired quad loads, the 1024-thread
instance that uniform tokens of at most 320 B take since round 5, the
split-role encrypt), across lengths that give every tail shape and both parities of
the quad count: tokens against the C oracle (Token.encrypt, Token.py:87-97)
on a sample, 1 % of them tampered and a few forged with a bad pad byte,
decrypt statuses, lengths and plaintexts exactly where the oracle
(Token.decrypt, Token.py:100-114) puts them, and every untouched packet
round-tripped; AES-128 keys and per-packet key tables too."""
import hashlib
import hmac as _hmac

import numpy as np
import pytest

from oracle import ctoken as oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt():
    import reticulum_amd
    from reticulum_amd import _native
    _native.context(0)
    return reticulum_amd


CASES = [(L, 64, 1) for L in (0, 15, 16, 63, 64, 100, 128, 143, 191, 255, 500, 1000)] + \
        [(500, 32, 1), (143, 32, 1), (500, 64, 4099), (191, 32, 4099), (64, 64, 65536)]


@pytest.mark.parametrize("L,klen,nk", CASES)
def test_multipass_uniform_batches_vs_oracle(rt, L, klen, nk):
    import torch
    from reticulum_amd import _native, device
    lib, ctx = _native.load(), _native.context(0)
    n_cu = lib.rt_num_cus(ctx)
    n = 1200 * n_cu + 77                      # > 1 024 tokens per CU, ragged
    rng = np.random.Generator(np.random.PCG64(31000 + L + klen + nk))
    keys = rng.integers(0, 256, (nk, klen), dtype=np.uint8)
    ks = rt.KeySet(keys if nk > 1 else keys[0].tobytes())
    kx = rng.integers(0, nk, n).astype(np.int32) if nk > 1 else np.zeros(n, np.int32)
    kidx = torch.from_numpy(kx).cuda() if nk > 1 else None
    key_of = lambda i: keys[kx[i]].tobytes()          # noqa: E731
    tl = rt.token_len(L)
    assert lib.rt_plan_uniform(ctx, n, L, int(nk > 1), 0) == _native.RT_KERNEL_ENC_SPLIT
    g = torch.Generator(device="cuda").manual_seed(L + 11)
    pt = torch.randint(0, 256, (n, max(L, 1)), dtype=torch.uint8, device="cuda", generator=g)[:, :L]
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, pt, L, iv, tok, key_idx=kidx)
    torch.cuda.synchronize()
    t = tok.cpu().numpy()
    p_h, iv_h = pt.cpu().numpy(), iv.cpu().numpy()
    for i in np.unique(np.concatenate([[0, 63, 64, n - 1], rng.integers(0, n, 60)])):
        assert t[i].tobytes() == oracle.encrypt(key_of(i), iv_h[i].tobytes(), p_h[i].tobytes()), i
    bad = rng.choice(n, n // 100, replace=False)
    for j, i in enumerate(bad):
        t[i, int(rng.integers(0, tl))] ^= 1 << int(j % 8)
    forged = {}
    if tl >= 64:                              # authentic tokens whose last plaintext byte is > 16
        for i in rng.choice(np.setdiff1d(np.arange(n), bad), 20, replace=False):
            body = bytearray(rng.integers(0, 256, tl - 48 - 16 if tl - 48 > 16 else 0, dtype=np.uint8).tobytes())
            body += bytes(rng.integers(0, 256, 15, dtype=np.uint8)) + bytes([int(rng.integers(17, 256))])
            ivb = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
            key = key_of(i)
            f = oracle.encrypt(key, ivb, bytes(body))[16:-32][:tl - 48]      # drop the pad block: tl - 48 B of ct
            t[i] = np.frombuffer(ivb + f + _hmac.new(key[:klen // 2], ivb + f, hashlib.sha256).digest(), np.uint8)
            forged[int(i)] = body[-1]
    back = torch.full((n, tl - 48), 0x5A, dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    device.decrypt_uniform(ks, torch.from_numpy(t).cuda(), tl, back, ol, st, key_idx=kidx)
    torch.cuda.synchronize()
    st_h, ol_h, b_h = st.cpu().numpy(), ol.cpu().numpy(), back.cpu().numpy()
    for i in list(bad[:40]) + list(forged)[:10] + list(rng.integers(0, n, 40)):
        s, p = oracle.decrypt(key_of(i), t[i].tobytes())
        assert st_h[i] == s, (i, int(st_h[i]), s)
        if s == 0:
            assert ol_h[i] == len(p) and b_h[i, :len(p)].tobytes() == p, i
        else:
            assert not b_h[i].any(), i
    assert set(np.nonzero(st_h == 2)[0].tolist()) == set(int(i) for i in bad)
    assert set(np.nonzero(st_h == 4)[0].tolist()) == set(forged)
    for i, v in forged.items():
        assert ol_h[i] == v
    ok = st_h == 0
    assert (ol_h[ok] == L).all()
    assert np.array_equal(b_h[ok, :L], p_h[ok])
