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


@pytest.mark.parametrize("nk,sort", [(1, True), (97, False)])
def test_packed_offsets_past_4gib(rt, nk, sort):
    """Packed batches whose offsets cross 2^32: 200 000 packets of 0-600 B laid
    end to end from 40 MB below the 4 GiB mark in 4.3-GB plaintext and token
    buffers (unaligned), sorted by length (the split kernel's packed instance)
    or not, one key or per-packet keys: every packet round-trips and a sample
    spanning the boundary matches the oracle."""
    import torch
    from reticulum_amd import device
    n = 200_000
    rng = np.random.Generator(np.random.PCG64(4242 + nk))
    L = rng.integers(0, 601, n).astype(np.int64)
    T = 16 + 16 * (L // 16 + 1) + 32
    start = (1 << 32) - 40_000_003
    po = start + np.concatenate(([0], np.cumsum(L)[:-1]))
    to = start + 7 + np.concatenate(([0], np.cumsum(T)[:-1]))
    assert po[-1] > (1 << 32) and to[-1] > (1 << 32)
    dev = torch.device("cuda")
    pt = torch.empty(int(po[-1] + L[-1]) + 1, dtype=torch.uint8, device=dev)
    pt[start:].random_(0, 256, generator=torch.Generator(device=dev).manual_seed(nk))
    keys = rng.integers(0, 256, (nk, 64), dtype=np.uint8)
    ks = rt.KeySet(keys)
    ki = torch.from_numpy(rng.integers(0, nk, n).astype(np.int32)).to(dev) if nk > 1 else None
    iv = torch.from_numpy(rng.integers(0, 256, (n, 16), dtype=np.uint8)).to(dev)
    tok = torch.zeros(int(to[-1] + T[-1]) + 1, dtype=torch.uint8, device=dev)
    t_po, t_to = torch.from_numpy(po).to(dev), torch.from_numpy(to).to(dev)
    t_L, t_T = torch.from_numpy(L.astype(np.int32)).to(dev), torch.from_numpy(T.astype(np.int32)).to(dev)
    device.encrypt(ks, pt, t_po, t_L, iv, tok, t_to, key_idx=ki, sort=sort)
    # plaintexts back at their own offsets, each with room for its pad block
    bo = start + 5 + np.concatenate(([0], np.cumsum(T - 48)[:-1]))
    back = torch.zeros(int(bo[-1] + T[-1] - 48) + 1, dtype=torch.uint8, device=dev)
    t_bo = torch.from_numpy(bo).to(dev)
    ol = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.full((n,), -1, dtype=torch.int32, device=dev)
    device.decrypt(ks, tok, t_to, t_T, back, t_bo, ol, st, key_idx=ki, sort=sort)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0 and torch.equal(ol.cpu(), t_L.cpu())
    # every plaintext byte, gathered on the device
    tl64 = t_L.to(torch.int64)
    first = torch.repeat_interleave(torch.cumsum(tl64, 0) - tl64, tl64)
    k = torch.arange(int(L.sum()), device=dev) - first
    assert torch.equal(back[torch.repeat_interleave(t_bo, tl64) + k], pt[torch.repeat_interleave(t_po, tl64) + k])
    cross = int(np.searchsorted(po, 1 << 32))
    sel = np.unique(np.concatenate([np.arange(max(cross - 40, 0), min(cross + 40, n)),
                                    rng.choice(n, 120, replace=False)]))
    kih = ki.cpu().numpy() if ki is not None else np.zeros(n, np.int32)
    ivh = iv.cpu().numpy()
    for i in sel:
        p = pt[int(po[i]):int(po[i] + L[i])].cpu().numpy().tobytes()
        ref = oracle.encrypt(keys[kih[i]].tobytes(), ivh[i].tobytes(), p)
        assert tok[int(to[i]):int(to[i] + T[i])].cpu().numpy().tobytes() == ref, int(i)
