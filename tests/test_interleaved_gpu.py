"""The unit-interleaved device layout (rt_encrypt_interleaved /
rt_decrypt_interleaved): 16-B unit u of packet p at
16*(u*n + p), so each wave's loads and stores are contiguous KiBs.  Tokens must
be bit-identical to the row layout's and to the oracle's; decrypt statuses,
lengths and the zeroing of failed packets as the row layout."""
import numpy as np
import pytest

from oracle import ctoken as oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt():
    import reticulum_amd
    from reticulum_amd import _native
    assert _native.load().rt_device_count() >= 1, "no HIP device visible"
    _native.context(0)
    return reticulum_amd


@pytest.mark.parametrize("n,L,n_keys,klen", [(3000, 500, 1, 64), (3000, 0, 1, 64), (2049, 1, 1, 64),
                                             (5000, 15, 97, 64), (777, 16, 1, 32), (4096, 17, 1, 64),
                                             (1, 100, 1, 64), (70000, 100, 1, 64), (3000, 1023, 65, 32),
                                             (256 * 1024 + 3, 64, 1, 64), (300, 4096, 3, 64)])
def test_interleaved_equals_rows_and_oracle(rt, n, L, n_keys, klen):
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(n * 7 + L))
    keys = rng.integers(0, 256, (n_keys, klen), dtype=np.uint8)
    ks = rt.KeySet(keys if n_keys > 1 else keys[0].tobytes())
    tl = rt.token_len(L)
    g = torch.Generator(device="cuda").manual_seed(L + 1)
    pt = torch.randint(0, 256, (n, max(L, 1)), dtype=torch.uint8, device="cuda", generator=g)[:, :L]
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    kidx = torch.from_numpy(rng.integers(0, n_keys, n).astype(np.int32)).cuda() if n_keys > 1 else None
    # row layout (oracle-checked elsewhere) and interleaved layout
    tok_rows = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, pt, L, iv, tok_rows, key_idx=kidx)
    pu = device.interleave(pt, L)
    tu = torch.full((tl // 16, n, 16), 0xEE, dtype=torch.uint8, device="cuda")
    device.encrypt_interleaved(ks, pu, L, iv, tu, key_idx=kidx)
    torch.cuda.synchronize()
    assert torch.equal(device.deinterleave(tu, tl), tok_rows)
    # a seeded sample straight against the oracle
    sel = np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, 24)]))
    t_h, p_h, iv_h = tok_rows.cpu().numpy(), pt.cpu().numpy(), iv.cpu().numpy()
    kx = kidx.cpu().numpy() if kidx is not None else np.zeros(n, np.int64)
    for i in sel:
        assert t_h[i].tobytes() == oracle.encrypt(keys[kx[i]].tobytes(), iv_h[i].tobytes(), p_h[i].tobytes())
    # decrypt both layouts: same plaintexts (pad block included), lengths, statuses
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    bu = torch.full(((tl - 48) // 16, n, 16), 0x55, dtype=torch.uint8, device="cuda")
    device.decrypt_interleaved(ks, tu, tl, bu, ol, st, key_idx=kidx)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0 and bool((ol == L).all())
    assert torch.equal(device.deinterleave(bu, tl - 48)[:, :L], pt)


def test_interleaved_decrypt_failures_match_rows(rt):
    """Tampered tags / ciphertexts / IVs give BAD_HMAC with the plaintext
    units zeroed, an authentic token with a bad pad byte BAD_PAD, exactly as
    the row layout reports them."""
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(99))
    n, L = 5000, 200
    key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    ks = rt.KeySet(key)
    tl = rt.token_len(L)
    pt = torch.from_numpy(rng.integers(0, 256, (n, L), dtype=np.uint8)).cuda()
    iv = torch.from_numpy(rng.integers(0, 256, (n, 16), dtype=np.uint8)).cuda()
    tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, pt, L, iv, tok)
    torch.cuda.synchronize()
    bad = rng.choice(n, 60, replace=False)
    for j, i in enumerate(bad):
        tok[int(i), int(rng.integers(0, tl))] ^= 1 << int(j % 8)
    t = tok.cpu().numpy()
    bp = int(np.setdiff1d(np.arange(n), bad)[0])
    t[bp, :] = 0                                                # an all-zero token: BAD_HMAC too
    tok2 = torch.from_numpy(t).cuda()
    ol_r, st_r = torch.empty(n, dtype=torch.int32, device="cuda"), torch.empty(n, dtype=torch.int32, device="cuda")
    back_r = torch.empty((n, tl - 48), dtype=torch.uint8, device="cuda")
    device.decrypt_uniform(ks, tok2, tl, back_r, ol_r, st_r)
    ol_i, st_i = torch.empty_like(ol_r), torch.empty_like(st_r)
    bu = torch.full(((tl - 48) // 16, n, 16), 0x77, dtype=torch.uint8, device="cuda")
    device.decrypt_interleaved(ks, device.interleave(tok2, tl), tl, bu, ol_i, st_i)
    torch.cuda.synchronize()
    assert torch.equal(st_i, st_r) and torch.equal(ol_i, ol_r)
    assert torch.equal(device.deinterleave(bu, tl - 48), back_r)
    failed = set(torch.nonzero(st_r).flatten().tolist())
    assert failed == set(int(i) for i in bad) | {bp}
    # bad pad, authentic: a 4-block body whose last byte is 0x20 (> 16), tagged with the key
    import hashlib
    import hmac as _hmac
    forged = oracle.encrypt(key, bytes(16), bytes(range(48)) + b"\x20" * 16)   # + a 16 x 0x10 pad block
    ivb, ct = forged[:16], forged[16:-32][:-16]                                # drop the pad block
    tb = ivb + ct + _hmac.new(key[:32], ivb + ct, hashlib.sha256).digest()
    assert oracle.decrypt(key, tb)[0] == rt.RT_ST_BAD_PAD
    tl4 = 16 + 64 + 32
    one = torch.from_numpy(np.frombuffer(tb, np.uint8).copy()).cuda().view(1, tl4)
    o1, s1 = torch.empty(1, dtype=torch.int32, device="cuda"), torch.empty(1, dtype=torch.int32, device="cuda")
    b1 = torch.full((4, 1, 16), 0x33, dtype=torch.uint8, device="cuda")
    device.decrypt_interleaved(ks, device.interleave(one, tl4), tl4, b1, o1, s1)
    torch.cuda.synchronize()
    assert int(s1[0]) == rt.RT_ST_BAD_PAD and int(o1[0]) == 0x20 and int(b1.abs().sum()) == 0


def test_interleaved_rejects_malformed_lengths(rt):
    import torch
    from reticulum_amd import _native, device
    ks = rt.KeySet(bytes(64))
    ol = torch.empty(4, dtype=torch.int32, device="cuda")
    st = torch.empty(4, dtype=torch.int32, device="cuda")
    with pytest.raises(ValueError):
        device.decrypt_interleaved(ks, torch.zeros((3, 4, 16), dtype=torch.uint8, device="cuda"), 48,
                                   torch.zeros((0, 4, 16), dtype=torch.uint8, device="cuda"), ol, st)
    lib = _native.load()
    assert lib.rt_decrypt_interleaved(ks.handle, 1, 72, None, 1, ol.data_ptr(), st.data_ptr(), 4, None) == \
        _native.RT_E_INVAL
