"""The split-role encrypt kernel (k_encrypt_split: AES chains and HMAC chains
on waves of their own, the ciphertext handed over through an LDS ring or read
back) at the batch sizes that route to it (at least 512 packets per CU, single
key, uniform lengths), in both HBM layouts: tokens against the C oracle
(Token.encrypt, Token.py:87-97) and identical between the layouts, every
packet round-tripped, ragged last batches included; and decrypt's failures
(Token.py:100-114) at the same sizes — tampered tokens (BAD_HMAC, plaintext
zeroed), authentic tokens with a bad pad byte (BAD_PAD) — exactly where the
oracle puts them (k_decrypt_split was measured and not adopted, but these
shapes guard whichever decrypt kernel runs there)."""
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
    assert _native.load().rt_device_count() >= 1, "no HIP device visible"
    _native.context(0)
    return reticulum_amd


def _split_n(extra):
    from reticulum_amd import _native
    n_cu = _native.load().rt_num_cus(_native.context(0))
    return 64 * 8 * n_cu + extra


@pytest.mark.parametrize("L,klen,extra,n_keys", [(500, 64, 0, 1), (500, 64, 37, 1), (0, 64, 5, 1), (15, 64, 63, 1),
                                                 (16, 32, 64, 1), (17, 64, 1, 1), (100, 32, 0, 1), (1500, 64, 129, 1),
                                                 (63, 64, 3, 1), (500, 64, 11, 97), (100, 32, 64, 5), (1, 64, 0, 65536),
                                                 (128, 64, 9, 1), (143, 64, 0, 1), (191, 32, 2, 1),
                                                 # AES waves unevenly loaded (1.5 / 1.53 batches per wave): the
                                                 # row layout takes its batches from a chunk counter, the
                                                 # interleaved one keeps the static stride
                                                 (500, 64, 65541, 1), (1000, 32, 70000, 1), (256, 64, 65600, 3)])
def test_split_kernels_tokens_and_round_trip(rt, L, klen, extra, n_keys):
    import torch
    from reticulum_amd import _native, device
    n = _split_n(extra)
    lib, ctx = _native.load(), _native.context(0)
    tl = rt.token_len(L)
    pk = int(n_keys > 1)
    assert lib.rt_plan_uniform(ctx, n, L, pk, 0) == _native.RT_KERNEL_ENC_SPLIT
    assert lib.rt_plan_uniform(ctx, n - extra - 1, L, pk, 0) == _native.RT_KERNEL_GENERAL
    rng = np.random.Generator(np.random.PCG64(1000 + L + extra + n_keys))
    keys = rng.integers(0, 256, (n_keys, klen), dtype=np.uint8)
    ks = rt.KeySet(keys if n_keys > 1 else keys[0].tobytes())
    kidx = torch.from_numpy(rng.integers(0, n_keys, n).astype(np.int32)).cuda() if n_keys > 1 else None
    g = torch.Generator(device="cuda").manual_seed(L + 7)
    pt = torch.randint(0, 256, (n, max(L, 1)), dtype=torch.uint8, device="cuda", generator=g)[:, :L]
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    tok = torch.full((n, tl), 0xEE, dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, pt, L, iv, tok, key_idx=kidx)
    tu = torch.full((tl // 16, n, 16), 0xEE, dtype=torch.uint8, device="cuda")
    device.encrypt_interleaved(ks, device.interleave(pt, L), L, iv, tu, key_idx=kidx)
    torch.cuda.synchronize()
    assert torch.equal(device.deinterleave(tu, tl), tok)
    t_h, p_h, iv_h = tok.cpu().numpy(), pt.cpu().numpy(), iv.cpu().numpy()
    kx = kidx.cpu().numpy() if kidx is not None else np.zeros(n, np.int64)
    sel = np.unique(np.concatenate([[0, 63, 64, n - 65, n - 1], rng.integers(0, n, 40)]))
    for i in sel:
        assert t_h[i].tobytes() == oracle.encrypt(keys[kx[i]].tobytes(), iv_h[i].tobytes(), p_h[i].tobytes()), i
    # round trip through both layouts
    back = torch.full((n, tl - 48), 0x55, dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    device.decrypt_uniform(ks, tok, tl, back, ol, st, key_idx=kidx)
    bu = torch.full(((tl - 48) // 16, n, 16), 0x55, dtype=torch.uint8, device="cuda")
    ol2, st2 = torch.empty_like(ol), torch.empty_like(st)
    device.decrypt_interleaved(ks, tu, tl, bu, ol2, st2, key_idx=kidx)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0 and bool((ol == L).all()) and torch.equal(back[:, :L], pt)
    assert torch.equal(st2, st) and torch.equal(ol2, ol) and torch.equal(device.deinterleave(bu, tl - 48), back)


@pytest.mark.parametrize("layout", ["rows", "interleaved"])
def test_split_decrypt_failures_match_the_oracle(rt, layout):
    """1 % tampered tokens (tag, ciphertext, IV bytes) and authentic tokens
    whose last plaintext byte is above 16, spread over the batches of a
    split-size batch: statuses, lengths and zeroed plaintexts as the oracle's."""
    import torch
    from reticulum_amd import _native, device
    rng = np.random.Generator(np.random.PCG64(4242 + (layout == "rows")))
    n = _split_n(45)
    L = 50                                   # 4 ciphertext blocks: the forged bad-pad tokens' shape
    tl = rt.token_len(L)
    assert tl == 16 + 64 + 32
    lib, ctx = _native.load(), _native.context(0)
    key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    ks = rt.KeySet(key)
    pt = torch.from_numpy(rng.integers(0, 256, (n, L), dtype=np.uint8)).cuda()
    iv = torch.from_numpy(rng.integers(0, 256, (n, 16), dtype=np.uint8)).cuda()
    tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, pt, L, iv, tok)
    torch.cuda.synchronize()
    t = tok.cpu().numpy()
    bad = rng.choice(n, n // 100, replace=False)
    for j, i in enumerate(bad):
        t[i, int(rng.integers(0, tl))] ^= 1 << int(j % 8)
    rest = np.setdiff1d(np.arange(n), bad)
    forged_at = rng.choice(rest, 40, replace=False)
    last = {}
    for i in forged_at:                      # authentic, last byte 0x11..0xff (> 16)
        last[int(i)] = int(rng.integers(17, 256))
        body = bytes(rng.integers(0, 256, 63, dtype=np.uint8)) + bytes([last[int(i)]])
        f = oracle.encrypt(key, bytes(rng.integers(0, 256, 16, dtype=np.uint8)), body)
        ivb, ct = f[:16], f[16:-32][:-16]    # drop the pad block
        t[i] = np.frombuffer(ivb + ct + _hmac.new(key[:32], ivb + ct, hashlib.sha256).digest(), np.uint8)
    tok2 = torch.from_numpy(t).cuda()
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    if layout == "rows":
        out = torch.full((n, tl - 48), 0x33, dtype=torch.uint8, device="cuda")
        device.decrypt_uniform(ks, tok2, tl, out, ol, st)
        torch.cuda.synchronize()
        back = out.cpu().numpy()
    else:
        bu = torch.full(((tl - 48) // 16, n, 16), 0x33, dtype=torch.uint8, device="cuda")
        device.decrypt_interleaved(ks, device.interleave(tok2, tl), tl, bu, ol, st)
        torch.cuda.synchronize()
        back = device.deinterleave(bu, tl - 48).cpu().numpy()
    st_h, ol_h = st.cpu().numpy(), ol.cpu().numpy()
    want_bad = set(int(i) for i in bad)
    assert set(np.nonzero(st_h == 2)[0].tolist()) == want_bad
    assert set(np.nonzero(st_h == 4)[0].tolist()) == set(int(i) for i in forged_at)
    for i in list(bad[:30]) + list(forged_at[:10]):
        s, p = oracle.decrypt(key, t[i].tobytes())
        assert st_h[i] == s and not back[i].any(), i
    for i in forged_at:
        assert ol_h[i] == last[int(i)] and st_h[i] == 4      # the authenticated pad byte
    ok = st_h == 0
    assert (ol_h[ok] == L).all()
    assert np.array_equal(back[ok, :L], pt.cpu().numpy()[ok])


@pytest.mark.parametrize("sort,n_keys,lo,hi", [(True, 97, 0, 700), (False, 1, 0, 300), (True, 1, 64, 4096),
                                              (False, 65536, 500, 520)])
def test_split_kernel_packed_batches(rt, sort, n_keys, lo, hi):
    """Packed batches (per-packet lengths and offsets, c5's shape) at split
    sizes, length-ordered (the chunk counter) or not: every token against the
    oracle on a sample, every packet round-tripped."""
    import torch
    from reticulum_amd import device
    n = _split_n(77)
    rng = np.random.Generator(np.random.PCG64(77 + n_keys + lo))
    keys = rng.integers(0, 256, (n_keys, 64), dtype=np.uint8)
    ks = rt.KeySet(keys if n_keys > 1 else keys[0].tobytes())
    lens = rng.integers(lo, hi + 1, n).astype(np.int32)
    off = np.zeros(n, np.int64)
    off[1:] = np.cumsum(lens[:-1].astype(np.int64))
    tl = (16 + 16 * (lens // 16 + 1) + 32).astype(np.int64)
    toff = np.zeros(n, np.int64)
    toff[1:] = np.cumsum(tl[:-1])
    g = torch.Generator(device="cuda").manual_seed(int(lo) + 3)
    pt = torch.randint(0, 256, (int(lens.sum()) + 1,), dtype=torch.uint8, device="cuda", generator=g)
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    kidx = torch.from_numpy(rng.integers(0, n_keys, n).astype(np.int32)).cuda() if n_keys > 1 else None
    d = lambda a: torch.from_numpy(a).cuda()     # noqa: E731
    tok = torch.full((int(tl.sum()),), 0xEE, dtype=torch.uint8, device="cuda")
    device.encrypt(ks, pt, d(off), d(lens), iv, tok, d(toff), key_idx=kidx, sort=sort)
    poff = np.zeros(n, np.int64)
    poff[1:] = np.cumsum((tl - 48)[:-1])
    back = torch.zeros(int((tl - 48).sum()), dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    device.decrypt(ks, tok, d(toff), d(tl.astype(np.int32)), back, d(poff), ol, st, key_idx=kidx, sort=sort)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0 and np.array_equal(ol.cpu().numpy(), lens)
    t_h, p_h, b_h, iv_h = tok.cpu().numpy(), pt.cpu().numpy(), back.cpu().numpy(), iv.cpu().numpy()
    kx = kidx.cpu().numpy() if kidx is not None else np.zeros(n, np.int64)
    for i in range(n):
        assert b_h[poff[i]:poff[i] + lens[i]].tobytes() == p_h[off[i]:off[i] + lens[i]].tobytes(), i
    sel = np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, 60)]))
    for i in sel:
        want = oracle.encrypt(keys[kx[i]].tobytes(), iv_h[i].tobytes(), p_h[off[i]:off[i] + lens[i]].tobytes())
        assert t_h[toff[i]:toff[i] + tl[i]].tobytes() == want, i


@pytest.mark.parametrize("L,extra_stride,base_off,n_keys", [(500, 0, 16, 1), (500, 16, 0, 1), (500, 32, 48, 1),
                                                            (500, 48, 32, 1), (17, 16, 16, 1), (47, 48, 0, 1),
                                                            (1500, 32, 16, 1), (383, 16, 48, 97), (0, 0, 32, 1),
                                                            (64, 16, 0, 65536)])
def test_split_sector_grouped_stores_every_phase(rt, L, extra_stride, base_off, n_keys):
    """k_encrypt_split stores each 64-B sector of ciphertext in one burst, holding
    the units a quad shares with the next (round 6).  Token rows at strides and
    first offsets that put the IV and every quad at each of the four sector
    phases, into a sentinel-filled buffer: every token equal to the interleaved
    layout's (which stores whole quads) and a sample to the oracle, and no byte
    between the rows written."""
    import torch
    from reticulum_amd import _native, device
    n = _split_n(5)
    lib, ctx = _native.load(), _native.context(0)
    tl = rt.token_len(L)
    assert lib.rt_plan_uniform(ctx, n, L, int(n_keys > 1), 0) == _native.RT_KERNEL_ENC_SPLIT
    rng = np.random.Generator(np.random.PCG64(77 + L + extra_stride + base_off))
    keys = rng.integers(0, 256, (n_keys, 64), dtype=np.uint8)
    ks = rt.KeySet(keys if n_keys > 1 else keys[0].tobytes())
    kidx = torch.from_numpy(rng.integers(0, n_keys, n).astype(np.int32)).cuda() if n_keys > 1 else None
    g = torch.Generator(device="cuda").manual_seed(L + 11)
    pt = torch.randint(0, 256, (n, max(L, 1)), dtype=torch.uint8, device="cuda", generator=g)[:, :L]
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    ts = tl + extra_stride
    buf = torch.full((n * ts + 256,), 0xEE, dtype=torch.uint8, device="cuda")
    base = (-buf.data_ptr()) % 64 + base_off
    tok = buf[base:].as_strided((n, tl), (ts, 1))
    device.encrypt_uniform(ks, pt, L, iv, tok, key_idx=kidx)
    tu = torch.full((tl // 16, n, 16), 0xEE, dtype=torch.uint8, device="cuda")
    device.encrypt_interleaved(ks, device.interleave(pt, L), L, iv, tu, key_idx=kidx)
    torch.cuda.synchronize()
    assert torch.equal(device.deinterleave(tu, tl), tok)
    # the gaps between rows and the bytes around the batch stay untouched
    mask = torch.ones(buf.numel(), dtype=torch.bool, device="cuda")
    rows = (base + torch.arange(n, device="cuda", dtype=torch.int64)[:, None] * ts
            + torch.arange(tl, device="cuda", dtype=torch.int64)[None, :]).reshape(-1)
    mask[rows] = False
    assert bool((buf[mask] == 0xEE).all())
    t_h, p_h, iv_h = tok.cpu().numpy(), pt.cpu().numpy(), iv.cpu().numpy()
    kx = kidx.cpu().numpy() if kidx is not None else np.zeros(n, np.int64)
    for i in np.unique(np.concatenate([[0, 1, 2, 3, 63, 64, n - 1], rng.integers(0, n, 24)])):
        assert t_h[i].tobytes() == oracle.encrypt(keys[kx[i]].tobytes(), iv_h[i].tobytes(), p_h[i].tobytes()), i


@pytest.mark.parametrize("n_keys,shift", [(1, 48), (65536, 48), (1, 7), (65536, 9)])
def test_split_sector_grouped_stores_packed_length_ordered(rt, n_keys, shift):
    """The length-ordered packed path (c5's encrypt half) with sector-grouped
    stores: tokens at prefix-sum offsets (on and off the 16-B grid), into a
    sentinel-filled buffer; every token round-trips, a sample equals the oracle,
    and no byte outside the tokens is written."""
    import torch
    from reticulum_amd import _native, device
    n = _split_n(3)
    rng = np.random.Generator(np.random.PCG64(4242 + n_keys + shift))
    keys = rng.integers(0, 256, (n_keys, 64), dtype=np.uint8)
    ks = rt.KeySet(keys if n_keys > 1 else keys[0].tobytes())
    kidx = torch.from_numpy(rng.integers(0, n_keys, n).astype(np.int32)).cuda() if n_keys > 1 else None
    lens = rng.integers(0, 700, n).astype(np.int32)
    off = np.zeros(n, np.int64)
    off[1:] = np.cumsum(lens[:-1])
    tl = (16 + 16 * (lens // 16 + 1) + 32).astype(np.int64)
    toff = np.zeros(n, np.int64)
    toff[1:] = np.cumsum(tl[:-1])
    toff += shift            # 48: 16-B-aligned tokens; 7 / 9: tokens off the 16-B grid
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    g = torch.Generator(device="cuda").manual_seed(99)
    buf = torch.randint(0, 256, (int(lens.astype(np.int64).sum()) + 1,), dtype=torch.uint8, device="cuda", generator=g)
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    tok = torch.full((int(toff[-1] + tl[-1]) + 64,), 0xEE, dtype=torch.uint8, device="cuda")
    ws = torch.empty(int(_native.load().rt_workspace_bytes(n)), dtype=torch.uint8, device="cuda")
    device.encrypt(ks, buf, cu(off), cu(lens), iv, tok, cu(toff), key_idx=kidx, sort=True, workspace=ws)
    torch.cuda.synchronize()
    th = tok.cpu().numpy()
    covered = np.zeros(th.size, bool)
    starts, ends = toff, toff + tl
    d = np.zeros(th.size + 1, np.int64)
    np.add.at(d, starts, 1)
    np.add.at(d, ends, -1)
    covered = np.cumsum(d)[:-1] > 0
    assert (th[~covered] == 0xEE).all()
    cap = tl - 48
    coff = np.zeros(n, np.int64)
    coff[1:] = np.cumsum(cap[:-1])
    back = torch.zeros(int(cap.sum()), dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    device.decrypt(ks, tok, cu(toff), cu(tl.astype(np.int32)), back, cu(coff), ol, st, key_idx=kidx, sort=True,
                   workspace=ws)
    torch.cuda.synchronize()
    assert bool((st == 0).all()) and np.array_equal(ol.cpu().numpy(), lens)
    hb, hiv, hback = buf.cpu().numpy(), iv.cpu().numpy(), back.cpu().numpy()
    kx = kidx.cpu().numpy() if kidx is not None else np.zeros(n, np.int64)
    for i in rng.integers(0, n, 300):
        p = hb[off[i]:off[i] + lens[i]].tobytes()
        assert hback[coff[i]:coff[i] + lens[i]].tobytes() == p, i
    for i in rng.integers(0, n, 48):
        p = hb[off[i]:off[i] + lens[i]].tobytes()
        assert th[toff[i]:toff[i] + tl[i]].tobytes() == oracle.encrypt(keys[kx[i]].tobytes(), hiv[i].tobytes(), p), i
