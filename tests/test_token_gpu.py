"""GPU parity tests: HIP kernels (through librnstok's C-ABI) vs the golden
vectors generated from the reference and vs the C oracle on seeded batches.

Bit-exact everywhere (integer/byte path).  Run with ``pytest -m gpu``.
"""
import numpy as np
import pytest

from oracle import ctoken as oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt():
    import reticulum_amd
    from reticulum_amd import _native
    lib = _native.load()
    assert lib.rt_device_count() >= 1, "no HIP device visible"
    _native.context(0)        # raises loudly if the HIP path is unusable
    return reticulum_amd


def _bytes(h):
    return bytes.fromhex(h)


def test_golden_encrypt_single_item(rt, golden):
    """Token.encrypt with the reference's IV reproduces the reference token."""
    for v in golden["encrypt"]:
        ks = rt.KeySet(_bytes(v["key"]))
        toks = ks.encrypt_batch([_bytes(v["pt"])], ivs=np.frombuffer(_bytes(v["iv"]), np.uint8))
        assert toks[0].hex() == v["token"], (len(v["pt"]) // 2, v["key"][:8])


def test_golden_encrypt_batched(rt, golden):
    """All golden vectors of one key in one batch (unaligned packed offsets)."""
    by_key = {}
    for v in golden["encrypt"]:
        by_key.setdefault(v["key"], []).append(v)
    for key, vs in by_key.items():
        ks = rt.KeySet(_bytes(key))
        ivs = np.frombuffer(b"".join(_bytes(v["iv"]) for v in vs), np.uint8)
        toks = ks.encrypt_batch([_bytes(v["pt"]) for v in vs], ivs=ivs)
        assert [t.hex() for t in toks.to_list()] == [v["token"] for v in vs]
        pts, st = ks.decrypt_batch(toks)
        assert (st == 0).all()
        assert [p.hex() for p in pts.to_list()] == [v["pt"] for v in vs]


def test_golden_decrypt_cases(rt, golden):
    """Negative/edge decrypt vectors: status and plaintext match the reference."""
    for c in golden["decrypt"]:
        ks = rt.KeySet(_bytes(c["key"]))
        pts, st = ks.decrypt_batch([_bytes(c["token"])])
        assert int(st[0]) == c["status"], c["name"]
        if c["status"] == 0:
            assert pts[0].hex() == c["pt"], c["name"]
        else:
            assert pts[0] == b"", c["name"]


def test_golden_token_class_messages(rt, golden):
    """Single-item Token raises the reference's exception class and message."""
    for c in golden["decrypt"]:
        t = rt.Token(_bytes(c["key"]))
        tok = _bytes(c["token"])
        if c["status"] == 0:
            assert t.decrypt(tok).hex() == c["pt"]
        else:
            with pytest.raises(ValueError) as e:
                t.decrypt(tok)
            assert str(e.value) == c["msg"], c["name"]


def test_reference_kat_fixed_token(rt, golden):
    """tests/identity.py:157-158 KAT through the derived token key."""
    k = golden["kat"]["fixed_token"]
    t = rt.Token(_bytes(k["derived_key"]))
    assert t.decrypt(_bytes(k["token"])).hex() == k["pt"]
    assert t.verify_hmac(_bytes(k["token"]))


def _random_batch(rng, n, lengths, n_keys, klen=64):
    keys = rng.integers(0, 256, (n_keys, klen), dtype=np.uint8)
    lens = np.asarray(lengths, dtype=np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    buf = rng.integers(0, 256, max(int(lens.sum()), 1), dtype=np.uint8)
    ivs = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    kidx = rng.integers(0, n_keys, n, dtype=np.uint32) if n_keys > 1 else None
    return keys, buf, off, lens, ivs, kidx


def _oracle_tokens(keys, buf, off, lens, ivs, kidx):
    n = len(off)
    tl = (16 + 16 * (lens.astype(np.uint64) // 16 + 1) + 32).astype(np.uint32)
    toff = np.zeros(n, np.uint64)
    toff[1:] = np.cumsum(tl[:-1].astype(np.uint64))
    tok = np.zeros(max(int(tl.astype(np.uint64).sum()), 1), np.uint8)
    oracle.encrypt_batch(keys, buf, off, lens, kidx, ivs, tok, toff, threads=8)
    return tok, toff, tl


@pytest.mark.parametrize("klen", [64, 32])
@pytest.mark.parametrize("n_keys", [1, 97])
def test_random_lengths_vs_oracle(rt, klen, n_keys):
    """Mixed lengths 0..4200 B, unaligned packing, single and per-packet keys,
    AES-256 and AES-128 tokens: bit-exact vs the C oracle, and round trip."""
    rng = np.random.Generator(np.random.PCG64(11 + klen + n_keys))
    n = 3000
    lens = rng.integers(0, 4200, n)
    lens[:64] = np.arange(64)                 # every tail shape
    keys, buf, off, lens, ivs, kidx = _random_batch(rng, n, lens, n_keys, klen)
    tok, toff, tl = _oracle_tokens(keys, buf, off, lens, ivs, kidx)
    ks = rt.KeySet(keys)
    got = ks.encrypt_batch(rt.Packed(buf, off, lens), ivs=ivs, key_idx=kidx)
    assert np.array_equal(got.length, tl)
    assert np.array_equal(got.buf[:tok.size], tok[:got.buf.size])
    pts, st = ks.decrypt_batch(got, key_idx=kidx)
    assert (st == 0).all()
    assert np.array_equal(pts.length, lens)
    for i in range(0, n, 7):
        assert pts[i] == buf[int(off[i]):int(off[i]) + int(lens[i])].tobytes()


def test_tampered_tokens_exact_failures(rt):
    """1 % tampered tokens (bit flips anywhere incl. tag): exactly those fail
    with BAD_HMAC, the others decrypt; failed plaintext regions are zeroed."""
    rng = np.random.Generator(np.random.PCG64(5))
    n = 4096
    keys, buf, off, lens, ivs, kidx = _random_batch(rng, n, rng.integers(64, 4097, n), 16)
    ks = rt.KeySet(keys)
    toks = ks.encrypt_batch(rt.Packed(buf, off, lens), ivs=ivs, key_idx=kidx)
    bad = rng.random(n) < 0.01
    for i in np.nonzero(bad)[0]:
        pos = int(toks.off[i]) + int(rng.integers(0, int(toks.length[i])))
        toks.buf[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
    pts, st = ks.decrypt_batch(toks, key_idx=kidx)
    assert np.array_equal(st != 0, bad)
    assert (st[bad] == rt.RT_ST_BAD_HMAC).all()
    assert (pts.length[bad] == 0).all()


def test_wrong_key_is_bad_hmac(rt):
    ks1 = rt.KeySet(bytes(range(64)))
    ks2 = rt.KeySet(bytes(range(1, 65)))
    toks = ks1.encrypt_batch([b"x" * 100, b""])
    _, st = ks2.decrypt_batch(toks)
    assert list(st) == [rt.RT_ST_BAD_HMAC] * 2


def test_device_uniform_full_size_round_trip(rt):
    """Config c2 at full size (2^20 x 500 B, one key) through the device-resident
    API: decrypt(encrypt(x)) == x, every status OK; a seeded sample of 2048
    tokens is bit-exact vs the oracle."""
    import torch
    from reticulum_amd import device
    n, L = 1 << 20, 500
    tl = rt.token_len(L)
    g = torch.Generator(device="cuda").manual_seed(2)
    pt = torch.randint(0, 256, (n, L), dtype=torch.uint8, device="cuda", generator=g)
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    key = bytes(range(64))
    ks = rt.KeySet(key)
    tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, pt, L, iv, tok)
    back = torch.empty((n, tl - 48), dtype=torch.uint8, device="cuda")
    out_len = torch.empty(n, dtype=torch.int32, device="cuda")
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    device.decrypt_uniform(ks, tok, tl, back, out_len, status)
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0
    assert bool((out_len == L).all())
    assert torch.equal(back[:, :L], pt)
    idx = torch.randperm(n, generator=torch.Generator().manual_seed(3))[:2048].sort().values
    s_pt = pt[idx.cuda()].cpu().numpy()
    s_iv = iv[idx.cuda()].cpu().numpy()
    s_tok = tok[idx.cuda()].cpu().numpy()
    keys = np.frombuffer(key, np.uint8).reshape(1, 64)
    lens = np.full(len(idx), L, np.uint32)
    off = (np.arange(len(idx), dtype=np.uint64) * L)
    ref, _, _ = _oracle_tokens(keys, s_pt.reshape(-1), off, lens, s_iv, None)
    assert np.array_equal(ref.reshape(len(idx), tl), s_tok)


def test_device_uniform_per_packet_keys(rt):
    """Config c3 shape: 65 536 keys, uniform random key_idx, 500 B packets."""
    import torch
    from reticulum_amd import device
    n, L, nk = 1 << 17, 500, 65536
    tl = rt.token_len(L)
    rng = np.random.Generator(np.random.PCG64(3))
    keys = rng.integers(0, 256, (nk, 64), dtype=np.uint8)
    ks = rt.KeySet(keys)
    kidx = rng.integers(0, nk, n).astype(np.int32)
    pt_h = rng.integers(0, 256, (n, L), dtype=np.uint8)
    iv_h = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    pt, iv, ki = torch.from_numpy(pt_h).cuda(), torch.from_numpy(iv_h).cuda(), torch.from_numpy(kidx).cuda()
    tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, pt, L, iv, tok, key_idx=ki)
    back = torch.empty((n, tl - 48), dtype=torch.uint8, device="cuda")
    out_len = torch.empty(n, dtype=torch.int32, device="cuda")
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    device.decrypt_uniform(ks, tok, tl, back, out_len, status, key_idx=ki)
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0
    assert torch.equal(back[:, :L], pt)
    sel = np.arange(0, n, 61)
    off = np.arange(len(sel), dtype=np.uint64) * L
    ref, _, _ = _oracle_tokens(keys, pt_h[sel].reshape(-1), off, np.full(len(sel), L, np.uint32), iv_h[sel],
                               kidx[sel].astype(np.uint32))
    assert np.array_equal(ref.reshape(len(sel), tl), tok.cpu().numpy()[sel])


@pytest.mark.parametrize("n, n_keys", [(300_001, 1), (200_003, 4096)])
def test_ragged_uniform_batch_chunk_loop(rt, n, n_keys):
    """A uniform batch that does not divide over the persistent grid's lanes
    (more than one pass, ragged last pass) runs the dynamic chunk loop: every
    packet is encrypted exactly once (round trip of all n) and a seeded sample
    is bit-exact vs the oracle, for one key and for per-packet keys."""
    import torch
    from reticulum_amd import device
    L = 100
    tl = rt.token_len(L)
    rng = np.random.Generator(np.random.PCG64(n))
    keys = rng.integers(0, 256, (n_keys, 64), dtype=np.uint8)
    ks = rt.KeySet(keys if n_keys > 1 else keys[0].tobytes())
    kidx = rng.integers(0, n_keys, n).astype(np.int32)
    pt_h = rng.integers(0, 256, (n, L), dtype=np.uint8)
    iv_h = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    pt, iv = torch.from_numpy(pt_h).cuda(), torch.from_numpy(iv_h).cuda()
    ki = torch.from_numpy(kidx).cuda() if n_keys > 1 else None
    tok = torch.zeros((n, tl), dtype=torch.uint8, device="cuda")
    for _ in range(2):          # the second launch takes another counter slot
        device.encrypt_uniform(ks, pt, L, iv, tok, key_idx=ki)
    back = torch.empty((n, tl - 48), dtype=torch.uint8, device="cuda")
    out_len = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    status = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    device.decrypt_uniform(ks, tok, tl, back, out_len, status, key_idx=ki)
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0
    assert bool((out_len == L).all())
    assert torch.equal(back[:, :L], pt)
    sel = np.concatenate([np.arange(0, n, 211), np.arange(n - 64, n)])
    ref, _, _ = _oracle_tokens(keys, pt_h[sel].reshape(-1), np.arange(len(sel), dtype=np.uint64) * L,
                               np.full(len(sel), L, np.uint32), iv_h[sel],
                               kidx[sel].astype(np.uint32) if n_keys > 1 else None)
    assert np.array_equal(ref.reshape(len(sel), tl), tok.cpu().numpy()[sel])


def test_resource_chunks_16k(rt):
    """Config c4 shape (Resource-sized 16 KiB tokens), reduced count."""
    import torch
    from reticulum_amd import device
    n, L = 4096, 16384
    tl = rt.token_len(L)
    rng = np.random.Generator(np.random.PCG64(4))
    pt_h = rng.integers(0, 256, (n, L), dtype=np.uint8)
    iv_h = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    key = rng.integers(0, 256, 64, dtype=np.uint8)
    ks = rt.KeySet(key.tobytes())
    tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, torch.from_numpy(pt_h).cuda(), L, torch.from_numpy(iv_h).cuda(), tok)
    sel = np.arange(0, n, 97)
    ref, _, _ = _oracle_tokens(key.reshape(1, 64), pt_h[sel].reshape(-1), np.arange(len(sel), dtype=np.uint64) * L,
                               np.full(len(sel), L, np.uint32), iv_h[sel], None)
    assert np.array_equal(ref.reshape(len(sel), tl), tok.cpu().numpy()[sel])


def test_sorted_variable_batch_matches_unsorted_and_oracle(rt):
    """Config c5 shape (64..4096 B, many keys) through the length-bucketed
    entry points: identical tokens to the unsorted launch and to the oracle,
    and sorted decrypt restores every plaintext."""
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(55))
    n, nk = 20000, 4096
    lens = rng.integers(64, 4097, n).astype(np.int32)
    lens[:100] = rng.integers(0, 64, 100)              # and some short ones
    keys = rng.integers(0, 256, (nk, 64), dtype=np.uint8)
    kidx = rng.integers(0, nk, n).astype(np.int32)
    off = np.zeros(n, np.int64)
    off[1:] = np.cumsum(lens[:-1])
    buf = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    ivs = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    tl = (16 + 16 * (lens // 16 + 1) + 32).astype(np.int32)
    toff = np.zeros(n, np.int64)
    toff[1:] = np.cumsum(tl[:-1])
    ks = rt.KeySet(keys)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    d_pt, d_off, d_len, d_iv, d_k, d_toff, d_tl = cu(buf), cu(off), cu(lens), cu(ivs), cu(kidx), cu(toff), cu(tl)
    tok_a = torch.zeros(int(tl.sum()), dtype=torch.uint8, device="cuda")
    tok_b = torch.zeros_like(tok_a)
    device.encrypt(ks, d_pt, d_off, d_len, d_iv, tok_a, d_toff, key_idx=d_k)
    device.encrypt(ks, d_pt, d_off, d_len, d_iv, tok_b, d_toff, key_idx=d_k, sort=True)
    torch.cuda.synchronize()
    assert torch.equal(tok_a, tok_b)
    ref, _, _ = _oracle_tokens(keys, buf, off.astype(np.uint64), lens.astype(np.uint32), ivs, kidx.astype(np.uint32))
    assert np.array_equal(ref[:tok_a.numel()], tok_a.cpu().numpy())
    # decrypt writes each token's whole body (tok_len - 48 bytes, pad block
    # included) at its pt_off, so output regions are sized by capacity
    cap = tl - 48
    coff = np.zeros(n, np.int64)
    coff[1:] = np.cumsum(cap[:-1])
    back = torch.zeros(int(cap.sum()), dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    device.decrypt(ks, tok_b, d_toff, d_tl, back, cu(coff), ol, st, key_idx=d_k, sort=True)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0
    assert torch.equal(ol.cpu(), torch.from_numpy(lens))
    bh = back.cpu().numpy()
    for i in range(0, n, 37):
        assert bh[coff[i]:coff[i] + lens[i]].tobytes() == buf[off[i]:off[i] + lens[i]].tobytes()


@pytest.mark.parametrize("n", [2, 63, 64, 65, 200])
@pytest.mark.parametrize("n_keys", [1, 7])
@pytest.mark.parametrize("klen", [64, 32])
def test_sorted_small_batches_chunk_edges(rt, n, n_keys, klen):
    """Length-ordered launches around the 64-packet chunk size of the dynamic
    packet loop (one partial chunk, exactly one, one plus one packet), AES-256
    and AES-128 tokens: the tokens equal the oracle's and sorted decrypt
    restores every plaintext."""
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(1000 + n + n_keys + klen))
    lens = rng.integers(0, 1200, n).astype(np.int32)
    keys, buf, off, ulens, ivs, kidx = _random_batch(rng, n, lens, n_keys, klen)
    ks = rt.KeySet(keys if n_keys > 1 else keys[0].tobytes())
    ref, toff, tl = _oracle_tokens(keys, buf, off, ulens, ivs, kidx)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    d_k = cu(kidx.astype(np.int32)) if kidx is not None else None
    tok = torch.zeros(ref.size, dtype=torch.uint8, device="cuda")
    device.encrypt(ks, cu(buf), cu(off.astype(np.int64)), cu(lens), cu(ivs), tok, cu(toff.astype(np.int64)),
                   key_idx=d_k, sort=True)
    torch.cuda.synchronize()
    assert np.array_equal(ref, tok.cpu().numpy())
    cap = tl.astype(np.int64) - 48
    coff = np.zeros(n, np.int64)
    coff[1:] = np.cumsum(cap[:-1])
    back = torch.zeros(int(cap.sum()), dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    device.decrypt(ks, tok, cu(toff.astype(np.int64)), cu(tl.astype(np.int32)), back, cu(coff), ol, st,
                   key_idx=d_k, sort=True)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0
    assert np.array_equal(ol.cpu().numpy(), lens)
    bh = back.cpu().numpy()
    for i in range(n):
        o, L = int(off[i]), int(lens[i])
        assert bh[coff[i]:coff[i] + L].tobytes() == buf[o:o + L].tobytes()


@pytest.mark.parametrize("n,L,klen", [(300, 1024, 64), (300, 1500, 64), (20000, 4095, 64), (2048, 16391, 64),
                                       (1, 1024, 64), (129, 1039, 64), (257, 1036, 64), (300, 2047, 32),
                                       (5000, 1055, 32), (64, 1064, 64),
                                       # short packets take the single-key long kernels too (round 2)
                                       (1, 0, 64), (1, 15, 64), (3, 16, 64), (129, 17, 64), (300, 100, 32),
                                       (1, 500, 64), (64, 500, 64), (32768, 500, 64), (257, 63, 64),
                                       (5, 1023, 32), (2, 47, 32), (200, 48, 64),
                                       # one multi-MiB token (no length limit in Token.py)
                                       (1, 4_194_309, 64), (3, 1_000_003, 32)])
def test_long_token_mode_vs_oracle(rt, n, L, klen):
    """Uniform batches of long tokens with few packets per CU take the
    long-token kernels (single key: a quad of lanes per CBC chain, AES waves
    -> LDS ring -> SHA waves); bit-exact vs the oracle for every tail shape
    (tail quads of 1-4 blocks, pad of 1-16 bytes), ragged last workgroups,
    AES-256 and AES-128, and decrypt round-trips."""
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(L + n))
    tl = rt.token_len(L)
    pt_h = rng.integers(0, 256, (n, L + 1), dtype=np.uint8)[:, :L]     # rows of L bytes, never a null pointer
    iv_h = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    key = rng.integers(0, 256, klen, dtype=np.uint8)
    ks = rt.KeySet(key.tobytes())
    pt = torch.from_numpy(np.ascontiguousarray(rng.integers(0, 1, (n, L + 1), dtype=np.uint8))).cuda()[:, :L]
    pt.copy_(torch.from_numpy(np.ascontiguousarray(pt_h)))
    pt_h = np.ascontiguousarray(pt_h)
    tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, pt, L, torch.from_numpy(iv_h).cuda(), tok)
    sel = np.unique(np.concatenate([np.arange(0, n, max(1, n // 40)), [n - 1]]))
    ref, _, _ = _oracle_tokens(key.reshape(1, klen), pt_h[sel].reshape(-1), np.arange(len(sel), dtype=np.uint64) * L,
                               np.full(len(sel), L, np.uint32), iv_h[sel], None)
    assert np.array_equal(ref.reshape(len(sel), tl), tok.cpu().numpy()[sel])
    back = torch.empty((n, tl - 48), dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    device.decrypt_uniform(ks, tok, tl, back, ol, st)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0 and torch.equal(back[:, :L], pt)


@pytest.mark.parametrize("n,L", [(1, 0), (3, 1), (100, 15), (100, 16), (129, 17), (64, 47), (65, 48), (300, 100),
                                 (1, 500), (3000, 500), (200, 1000), (32768, 200)])
def test_long_mode_per_key_short_vs_oracle(rt, n, L):
    """Uniform batches with per-packet keys and few packets per CU take the
    per-key long-token encrypt (a CBC chain per lane, hashing on waves of
    their own) at every length: bit-exact vs the oracle, and decrypt (general
    kernel) round-trips."""
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(5 * L + n))
    nk = 97
    tl = rt.token_len(L)
    pt_h = np.ascontiguousarray(rng.integers(0, 256, (n, L), dtype=np.uint8))
    iv_h = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    keys = rng.integers(0, 256, (nk, 64), dtype=np.uint8)
    kidx = rng.integers(0, nk, n).astype(np.int32)
    ks = rt.KeySet(keys)
    pt = torch.zeros((n, L + 1), dtype=torch.uint8, device="cuda")[:, :L]
    pt.copy_(torch.from_numpy(pt_h))
    d_k = torch.from_numpy(kidx).cuda()
    tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, pt, L, torch.from_numpy(iv_h).cuda(), tok, key_idx=d_k)
    sel = np.unique(np.concatenate([np.arange(0, n, max(1, n // 40)), [n - 1]]))
    ref, _, _ = _oracle_tokens(keys, pt_h[sel].reshape(-1), np.arange(len(sel), dtype=np.uint64) * L,
                               np.full(len(sel), L, np.uint32), iv_h[sel], kidx[sel].astype(np.uint32))
    assert np.array_equal(ref.reshape(len(sel), tl), tok.cpu().numpy()[sel])
    back = torch.empty((n, tl - 48), dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    device.decrypt_uniform(ks, tok, tl, back, ol, st, key_idx=d_k)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0 and torch.equal(back[:, :L], pt)


@pytest.mark.parametrize("m", [65, 1, 2, 5, 31])
@pytest.mark.parametrize("klen", [64, 32])
def test_long_decrypt_statuses(rt, klen, m):
    """Long-token decrypt (block-parallel AES + serial HMAC lanes): tokens with
    valid HMAC but a bad / zero / short pad byte, and tampered tokens, give the
    reference statuses (Token.py:103-114, PKCS7.unpad) and the same outputs as
    the general kernel (variable-length entry, no long mode)."""
    import hashlib
    import hmac as hm
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(77 + klen))
    n = 300                                   # body = 16*m bytes (1 KiB and up, and short ones)
    key = rng.integers(0, 256, klen, dtype=np.uint8)
    ks = rt.KeySet(key.tobytes())
    x = rng.integers(0, 256, (n, 16 * m), dtype=np.uint8)
    x[:, -1] = np.array([0x20, 0x05, 0x00, 0x10, 0x11], np.uint8)[np.arange(n) % 5]
    iv = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    full = torch.empty((n, rt.token_len(16 * m)), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, torch.from_numpy(x).cuda(), 16 * m, torch.from_numpy(iv).cuda(), full)
    fh = full.cpu().numpy()
    sk = key[: klen // 2].tobytes()
    tl = 16 + 16 * m + 32
    toks = np.zeros((n, tl), np.uint8)
    for i in range(n):                       # drop the all-pad block, re-MAC: last byte of x is the pad byte
        body = fh[i, : 16 + 16 * m].tobytes()
        toks[i] = np.frombuffer(body + hm.new(sk, body, hashlib.sha256).digest(), np.uint8)
    toks[7::11, min(100, tl - 33)] ^= 1       # tampered ciphertext
    toks[9::13, -1] ^= 0x80                   # tampered tag
    tok = torch.from_numpy(toks).cuda()

    def run(uniform):
        back = torch.full((n, 16 * m), 0xAA, dtype=torch.uint8, device="cuda")
        ol = torch.empty(n, dtype=torch.int32, device="cuda")
        st = torch.empty(n, dtype=torch.int32, device="cuda")
        if uniform:
            device.decrypt_uniform(ks, tok, tl, back, ol, st)
        else:
            offs = torch.arange(n, dtype=torch.int64, device="cuda")
            lens = torch.full((n,), tl, dtype=torch.int32, device="cuda")
            device.decrypt(ks, tok.reshape(-1), offs * tl, lens, back.reshape(-1), offs * (16 * m), ol, st)
        torch.cuda.synchronize()
        return back.cpu().numpy(), ol.cpu().numpy(), st.cpu().numpy()

    b_long, ol_long, st_long = run(True)
    b_gen, ol_gen, st_gen = run(False)
    assert np.array_equal(st_long, st_gen) and np.array_equal(ol_long, ol_gen) and np.array_equal(b_long, b_gen)
    for i in range(n):
        tampered = (i >= 7 and (i - 7) % 11 == 0) or (i >= 9 and (i - 9) % 13 == 0)
        padn = int(x[i, -1])
        if tampered:
            assert st_long[i] == 2 and ol_long[i] == 0 and not b_long[i].any(), i
        elif padn > 16:
            assert st_long[i] == 4 and ol_long[i] == padn and not b_long[i].any(), i
        else:
            assert st_long[i] == 0 and ol_long[i] == 16 * m - padn, i
            assert np.array_equal(b_long[i, : 16 * m - padn], x[i, : 16 * m - padn]), i


def test_device_uniform_row_views(rt):
    """The uniform device entry points take row views of wider buffers (row
    stride >= row): tokens and plaintexts equal the packed-layout launch."""
    import torch
    from reticulum_amd import device
    n, L = 5000, 500
    tl = rt.token_len(L)
    g = torch.Generator(device="cuda").manual_seed(21)
    wide = torch.randint(0, 256, (n, 512), dtype=torch.uint8, device="cuda", generator=g)
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    ks = rt.KeySet(bytes(range(64)))
    tok_a = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, wide[:, :L].contiguous(), L, iv, tok_a)
    tok_b = torch.zeros((n, 640), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, wide[:, :L], L, iv, tok_b[:, :tl])
    back = torch.zeros((n, 576), dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    device.decrypt_uniform(ks, tok_b[:, :tl], tl, back[:, :tl - 48], ol, st)
    torch.cuda.synchronize()
    assert torch.equal(tok_a, tok_b[:, :tl])
    assert int((tok_b[:, tl:] != 0).sum()) == 0             # bytes past each row untouched
    assert int(st.abs().sum()) == 0 and torch.equal(back[:, :L], wide[:, :L])
    with pytest.raises(ValueError):
        device.encrypt_uniform(ks, wide[:, ::2], 256, iv, tok_a)       # bytes of a row not contiguous


@pytest.mark.parametrize("n,L", [(5000, 500), (300_000, 500), (70_000, 1500), (9000, 128)])
def test_device_uniform_aligned_slots(rt, n, L):
    """Rows in 128-B-aligned slots as INTEGRATION.md §3 recommends them (a
    token buffer whose first row starts 112 B in, so every ciphertext starts
    on a line; plaintext rows at a multiple-of-128 stride): the same tokens
    and plaintexts as packed rows, the bytes between slots untouched, at a
    one-pass, a multi-pass and a long-packet size."""
    import torch
    from reticulum_amd import device
    tl = rt.token_len(L)
    ps, ts, to = -(-L // 128) * 128, -(-tl // 128) * 128, 112
    g = torch.Generator(device="cuda").manual_seed(n + L)
    pt = torch.randint(0, 256, (n, L), dtype=torch.uint8, device="cuda", generator=g)
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    ks = rt.KeySet(bytes(range(64)))
    tok_p = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, pt, L, iv, tok_p)
    pt_s = torch.zeros((n, ps), dtype=torch.uint8, device="cuda")
    pt_s[:, :L] = pt
    buf = torch.zeros(n * ts + to, dtype=torch.uint8, device="cuda")
    tok_s = buf[to:].as_strided((n, tl), (ts, 1))
    assert (tok_s.data_ptr() + 16) % 128 == 0
    device.encrypt_uniform(ks, pt_s[:, :L], L, iv, tok_s)
    back = torch.zeros((n, -(-(tl - 48) // 128) * 128), dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    device.decrypt_uniform(ks, tok_s, tl, back[:, :tl - 48], ol, st)
    torch.cuda.synchronize()
    assert torch.equal(tok_s, tok_p)
    assert int(buf[:to].count_nonzero()) == 0
    assert int(buf[to:].view(n, ts)[:, tl:].count_nonzero()) == 0       # bytes between slots untouched
    assert int(st.abs().sum()) == 0 and bool((ol == L).all()) and torch.equal(back[:, :L], pt)
    assert int(back[:, tl - 48:].count_nonzero()) == 0


def test_verify_trials_vs_oracle(rt):
    """Ratchet trials (Identity.py:865-878) on the GPU: the first candidate
    key that opens each token (right key at a random rank, missing, twice;
    malformed and short tokens never open), host entry point and
    decrypt_trials, against the oracle's per-key decrypt."""
    from tests_helpers import trial_case
    keys, toks, cands, expect = trial_case(7, n_tok=300, n_keys=33)
    ks = rt.KeySet(keys)
    assert ks.verify_trials(toks, cands).tolist() == expect.tolist()
    pts, st, used = ks.decrypt_trials(toks, cands)
    from oracle import ctoken
    for i, tok in enumerate(toks):
        if expect[i] >= 0:
            s, p = ctoken.decrypt(keys[expect[i]].tobytes(), tok)
            assert int(st[i]) == s and (s != 0 or pts[i] == p), i
        else:
            assert int(st[i]) == rt.RT_ST_BAD_HMAC and int(used[i]) == -1


def test_verify_trials_device_batch(rt):
    """Device entry point at batch scale: 4096 tokens of 500 B, 16 candidate
    keys each out of 1024, the right one at a random rank (none for every
    7th token); bit-exact first ranks."""
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(77))
    n, L, nk, per = 4096, 500, 1024, 16
    keys = rng.integers(0, 256, (nk, 64), dtype=np.uint8)
    ks = rt.KeySet(keys)
    kidx = rng.integers(0, nk, n).astype(np.int32)
    pt = torch.from_numpy(rng.integers(0, 256, (n, L), dtype=np.uint8)).cuda()
    iv = torch.from_numpy(rng.integers(0, 256, (n, 16), dtype=np.uint8)).cuda()
    tl = rt.token_len(L)
    tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, pt, L, iv, tok, key_idx=torch.from_numpy(kidx).cuda())
    cand = rng.integers(0, nk, (n, per)).astype(np.int32)
    rank = rng.integers(0, per, n)
    expect = np.full(n, -1, np.int64)
    for t in range(n):
        cand[t][cand[t] == kidx[t]] = (kidx[t] + 1) % nk           # no accidental earlier hit
        if t % 7:
            cand[t, rank[t]] = kidx[t]
            expect[t] = rank[t]
    pair_off = torch.arange(0, n * per + 1, per, dtype=torch.int32, device="cuda")
    first = torch.empty(n, dtype=torch.int32, device="cuda")
    device.verify_trials(ks, tok.reshape(-1), torch.arange(n, dtype=torch.int64, device="cuda") * tl,
                         torch.full((n,), tl, dtype=torch.int32, device="cuda"), pair_off,
                         torch.from_numpy(cand.reshape(-1)).cuda(), first)
    torch.cuda.synchronize()
    assert first.cpu().numpy().astype(np.int64).tolist() == expect.tolist()
