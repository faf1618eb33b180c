"""GPU tests of the C-ABI runtime and of every BASELINE config at full size.

* Token.verify_hmac through the verify-only kernel (no AES), against the
  reference-generated goldens and hashlib's HMAC on random tokens.
* Stream ordering of the runtime: the chunk-counter ring under two streams
  and > 1000 ragged launches each, key sets created and destroyed per packet
  while another stream runs c2, a derived key set used right away from the
  host path, and the fused HKDF + key setup against the two-launch path.
* Configs c3, c4 (general kernel) at BASELINE.json's full sizes and c5 at
  its 8-GPU rank share (the whole c5 batch: tests/test_c5_full_gpu.py):
  size-independent properties (round trip, exact tamper set) plus seeded
  oracle samples of both directions.

Bit-exact everywhere.  Run with ``pytest -m gpu``.
"""
import hashlib
import hmac

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


def _hmac_ok(key, tok):
    sk = key[: len(key) // 2]
    return hmac.compare_digest(hmac.new(sk, tok[:-32], hashlib.sha256).digest(), tok[-32:])


# ---------------------------------------------------------------- verify_hmac

def test_verify_hmac_goldens(rt, golden):
    """Token.verify_hmac (Token.py:77-84) on every golden decrypt case: True
    wherever the reference's tag check passes — including tokens whose
    ciphertext is empty or not whole blocks (len40_validtag, ...), which
    decrypt rejects later — False on a bad tag, ValueError at <= 32 bytes."""
    by_key = {}
    for c in golden["decrypt"]:
        t = rt.Token(bytes.fromhex(c["key"]))
        tok = bytes.fromhex(c["token"])
        if c["status"] == 1:
            with pytest.raises(ValueError) as e:
                t.verify_hmac(tok)
            assert str(e.value) == c["msg"]
        else:
            assert t.verify_hmac(tok) is (c["status"] != 2), c["name"]
        by_key.setdefault(c["key"], []).append(c)
    for key, cs in by_key.items():
        st = rt.KeySet(bytes.fromhex(key)).verify_batch([bytes.fromhex(c["token"]) for c in cs])
        want = [1 if c["status"] == 1 else (2 if c["status"] == 2 else 0) for c in cs]
        assert st.tolist() == want
    for v in golden["encrypt"][:20]:
        assert rt.Token(bytes.fromhex(v["key"])).verify_hmac(bytes.fromhex(v["token"]))


@pytest.mark.parametrize("n_keys", [1, 37])
def test_verify_random_lengths_vs_hashlib(rt, n_keys):
    """3000 tokens of every length 0..3000 (whole blocks or not), 2 % with a
    flipped bit, host and device entry points: status == hashlib's HMAC
    verdict; the device path writes nothing but the status."""
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(17 + n_keys))
    n = 3000
    keys = rng.integers(0, 256, (n_keys, 64), dtype=np.uint8)
    kidx = rng.integers(0, n_keys, n).astype(np.int32)
    lens = rng.integers(0, 3000, n)
    lens[:100] = np.arange(100)
    toks = []
    for i in range(n):
        k = keys[kidx[i]].tobytes()
        body = rng.integers(0, 256, int(lens[i]), dtype=np.uint8).tobytes()
        tok = body + hmac.new(k[:32], body, hashlib.sha256).digest() if lens[i] >= 16 else body
        if rng.random() < 0.02 and tok:
            b = bytearray(tok)
            b[int(rng.integers(0, len(b)))] ^= 1 << int(rng.integers(0, 8))
            tok = bytes(b)
        toks.append(tok)
    want = np.array([1 if len(t) <= 32 else (0 if _hmac_ok(keys[kidx[i]].tobytes(), t) else 2)
                     for i, t in enumerate(toks)], np.int32)
    ks = rt.KeySet(keys)
    ki = kidx if n_keys > 1 else None
    assert np.array_equal(ks.verify_batch(toks, key_idx=ki), want)
    packed = rt.Packed.from_list(toks)
    d_tok = torch.from_numpy(packed.buf).cuda()
    snapshot = d_tok.clone()
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    device.verify(ks, d_tok, torch.from_numpy(packed.off.astype(np.int64)).cuda(),
                  torch.from_numpy(packed.length.astype(np.int32)).cuda(), st,
                  key_idx=torch.from_numpy(kidx).cuda() if n_keys > 1 else None)
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), want)
    assert torch.equal(d_tok, snapshot)


# ------------------------------------------------------------ stream ordering

def _ragged_case(rt, n, L, n_keys, seed):
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(seed))
    keys = rng.integers(0, 256, (n_keys, 64), dtype=np.uint8)
    ks = rt.KeySet(keys if n_keys > 1 else keys[0].tobytes())
    pt_h = rng.integers(0, 256, (n, L), dtype=np.uint8)
    iv_h = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    kidx = rng.integers(0, n_keys, n).astype(np.int32)
    pt, iv = torch.from_numpy(pt_h).cuda(), torch.from_numpy(iv_h).cuda()
    ki = torch.from_numpy(kidx).cuda() if n_keys > 1 else None
    tl = rt.token_len(L)
    ref = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, pt, L, iv, ref, key_idx=ki)
    torch.cuda.synchronize()
    sel = np.concatenate([np.arange(0, n, 997), np.arange(n - 64, n)])
    o, _, _ = _oracle_rows(keys, pt_h[sel], iv_h[sel], kidx[sel] if n_keys > 1 else None)
    assert np.array_equal(o, ref.cpu().numpy()[sel])
    return ks, pt, iv, ki, ref


def _oracle_rows(keys, pt_rows, iv_rows, kidx):
    n, L = pt_rows.shape
    tl = 16 + 16 * (L // 16 + 1) + 32
    tok = np.zeros(n * tl, np.uint8)
    oracle.encrypt_batch(keys, pt_rows.reshape(-1), np.arange(n, dtype=np.uint64) * L, np.full(n, L, np.uint32),
                         None if kidx is None else kidx.astype(np.uint32), iv_rows, tok,
                         np.arange(n, dtype=np.uint64) * tl, threads=8)
    return tok.reshape(n, tl), None, None


def test_counter_ring_two_streams_1100_ragged_launches(rt):
    """The ragged-batch chunk counters are a ring of slots reused across
    launches.  Two streams each issue 1100 ragged launches (more passes than
    the persistent grid has lanes, last pass partial: the dynamic chunk loop)
    of different batches — one key and per-packet keys — with the output
    zeroed before every launch; every output must equal the batch's
    reference tokens (a counter zeroed or advanced under a running launch
    would skip or repeat chunks and leave zeros)."""
    import torch
    from reticulum_amd import device
    cases = [_ragged_case(rt, 262_211, 16, 1, 1), _ragged_case(rt, 196_999, 32, 513, 2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.empty_like(c[4]) for c in cases]
    bad = [torch.zeros((), dtype=torch.int64, device="cuda") for _ in cases]
    torch.cuda.synchronize()
    for it in range(1100):
        for j, (ks, pt, iv, ki, ref) in enumerate(cases):
            with torch.cuda.stream(streams[j]):
                outs[j].zero_()
                device.encrypt_uniform(ks, pt, pt.shape[1], iv, outs[j], key_idx=ki, stream=streams[j])
                bad[j] += (outs[j] != ref).any(dim=1).sum()
    torch.cuda.synchronize()
    assert [int(b) for b in bad] == [0, 0]


def test_token_per_packet_churn_beside_c2(rt):
    """Identity.encrypt builds a Token per packet (Identity.py:829-830): 10 000
    Tokens created, used once and destroyed while another stream runs c2
    (2^20 x 500 B) launches.  Creation and destruction block neither stream;
    every per-packet token opens under the oracle and every c2 output equals
    its reference."""
    import gc
    import torch
    from reticulum_amd import device
    n, L = 1 << 20, 500
    tl = rt.token_len(L)
    g = torch.Generator(device="cuda").manual_seed(9)
    pt = torch.randint(0, 256, (n, L), dtype=torch.uint8, device="cuda", generator=g)
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    ks = rt.KeySet(bytes(range(64)))
    ref = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, pt, L, iv, ref)
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    out = torch.empty_like(ref)
    bad = torch.zeros((), dtype=torch.int64, device="cuda")
    with torch.cuda.stream(side):
        for _ in range(100):                      # ~0.1 s of device work queued
            device.encrypt_uniform(ks, pt, L, iv, out, stream=side)
            bad += (out != ref).any(dim=1).sum()
    rng = np.random.Generator(np.random.PCG64(10))
    failures = 0
    for i in range(10_000):
        key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
        msg = rng.integers(0, 256, int(rng.integers(0, 600)), dtype=np.uint8).tobytes()
        t = rt.Token(key)
        tok = t.encrypt(msg)
        st, back = oracle.decrypt(key, tok)
        failures += st != 0 or back != msg
        del t
        if i % 1000 == 999:
            gc.collect()
    torch.cuda.synchronize()
    assert failures == 0
    assert int(bad) == 0


def test_derived_keyset_used_at_once_from_host_path(rt):
    """A key set derived on a side stream (device.derive_keyset enqueues and
    returns) is used immediately by the host entry points, which run on the
    library's own staging streams: they wait for the derivation, so every
    token decrypts (no ordering existed before)."""
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(12))
    n = 20000
    ikm = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    salt = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    side = torch.cuda.Stream()
    d_ikm, d_salt = torch.from_numpy(ikm).cuda(), torch.from_numpy(salt).cuda()
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        ks = device.derive_keyset(d_ikm, d_salt, key_len=64, stream=side)
    pts = [rng.integers(0, 256, 100, dtype=np.uint8).tobytes() for _ in range(n)]
    kidx = np.arange(n, dtype=np.uint32)
    toks = ks.encrypt_batch(pts, key_idx=kidx)
    back, st = ks.decrypt_batch(toks, key_idx=kidx)
    assert (st == 0).all() and back.to_list() == pts
    for i in range(0, n, 997):
        key = oracle.hkdf(64, ikm[i].tobytes(), salt[i].tobytes())
        assert oracle.decrypt(key, toks[i]) == (0, pts[i]), i


@pytest.mark.parametrize("key_len", [64, 32])
@pytest.mark.parametrize("shared", [False, True])
def test_fused_hkdf_key_setup_equals_two_launch_path(rt, key_len, shared):
    """rt_keyset_create_hkdf derives and expands keys in one launch for the
    per-packet keying shape; a context string forces the two-launch path
    (HKDF into a temporary, then key setup).  Tokens under each key set match
    the oracle with the oracle's derived keys, for row salts and for one
    shared salt row (grid-stride instance), AES-256 and AES-128."""
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(40 + key_len + shared))
    n, L = 300_000, 64
    ikm = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    salt = rng.integers(0, 256, (1 if shared else n, 16), dtype=np.uint8)
    d_salt = torch.from_numpy(salt).cuda()
    d_salt = d_salt.expand(n, 16) if shared else d_salt
    ctx = torch.from_numpy(np.frombuffer(b"ctx", np.uint8).copy()).cuda()
    ks_fused = device.derive_keyset(torch.from_numpy(ikm).cuda(), d_salt, key_len=key_len)
    ks_two = device.derive_keyset(torch.from_numpy(ikm).cuda(), d_salt, context=ctx, key_len=key_len)
    pt = rng.integers(0, 256, (n, L), dtype=np.uint8)
    iv = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    tl = rt.token_len(L)
    kidx = torch.arange(n, dtype=torch.int32, device="cuda")
    outs = []
    for ks in (ks_fused, ks_two):
        tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
        device.encrypt_uniform(ks, torch.from_numpy(pt).cuda(), L, torch.from_numpy(iv).cuda(), tok, key_idx=kidx)
        outs.append(tok.cpu().numpy())
    for i in list(range(0, n, 4999)) + [n - 1]:
        s = salt[0 if shared else i].tobytes()
        k1 = oracle.hkdf(key_len, ikm[i].tobytes(), s)
        k2 = oracle.hkdf(key_len, ikm[i].tobytes(), s, b"ctx")
        assert outs[0][i].tobytes() == oracle.encrypt(k1, iv[i].tobytes(), pt[i].tobytes()), i
        assert outs[1][i].tobytes() == oracle.encrypt(k2, iv[i].tobytes(), pt[i].tobytes()), i


# -------------------------------------------------------- configs at full size

def test_config_c3_full_size(rt):
    """c3: 2^20 x 500 B, 65 536 per-packet keys (uniform random key_idx):
    decrypt(encrypt(x)) == x for every packet, and a seeded sample of 2048
    tokens and of their decrypted plaintexts equals the oracle's."""
    import torch
    from reticulum_amd import device
    n, L, nk = 1 << 20, 500, 65536
    tl = rt.token_len(L)
    rng = np.random.Generator(np.random.PCG64(33))
    keys = rng.integers(0, 256, (nk, 64), dtype=np.uint8)
    ks = rt.KeySet(keys)
    g = torch.Generator(device="cuda").manual_seed(33)
    pt = torch.randint(0, 256, (n, L), dtype=torch.uint8, device="cuda", generator=g)
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    ki = torch.randint(0, nk, (n,), dtype=torch.int32, device="cuda", generator=g)
    tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, pt, L, iv, tok, key_idx=ki)
    back = torch.empty((n, tl - 48), dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    device.decrypt_uniform(ks, tok, tl, back, ol, st, key_idx=ki)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0 and bool((ol == L).all()) and torch.equal(back[:, :L], pt)
    sel = np.sort(np.random.Generator(np.random.PCG64(34)).choice(n, 2048, replace=False))
    s = torch.from_numpy(sel).cuda()
    ref, _, _ = _oracle_rows(keys, pt[s].cpu().numpy(), iv[s].cpu().numpy(), ki[s].cpu().numpy())
    assert np.array_equal(ref, tok[s].cpu().numpy())
    for j, i in enumerate(sel[:256]):
        k = keys[int(ki[int(i)])].tobytes()
        assert oracle.decrypt(k, ref[j].tobytes()) == (0, back[int(i), :L].cpu().numpy().tobytes())


def test_config_c4_full_size_general_kernel(rt):
    """c4 on one GPU: 262 144 x 16 KiB Resource chunks, one key (more than
    128 tokens per CU, so the one-lane-per-token kernels run, not the
    long-token ones): round trip of all 4 GiB and an oracle sample of 64
    tokens."""
    import torch
    from reticulum_amd import device
    n, L = 262_144, 16384
    tl = rt.token_len(L)
    g = torch.Generator(device="cuda").manual_seed(44)
    pt = torch.randint(0, 256, (n, L), dtype=torch.uint8, device="cuda", generator=g)
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    key = bytes(range(7, 71))
    ks = rt.KeySet(key)
    tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, pt, L, iv, tok)
    back = torch.empty((n, tl - 48), dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    device.decrypt_uniform(ks, tok, tl, back, ol, st)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0 and bool((ol == L).all()) and torch.equal(back[:, :L], pt)
    sel = np.sort(np.random.Generator(np.random.PCG64(45)).choice(n, 64, replace=False))
    s = torch.from_numpy(sel).cuda()
    ref, _, _ = _oracle_rows(np.frombuffer(key, np.uint8).reshape(1, 64), pt[s].cpu().numpy(), iv[s].cpu().numpy(),
                             None)
    assert np.array_equal(ref, tok[s].cpu().numpy())


def test_config_c5_rank_share(rt):
    """c5's per-rank share at 8 GPUs, on one GPU (the whole 8 M-packet batch
    is tests/test_c5_full_gpu.py): 2^20 packets of 64-4096 B, 65 536 keys, half encrypted
    and half decrypted (length-bucketed launches), 1 % of the decrypt half
    tampered: exactly the tampered tokens fail with BAD_HMAC, every other
    plaintext round-trips, and seeded samples of the encrypt output and of
    the decrypt output equal the oracle's."""
    import torch
    from reticulum_amd import device
    n, nk = 1 << 20, 65536
    rng = np.random.Generator(np.random.PCG64(55))
    keys = rng.integers(0, 256, (nk, 64), dtype=np.uint8)
    ks = rt.KeySet(keys)
    lens = rng.integers(64, 4097, n).astype(np.int32)
    off = np.zeros(n, np.int64)
    off[1:] = np.cumsum(lens[:-1])
    tl = (16 + 16 * (lens // 16 + 1) + 32).astype(np.int32)
    toff = np.zeros(n, np.int64)
    toff[1:] = np.cumsum(tl[:-1].astype(np.int64))
    g = torch.Generator(device="cuda").manual_seed(55)
    buf = torch.randint(0, 256, (int(lens.sum()),), dtype=torch.uint8, device="cuda", generator=g)
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    kidx = rng.integers(0, nk, n).astype(np.int32)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    d_off, d_len, d_toff, d_tl, d_k = cu(off), cu(lens), cu(toff), cu(tl), cu(kidx)
    tok = torch.zeros(int(tl.astype(np.int64).sum()), dtype=torch.uint8, device="cuda")
    ws = torch.empty(int(rt._native.load().rt_workspace_bytes(n)), dtype=torch.uint8, device="cuda")
    # encrypt half: packets [0, n/2); the decrypt half's tokens are made first
    # by encrypting [n/2, n), then 1 % of them are tampered
    h = n // 2
    device.encrypt(ks, buf, d_off[h:], d_len[h:], iv[h:], tok, d_toff[h:], key_idx=d_k[h:], sort=True, workspace=ws)
    torch.cuda.synchronize()
    bad = rng.random(n - h) < 0.01
    bad_idx = np.nonzero(bad)[0] + h
    flip = (toff[bad_idx] + rng.integers(0, tl[bad_idx])).astype(np.int64)
    tok[cu(flip)] ^= 1
    torch.cuda.synchronize()
    # the timed c5 shape: one encrypt of the first half and one decrypt of the second
    device.encrypt(ks, buf, d_off[:h], d_len[:h], iv[:h], tok, d_toff[:h], key_idx=d_k[:h], sort=True, workspace=ws)
    cap = tl.astype(np.int64) - 48
    coff = np.zeros(n, np.int64)
    coff[1:] = np.cumsum(cap[:-1])
    back = torch.zeros(int(cap.sum()), dtype=torch.uint8, device="cuda")
    ol = torch.empty(n - h, dtype=torch.int32, device="cuda")
    st = torch.full((n - h,), -1, dtype=torch.int32, device="cuda")
    ws2 = torch.empty_like(ws)
    device.decrypt(ks, tok, d_toff[h:], d_tl[h:], back, cu(coff[h:]), ol, st, key_idx=d_k[h:], sort=True,
                   workspace=ws2)
    torch.cuda.synchronize()
    sth, olh = st.cpu().numpy(), ol.cpu().numpy()
    assert np.array_equal(sth != 0, bad) and (sth[bad] == rt.RT_ST_BAD_HMAC).all()
    assert np.array_equal(olh[~bad], lens[h:][~bad]) and (olh[bad] == 0).all()
    # round trip of every untampered packet of the decrypt half, on the device
    good = np.nonzero(~bad)[0] + h
    src_idx = torch.from_numpy(np.concatenate([np.arange(off[i], off[i] + lens[i]) for i in good[:: 50]])).cuda()
    dst_idx = torch.from_numpy(np.concatenate([np.arange(coff[i], coff[i] + lens[i]) for i in good[:: 50]])).cuda()
    assert torch.equal(buf[src_idx], back[dst_idx])
    # oracle samples: encrypt half tokens, decrypt half plaintexts
    hb, hiv, htok, hback = buf.cpu().numpy(), iv.cpu().numpy(), tok.cpu().numpy(), back.cpu().numpy()
    for i in np.random.Generator(np.random.PCG64(56)).choice(h, 512, replace=False):
        p = hb[off[i]:off[i] + lens[i]].tobytes()
        want = oracle.encrypt(keys[kidx[i]].tobytes(), hiv[i].tobytes(), p)
        assert htok[toff[i]:toff[i] + tl[i]].tobytes() == want, i
    for i in np.random.Generator(np.random.PCG64(57)).choice(np.arange(h, n), 512, replace=False):
        s, p = oracle.decrypt(keys[kidx[i]].tobytes(), htok[toff[i]:toff[i] + tl[i]].tobytes())
        assert s == int(sth[i - h]), i
        if s == 0:
            assert hback[coff[i]:coff[i] + lens[i]].tobytes() == p, i


# ------------------------------------------------ key table from device memory

@pytest.mark.parametrize("klen", [64, 32])
def test_device_keyset_from_table(rt, klen):
    """device.keyset (the per-rank step after shard.broadcast_keys): a key
    table already in HBM expanded on the device; used at once from the device
    path and from the host path, every token bit-exact vs the oracle."""
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(41 + klen))
    nk, n, L = 300, 2000, 77
    keys = rng.integers(0, 256, (nk, klen), dtype=np.uint8)
    ks = device.keyset(torch.from_numpy(keys).cuda())
    assert (ks.n_keys, ks.key_len) == (nk, klen)
    kidx = rng.integers(0, nk, n).astype(np.int32)
    pt = rng.integers(0, 256, (n, L), dtype=np.uint8)
    iv = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    tl = rt.token_len(L)
    tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, torch.from_numpy(pt).cuda(), L, torch.from_numpy(iv).cuda(), tok,
                           key_idx=torch.from_numpy(kidx).cuda())
    torch.cuda.synchronize()
    t = tok.cpu().numpy()
    for i in range(0, n, 97):
        assert t[i].tobytes() == oracle.encrypt(keys[kidx[i]].tobytes(), iv[i].tobytes(), pt[i].tobytes())
    back, status = ks.decrypt_batch([t[i].tobytes() for i in range(n)], key_idx=kidx)
    assert (status == 0).all() and back.to_list() == [pt[i].tobytes() for i in range(n)]
    with pytest.raises(ValueError):
        device.keyset(torch.zeros((4, 48), dtype=torch.uint8, device="cuda"))


def test_device_keyset_on_side_stream_after_current_stream_fill(rt):
    """a key table filled on the current stream (as an
    RCCL broadcast leaves it: only the current stream waits for the
    collective) and expanded on a side stream, the caller dropping the table
    at once.  The side stream must wait for the fill and the table's memory
    must not be reused before the key setup read it: every token opens under
    the oracle with the table's keys."""
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(4242))
    nk, n, L = 512, 1500, 64
    keys = rng.integers(0, 256, (nk, 64), dtype=np.uint8)
    side = torch.cuda.Stream()
    for trial in range(3):
        table = torch.zeros((nk, 64), dtype=torch.uint8, device="cuda")
        # a slow producer on the current stream: spin the GPU, then fill
        torch.cuda._sleep(2_000_000)
        table.copy_(torch.from_numpy(keys).cuda(non_blocking=True))
        ks = device.keyset(table, stream=side)
        del table                                        # the caller lets go at once
        junk = torch.full((nk, 64), 0xA5, dtype=torch.uint8, device="cuda")   # may land on the freed block
        kidx = rng.integers(0, nk, n).astype(np.int32)
        pt = rng.integers(0, 256, (n, L), dtype=np.uint8)
        iv = rng.integers(0, 256, (n, 16), dtype=np.uint8)
        tok = torch.empty((n, rt.token_len(L)), dtype=torch.uint8, device="cuda")
        device.encrypt_uniform(ks, torch.from_numpy(pt).cuda(), L, torch.from_numpy(iv).cuda(), tok,
                               key_idx=torch.from_numpy(kidx).cuda())
        torch.cuda.synchronize()
        t = tok.cpu().numpy()
        for i in range(0, n, 61):
            assert t[i].tobytes() == oracle.encrypt(keys[kidx[i]].tobytes(), iv[i].tobytes(), pt[i].tobytes()), trial
        del junk


def test_counter_ring_eight_threads_ragged_launches(rt):
    """the chunk-counter ring holds no lock across a
    launch.  Eight host threads, each on its own torch stream, issue ragged
    launches (the dynamic chunk loop: one slot per launch) of their own
    batches, 1-key and per-packet-key, with the output zeroed before every
    launch; every output must equal the batch's reference (a slot handed to
    two launches at once, or zeroed under a running one, would skip or repeat
    chunks and leave zeros).  Prints launches/s for 1 and 8 threads."""
    import threading
    import time
    import torch
    from reticulum_amd import device
    base = [_ragged_case(rt, 262_211, 16, 1, 11), _ragged_case(rt, 196_999, 32, 77, 12)]   # > 1 pass, ragged
    n_thr, iters = 8, 150
    streams = [torch.cuda.Stream() for _ in range(n_thr)]
    outs = [torch.empty_like(base[t % 2][4]) for t in range(n_thr)]
    bad = [torch.zeros((), dtype=torch.int64, device="cuda") for _ in range(n_thr)]
    errors = []

    def worker(t, k):
        try:
            ks, pt, iv, ki, ref = base[t % 2]
            with torch.cuda.stream(streams[t]):
                for _ in range(k):
                    outs[t].zero_()
                    device.encrypt_uniform(ks, pt, pt.shape[1], iv, outs[t], key_idx=ki, stream=streams[t])
                    bad[t] += (outs[t] != ref).any(dim=1).sum()
        except Exception as e:   # noqa: BLE001 (reported below)
            errors.append(repr(e))

    rates = {}
    for nt in (1, n_thr):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        th = [threading.Thread(target=worker, args=(t, iters)) for t in range(nt)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        torch.cuda.synchronize()
        rates[nt] = nt * iters / (time.perf_counter() - t0)
    assert not errors, errors
    assert [int(b) for b in bad] == [0] * n_thr
    print(f"\nragged launches/s (launch + zero + compare per iteration): 1 thread {rates[1]:.0f}, "
          f"{n_thr} threads {rates[n_thr]:.0f}")
