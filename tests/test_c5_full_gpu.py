"""BASELINE config c5 as ONE batch on one GPU: 8 M packets (2^23) of 64-4096 B,
65 536 per-packet keys, half encrypted and half decrypted through the
length-bucketed packed launches (the reference's per-packet Token.encrypt /
Token.decrypt, RNS/Cryptography/Token.py:87-114, with per-packet keys,
RNS/Identity.py:829-845), 1 % of the decrypt half tampered.  About 45 GB of
HBM; one MI355X holds it.

Size-independent checks over EVERY packet, on the device:
* the decrypt half: exactly the tampered tokens fail (BAD_HMAC), every other
  plaintext equals its source bytes and its out_len its length;
* the encrypt half: every token decrypts back to its plaintext (round trip)
  and no token fails;
plus seeded oracle samples (C oracle, tests only) from every length bucket
of both halves: tokens bit-exact, statuses and plaintexts equal."""
import numpy as np
import pytest

from oracle import ctoken as oracle

pytestmark = pytest.mark.gpu

N, NK = 1 << 23, 65536


@pytest.fixture(scope="module")
def rt():
    import reticulum_amd
    from reticulum_amd import _native
    assert _native.load().rt_device_count() >= 1, "no HIP device visible"
    _native.context(0)
    return reticulum_amd


def _segments_equal(a, a_off, b, b_off, lens, chunk=1 << 16):
    """For every packet i: a[a_off[i] : a_off[i] + lens[i]] == b[b_off[i] : ...]
    (device tensors; index tensors built per chunk of packets on the device).
    Returns the indices of packets that differ."""
    import torch
    bad = []
    n = lens.numel()
    for s in range(0, n, chunk):
        ln = lens[s:s + chunk].to(torch.int64)
        tot = int(ln.sum())
        if tot == 0:
            continue
        seg = torch.repeat_interleave(torch.arange(ln.numel(), device=ln.device), ln)
        start = torch.cumsum(ln, 0) - ln
        pos = torch.arange(tot, device=ln.device) - start[seg]
        ia, ib = a_off[s:s + chunk][seg] + pos, b_off[s:s + chunk][seg] + pos
        diff = a[ia] != b[ib]
        if bool(diff.any()):
            bad.extend((s + torch.unique(seg[diff])).tolist())
        del seg, pos, ia, ib, diff
    return bad


def _bucket_sample(lens, idx, k, seed):
    """k packet indices from `idx`, spread over 16 length buckets."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    edges = np.linspace(64, 4097, 17)
    for lo, hi in zip(edges[:-1], edges[1:]):
        sel = idx[(lens[idx] >= lo) & (lens[idx] < hi)]
        if sel.size:
            out.extend(rng.choice(sel, min(k // 16, sel.size), replace=False).tolist())
    return out


def test_config_c5_whole_batch(rt):
    import torch
    from reticulum_amd import device
    n, nk, h = N, NK, N // 2
    rng = np.random.Generator(np.random.PCG64(505))
    keys = rng.integers(0, 256, (nk, 64), dtype=np.uint8)
    ks = rt.KeySet(keys)
    lens = rng.integers(64, 4097, n).astype(np.int32)
    off = np.zeros(n, np.int64)
    off[1:] = np.cumsum(lens[:-1])
    tl = (16 + 16 * (lens // 16 + 1) + 32).astype(np.int32)
    toff = np.zeros(n, np.int64)
    toff[1:] = np.cumsum(tl[:-1].astype(np.int64))
    cap = tl.astype(np.int64) - 48
    coff = np.zeros(n, np.int64)
    coff[1:] = np.cumsum(cap[:-1])
    kidx = rng.integers(0, nk, n).astype(np.int32)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    d_off, d_len, d_toff, d_tl, d_k, d_coff = cu(off), cu(lens), cu(toff), cu(tl), cu(kidx), cu(coff)
    g = torch.Generator(device="cuda").manual_seed(505)
    buf = torch.randint(0, 256, (int(lens.astype(np.int64).sum()),), dtype=torch.uint8, device="cuda", generator=g)
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    tok = torch.zeros(int(tl.astype(np.int64).sum()), dtype=torch.uint8, device="cuda")
    ws = torch.empty(int(rt._native.load().rt_workspace_bytes(n)), dtype=torch.uint8, device="cuda")
    # the decrypt half's tokens are made first, then 1 % of them tampered
    device.encrypt(ks, buf, d_off[h:], d_len[h:], iv[h:], tok, d_toff[h:], key_idx=d_k[h:], sort=True, workspace=ws)
    torch.cuda.synchronize()
    bad = rng.random(n - h) < 0.01
    bad_idx = np.nonzero(bad)[0] + h
    flip = (toff[bad_idx] + rng.integers(0, tl[bad_idx])).astype(np.int64)
    tok[cu(flip)] ^= 1
    # c5 itself: one encrypt of the first half, one decrypt of the second
    device.encrypt(ks, buf, d_off[:h], d_len[:h], iv[:h], tok, d_toff[:h], key_idx=d_k[:h], sort=True, workspace=ws)
    back = torch.zeros(int(cap.sum()), dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    ws2 = torch.empty_like(ws)
    device.decrypt(ks, tok, d_toff[h:], d_tl[h:], back, d_coff[h:], ol[h:], st[h:], key_idx=d_k[h:], sort=True,
                   workspace=ws2)
    torch.cuda.synchronize()
    sth, olh = st[h:].cpu().numpy(), ol[h:].cpu().numpy()
    # the exact tamper set
    assert np.array_equal(sth != 0, bad) and (sth[bad] == rt.RT_ST_BAD_HMAC).all()
    assert np.array_equal(olh[~bad], lens[h:][~bad]) and (olh[bad] == 0).all()
    # every untampered plaintext of the decrypt half equals its source
    good = torch.from_numpy(np.nonzero(~bad)[0] + h).cuda()
    assert _segments_equal(buf, d_off[good], back, d_coff[good], d_len[good]) == []
    # round trip of every token of the encrypt half
    device.decrypt(ks, tok, d_toff[:h], d_tl[:h], back, d_coff[:h], ol[:h], st[:h], key_idx=d_k[:h], sort=True,
                   workspace=ws2)
    torch.cuda.synchronize()
    assert bool((st[:h] == 0).all()) and torch.equal(ol[:h], d_len[:h])
    assert _segments_equal(buf, d_off[:h], back, d_coff[:h], d_len[:h]) == []
    # oracle samples over the length buckets: encrypt-half tokens, decrypt-half statuses and plaintexts
    hiv = iv.cpu().numpy()
    for i in _bucket_sample(lens, np.arange(h), 512, 506):
        p = buf[off[i]:off[i] + lens[i]].cpu().numpy().tobytes()
        want = oracle.encrypt(keys[kidx[i]].tobytes(), hiv[i].tobytes(), p)
        assert tok[toff[i]:toff[i] + tl[i]].cpu().numpy().tobytes() == want, i
    for i in _bucket_sample(lens, np.arange(h, n), 512, 507) + bad_idx[:32].tolist():
        s, p = oracle.decrypt(keys[kidx[i]].tobytes(), tok[toff[i]:toff[i] + tl[i]].cpu().numpy().tobytes())
        assert s == int(sth[i - h]), i
        if s == 0:
            assert back[coff[i]:coff[i] + lens[i]].cpu().numpy().tobytes() == p, i
