"""The round-5 routing rules at their edges, against the C oracle:

* the split encrypt takes its 64-packet batches from a chunk counter when
  the static stride would load its AES waves unevenly (batches not a multiple
  of 8 x CUs) and packets are at least RNSTOK_SPLIT_DYN_MIN_LEN (256) bytes;
* uniform tokens of at most RNSTOK_DEC1024_MAX_TOKEN (320) bytes decrypt on
  the 1024-thread instance at every batch size.

Batch sizes and lengths just below, at and above each threshold, one key and
per-packet keys: every packet round-trips, a sample of tokens equals the
oracle's (Token.encrypt, Token.py:87-97), and 1 % tampered tokens fail with
BAD_HMAC and a zeroed plaintext exactly where the oracle says
(Token.decrypt, Token.py:100-114)."""
import numpy as np
import pytest

from oracle import ctoken as oracle

pytestmark = pytest.mark.gpu


def _n_cu():
    from reticulum_amd import _native
    return _native.load().rt_num_cus(_native.context(0))


def _cases():
    out = []
    for L in (255, 256, 271, 272):                           # split counter min length; short-token edge
        for extra_batches in (0, 1, 7):                      # even load, one batch over, a few over
            out.append((L, extra_batches, 1))
    out += [(256, 1, 300), (271, 0, 300), (500, 3, 1), (1000, 1, 97)]
    return out


@pytest.mark.parametrize("L,extra_batches,n_keys", _cases())
def test_routing_edges_round_trip_and_tamper(L, extra_batches, n_keys):
    import torch
    import reticulum_amd as rt
    from reticulum_amd import _native, device
    n_cu = _n_cu()
    n = 64 * (8 * n_cu * 2 + extra_batches) - (5 if extra_batches else 0)   # 2 batches per AES wave (+ extra)
    tl = rt.token_len(L)
    lib, ctx = _native.load(), _native.context(0)
    assert lib.rt_plan_uniform(ctx, n, L, int(n_keys > 1), 0) == _native.RT_KERNEL_ENC_SPLIT
    rng = np.random.Generator(np.random.PCG64(7000 + L * 31 + extra_batches * 7 + n_keys))
    keys = rng.integers(0, 256, (n_keys, 64), dtype=np.uint8)
    ks = rt.KeySet(keys if n_keys > 1 else keys[0].tobytes())
    kx = rng.integers(0, n_keys, n).astype(np.int32)
    kidx = torch.from_numpy(kx).cuda() if n_keys > 1 else None
    pt = torch.from_numpy(rng.integers(0, 256, (n, L), dtype=np.uint8)).cuda()
    iv = torch.from_numpy(rng.integers(0, 256, (n, 16), dtype=np.uint8)).cuda()
    tok = torch.full((n, tl), 0xEE, dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, pt, L, iv, tok, key_idx=kidx)
    torch.cuda.synchronize()
    t, p_h, iv_h = tok.cpu().numpy(), pt.cpu().numpy(), iv.cpu().numpy()
    kk = kx if n_keys > 1 else np.zeros(n, np.int64)
    for i in np.unique(np.concatenate([[0, 63, 64, n - 65, n - 1], rng.integers(0, n, 40)])):
        assert t[i].tobytes() == oracle.encrypt(keys[kk[i]].tobytes(), iv_h[i].tobytes(), p_h[i].tobytes()), i
    bad = rng.choice(n, max(n // 100, 1), replace=False)
    for j, i in enumerate(bad):
        t[i, int(rng.integers(0, tl))] ^= 1 << int(j % 8)
    tok2 = torch.from_numpy(t).cuda()
    out = torch.full((n, tl - 48), 0x33, dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    device.decrypt_uniform(ks, tok2, tl, out, ol, st, key_idx=kidx)
    torch.cuda.synchronize()
    st_h, ol_h, back = st.cpu().numpy(), ol.cpu().numpy(), out.cpu().numpy()
    assert set(np.nonzero(st_h != 0)[0].tolist()) == set(int(i) for i in bad)
    for i in bad[:20]:
        s, _ = oracle.decrypt(keys[kk[i]].tobytes(), t[i].tobytes())
        assert st_h[i] == s == 2 and not back[i].any(), i
    ok = st_h == 0
    assert bool((ol_h[ok] == L).all()) and np.array_equal(back[ok, :L], p_h[ok])
