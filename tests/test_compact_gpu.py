"""rt_frames_compact and rt_token_spans (the inbound pipeline's glue between
deframing, IFAC unmask, unpack and decrypt) against a numpy restatement of
what they must do: the frames a read hands on (TCPInterface.py:391-401) in
stream order with empty entries past them, and each unpacked packet's data
span (Packet.py:262-275)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _compact_expected(d_off, d_len, st, pairs):
    m = len(d_off)
    ok = (np.arange(m) < pairs) & (st == 0)
    k = np.nonzero(ok)[0]
    f_off = np.zeros(m, np.int64)
    f_len = np.zeros(m, np.int32)
    fp = np.full(m, -1, np.int64)
    f_off[:len(k)], f_len[:len(k)], fp[:len(k)] = d_off[k], d_len[k], k
    return f_off, f_len, fp, len(k)


@pytest.mark.parametrize("m,pairs,p_ok", [(1, 1, 1.0), (1, 0, 1.0), (1000, 999, 0.5), (1024, 1024, 1.0),
                                          (1025, 2000, 0.5), (5000, 3000, 0.0), (70001, 70001, 0.47),
                                          (2 ** 21, 2 ** 21 - 1, 0.5)])
def test_frames_compact_matches_the_read_loop(m, pairs, p_ok):
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(m + pairs))
    d_off = rng.integers(0, 1 << 40, m, dtype=np.int64)
    d_len = rng.integers(0, 1 << 20, m, dtype=np.int32)
    st = np.where(rng.random(m) < p_ok, 0, rng.integers(1, 3, m)).astype(np.int32)
    st[pairs:] = -1
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    counts = t(np.array([pairs, 0], np.int64))
    f_off = torch.full((m,), 7, dtype=torch.int64, device="cuda")         # garbage the kernel must overwrite
    f_len = torch.full((m,), 7, dtype=torch.int32, device="cuda")
    fp = torch.full((m,), 7, dtype=torch.int64, device="cuda")
    n = torch.full((), 7, dtype=torch.int64, device="cuda")
    device.frames_compact(t(d_off), t(d_len), t(st), counts, f_off, f_len, fp, n)
    e_off, e_len, e_fp, e_n = _compact_expected(d_off, d_len, st, pairs)
    assert int(n) == e_n
    assert np.array_equal(f_off.cpu().numpy(), e_off)
    assert np.array_equal(f_len.cpu().numpy(), e_len)
    assert np.array_equal(fp.cpu().numpy(), e_fp)


def test_frames_compact_empty():
    import torch
    from reticulum_amd import device
    e64 = torch.empty(0, dtype=torch.int64, device="cuda")
    e32 = torch.empty(0, dtype=torch.int32, device="cuda")
    n = torch.full((), 7, dtype=torch.int64, device="cuda")
    device.frames_compact(e64, e32, e32, torch.zeros(2, dtype=torch.int64, device="cuda"), e64.clone(), e32.clone(),
                          e64.clone(), n)
    assert int(n) == 0


@pytest.mark.parametrize("n", [1, 255, 256, 257, 100003])
def test_token_spans_follow_unpack_records(n):
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(n))
    fields = rng.integers(0, 256, (n, 96), dtype=np.uint8)
    fields[:, 0] = np.where(rng.random(n) < 0.7, 1, rng.integers(0, 3, n))       # ok flag (2 is not ok)
    words = fields.view(np.uint32)
    words[:, 3] = rng.integers(0, 36, n)              # data_offset
    words[:, 4] = rng.integers(0, 1 << 20, n)         # data_len
    off = rng.integers(0, 1 << 40, n, dtype=np.int64)
    tok_off = torch.empty(n, dtype=torch.int64, device="cuda")
    tok_len = torch.empty(n, dtype=torch.int32, device="cuda")
    device.token_spans(torch.from_numpy(fields).cuda(), torch.from_numpy(off).cuda(), tok_off, tok_len)
    ok = fields[:, 0] == 1
    assert np.array_equal(tok_off.cpu().numpy(), np.where(ok, off + words[:, 3].astype(np.int64), off))
    assert np.array_equal(tok_len.cpu().numpy(), np.where(ok, words[:, 4], 0).astype(np.int32))
