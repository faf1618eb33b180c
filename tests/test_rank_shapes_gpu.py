"""The exact per-rank shapes of the 8-GPU runs (VERDICT r02 missing #5).

At N = 8 the driver's SCALE run takes its c4 numbers from each rank's
32 768 x 16 KiB share (exactly 128 tokens per CU on 256 CUs, which routes to
the long-token kernels k_encrypt_long4 / k_decrypt_long2) and its c5 numbers
from each rank's 2^20 mixed packets under 65 536 keys.  These tests run those
shapes on one GPU: the kernel plan of the shape, a full round trip, and a
seeded oracle sample; and bench.sharded_bench's own per-rank work functions
at those sizes (world size 1: the work runs directly, its outputs checked)."""
import argparse

import numpy as np
import pytest

from oracle import ctoken as oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    from reticulum_amd import _native
    lib = _native.load()
    assert lib.rt_device_count() >= 1, "no HIP device visible"
    return lib


def test_c4_rank_shape_runs_long_kernels_bit_exact(lib):
    import torch
    import reticulum_amd as rt
    from reticulum_amd import _native, device
    ctx = _native.context(0)
    n_cu = lib.rt_num_cus(ctx)
    n, L = 128 * n_cu, 16384                  # 32 768 on MI355X: c4 / 8 ranks
    tl = rt.token_len(L)
    assert lib.rt_plan_uniform(ctx, n, L, 0, 0) == _native.RT_KERNEL_ENC_LONG4
    assert lib.rt_plan_uniform(ctx, n, tl, 0, 1) == _native.RT_KERNEL_DEC_LONG2
    # one more token per CU leaves the long-token kernels (the routing edge)
    assert lib.rt_plan_uniform(ctx, n + 1, L, 0, 0) == _native.RT_KERNEL_GENERAL
    assert lib.rt_plan_uniform(ctx, n + 1, tl, 0, 1) == _native.RT_KERNEL_GENERAL
    g = torch.Generator(device="cuda").manual_seed(32768)
    pt = torch.randint(0, 256, (n, L), dtype=torch.uint8, device="cuda", generator=g)
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    key = np.random.Generator(np.random.PCG64(16384)).integers(0, 256, 64, dtype=np.uint8)
    ks = rt.KeySet(key.tobytes())
    tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    device.encrypt_uniform(ks, pt, L, iv, tok)
    back = torch.empty((n, tl - 48), dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    device.decrypt_uniform(ks, tok, tl, back, ol, st)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0 and bool((ol == L).all())
    assert torch.equal(back[:, :L], pt)
    # seeded sample (first, last, and every wave / workgroup edge class) vs the oracle
    rng = np.random.Generator(np.random.PCG64(7))
    sel = np.unique(np.concatenate([[0, 1, 15, 16, 127, 128, n - 1], rng.integers(0, n, 41)]))
    idx = torch.from_numpy(sel).cuda()
    s_pt, s_iv, s_tok = pt[idx].cpu().numpy(), iv[idx].cpu().numpy(), tok[idx].cpu().numpy()
    m = len(sel)
    ref = np.zeros(m * tl, np.uint8)
    oracle.encrypt_batch(key.reshape(1, 64), s_pt.reshape(-1), np.arange(m, dtype=np.uint64) * L,
                         np.full(m, L, np.uint32), None, s_iv, ref, np.arange(m, dtype=np.uint64) * tl, threads=8)
    assert np.array_equal(ref.reshape(m, tl), s_tok)
    # a tampered token of this shape fails exactly there, its plaintext zeroed
    tok[777, 5000] ^= 1
    device.decrypt_uniform(ks, tok, tl, back, ol, st)
    torch.cuda.synchronize()
    bad = torch.nonzero(st).flatten().tolist()
    assert bad == [777] and int(st[777]) == rt.RT_ST_BAD_HMAC and int(back[777].abs().sum()) == 0


@pytest.mark.parametrize("cfg", ["c4", "c5"])
def test_sharded_bench_work_at_8gpu_rank_share(cfg):
    """bench.sharded_bench's per-rank work functions at one rank's share of an
    8-GPU run: c4 32 768 x 16 KiB (one key), c5 2^20 packets of 64 B-4 KiB
    under 65 536 keys, half encrypted and half decrypted (length-bucketed).
    Every token of the encrypt half is decrypted back and compared; the
    decrypt half's plaintexts are compared with the inputs."""
    import bench
    from reticulum_amd import _native
    n_cu = _native.load().rt_num_cus(_native.context(0))
    shard_n = 128 * n_cu if cfg == "c4" else 1 << 20
    args = argparse.Namespace(packets=1 << 20, shard_n=shard_n, sharded_chunks=0)
    rep = bench.sharded_bench(cfg, args, world=1, rank=0, local=0, reps=1)
    assert rep["ok"] is True
    assert rep["config"]["packets"] == shard_n
    assert rep["value"] > 0
