"""HKDF-SHA256 (RNS/Cryptography/HKDF.py:35-62) and per-packet keying
(Identity.py:837-846).

CPU: the C oracle against the golden vectors made from the reference
(tests/golden/gen_hkdf.py), including the derivation the reference performs
while decrypting its own identity KAT (tests/identity.py:11-19,148-158); the
host layer's argument errors and batching logic (fake library).
GPU (-m gpu): the k_hkdf kernel through the C-ABI, bit-exact against the same
vectors and the oracle, and the derived-keyset path end to end.
"""
import numpy as np
import pytest

import reticulum_amd as rt
from oracle import ctoken
from tests_helpers import b


def _h(x):
    return None if x is None else bytes.fromhex(x)


@pytest.fixture
def fake(monkeypatch):
    import fake_native
    return fake_native.install(monkeypatch)


# ------------------------------------------------------------------ oracle --

def test_oracle_hkdf_vectors(golden_hkdf):
    for v in golden_hkdf["vectors"]:
        assert ctoken.hkdf(v["length"], _h(v["ikm"]), _h(v["salt"]), _h(v["context"])).hex() == v["okm"], v["note"]
    bt = golden_hkdf["batch"]
    for ikm, salt, okm in zip(bt["ikm"], bt["salt"], bt["okm"]):
        assert ctoken.hkdf(bt["length"], b(ikm), b(salt)).hex() == okm


def test_oracle_hkdf_identity_kat(golden_hkdf, golden):
    """The reference's own derivation while decrypting fixed_token: the okm is
    the token key captured in token_vectors.json, and it opens the token."""
    k = golden_hkdf["identity_kat"]
    okm = ctoken.hkdf(k["length"], b(k["ikm"]), _h(k["salt"]), _h(k["context"]))
    assert okm.hex() == k["okm"] == golden["kat"]["fixed_token"]["derived_key"]
    st, pt = ctoken.decrypt(okm, b(golden["kat"]["fixed_token"]["token"]))
    assert st == 0 and pt.hex() == golden["kat"]["fixed_token"]["pt"]


def test_oracle_hkdf_errors(golden_hkdf):
    for e in golden_hkdf["errors"]:
        ikm = None if e["derive_from"] is None else ("" if e["derive_from"] == "str:" else b(e["derive_from"]))
        with pytest.raises(ValueError) as ex:
            ctoken.hkdf(e["length"], ikm)
        assert str(ex.value) == e["msg"]


# -------------------------------------------------------------- host layer --

def test_hkdf_argument_errors_match_reference(golden_hkdf):
    """Raised before any native call, with the reference's messages."""
    for e in golden_hkdf["errors"]:
        ikm = None if e["derive_from"] is None else ("" if e["derive_from"] == "str:" else b(e["derive_from"]))
        with pytest.raises(ValueError) as ex:
            rt.hkdf(length=e["length"], derive_from=ikm)
        assert str(ex.value) == e["msg"]
        with pytest.raises(ValueError):
            rt.hkdf_batch(e["length"], [ikm] if ikm is not None else None)
    with pytest.raises(TypeError):
        rt.hkdf(length=3, derive_from=b"abc", context="x")      # bytes + str in the reference
    with pytest.raises(ValueError):
        rt.derive_keyset([b"x" * 32], key_len=48)


def test_hkdf_host_layer_groups_mixed_lengths(fake, golden_hkdf):
    """Mixed ikm / salt lengths (salt None, b"" and bytes) are split into
    uniform launches and reassembled in order."""
    vs = [v for v in golden_hkdf["vectors"] if v["context"] is None and v["length"] == 64]
    ikm = [_h(v["ikm"]) for v in vs]
    salt = [_h(v["salt"]) for v in vs]
    out = rt.hkdf_batch(64, ikm, salt)
    assert [o.tobytes().hex() for o in out] == [v["okm"] for v in vs]
    launches = [c for c in fake.calls if c[0] == "rt_hkdf_host"]
    assert len(launches) == len({(len(i), 0 if s is None else len(s)) for i, s in zip(ikm, salt)})
    for v in golden_hkdf["vectors"]:
        assert rt.hkdf(v["length"], _h(v["ikm"]), _h(v["salt"]), _h(v["context"])).hex() == v["okm"], v["note"]


# --------------------------------------------------------------------- GPU --

@pytest.mark.gpu
def test_gpu_hkdf_golden(golden_hkdf):
    for v in golden_hkdf["vectors"]:
        assert rt.hkdf(v["length"], _h(v["ikm"]), _h(v["salt"]), _h(v["context"])).hex() == v["okm"], v["note"]
    bt = golden_hkdf["batch"]
    out = rt.hkdf_batch(bt["length"], [b(x) for x in bt["ikm"]], [b(x) for x in bt["salt"]])
    assert [o.tobytes().hex() for o in out] == bt["okm"]
    k = golden_hkdf["identity_kat"]
    assert rt.hkdf(k["length"], b(k["ikm"]), _h(k["salt"]), _h(k["context"])).hex() == k["okm"]


@pytest.mark.gpu
@pytest.mark.parametrize("salt_len,ctx_len,length", [(16, 0, 64), (0, 0, 32), (100, 30, 200), (64, 1, 33),
                                                    (64, 0, 64), (20, 0, 100), (18, 0, 64),
                                                    # the longest output HKDF allows (255 blocks), a context
                                                    # longer than a block
                                                    (16, 0, 8160), (0, 100, 8160), (32, 200, 96)])
def test_gpu_hkdf_device_batch_vs_oracle(salt_len, ctx_len, length):
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(salt_len * 7 + ctx_len + length))
    n = 3000
    ikm = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    salt = rng.integers(0, 256, (n, salt_len), dtype=np.uint8) if salt_len else None
    ctxb = rng.integers(0, 256, ctx_len, dtype=np.uint8).tobytes() if ctx_len else None
    out = torch.zeros((n, length), dtype=torch.uint8, device="cuda")
    device.hkdf(torch.from_numpy(ikm).cuda(), out, None if salt is None else torch.from_numpy(salt).cuda(),
                None if ctxb is None else torch.frombuffer(bytearray(ctxb), dtype=torch.uint8).cuda())
    got = out.cpu().numpy()
    for i in range(0, n, 97):
        ref = ctoken.hkdf(length, ikm[i].tobytes(), None if salt is None else salt[i].tobytes(), ctxb)
        assert got[i].tobytes() == ref, i



@pytest.mark.gpu
@pytest.mark.parametrize("ikm_len,ikm_stride", [(0, 4), (4, 4), (52, 52), (53, 53), (56, 56), (32, 34), (48, 64)])
def test_gpu_hkdf_ikm_shapes_vs_oracle(ikm_len, ikm_stride):
    """Both kernel instances: whole-word, <= 52-byte ikm at 4-aligned strides
    takes the FAST instance (dword loads, one-block PRK message); 53/56 bytes
    and the 34-byte stride take the generic byte-load instance."""
    import torch
    from reticulum_amd import _native
    rng = np.random.Generator(np.random.PCG64(1000 + ikm_len * 3 + ikm_stride))
    n = 2000
    ikm = torch.from_numpy(rng.integers(0, 256, n * ikm_stride + 1, dtype=np.uint8)).cuda()
    salt = torch.from_numpy(rng.integers(0, 256, (n, 16), dtype=np.uint8)).cuda()
    out = torch.zeros((n, 64), dtype=torch.uint8, device="cuda")
    lib = _native.load()
    ctx = _native.context(0)
    rc = lib.rt_hkdf(ctx, ikm.data_ptr(), ikm_stride, ikm_len, salt.data_ptr(), 16, 16, None, 0,
                     out.data_ptr(), 64, 64, n, torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    got, ih, sh = out.cpu().numpy(), ikm.cpu().numpy(), salt.cpu().numpy()
    for i in list(range(0, n, 89)) + [n - 1]:
        ref = ctoken.hkdf(64, ih[i * ikm_stride:i * ikm_stride + ikm_len].tobytes(), sh[i].tobytes(), None)
        assert got[i].tobytes() == ref, i


@pytest.mark.gpu
@pytest.mark.parametrize("salt_len,n", [(16, 70000), (16, 1), (18, 3000), (100, 3000)])
def test_gpu_hkdf_shared_salt_vs_oracle(salt_len, n):
    """salt_stride 0 (one salt row for every key, Identity.py:837-846 to one
    identity): the grid-stride instance computes the salt's midstates once per
    lane.  Also through rt_hkdf_host, which copies the one salt row."""
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(7000 + salt_len + n))
    ikm = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    salt = rng.integers(0, 256, (1, salt_len), dtype=np.uint8)
    out = torch.zeros((n, 64), dtype=torch.uint8, device="cuda")
    device.hkdf(torch.from_numpy(ikm).cuda(), out, torch.from_numpy(salt).cuda().expand(n, salt_len))
    got = out.cpu().numpy()
    for i in sorted(set(list(range(0, n, max(1, n // 40))) + [n - 1])):
        assert got[i].tobytes() == ctoken.hkdf(64, ikm[i].tobytes(), salt[0].tobytes(), None), i
    from reticulum_amd import _native
    host = np.zeros((n, 64), dtype=np.uint8)
    rc = _native.load().rt_hkdf_host(_native.context(0), ikm.ctypes.data, 32, 32, salt.ctypes.data, 0, salt_len,
                                     None, 0, host.ctypes.data, 64, 64, n)
    assert rc == 0 and np.array_equal(host, got)


@pytest.mark.gpu
def test_gpu_hkdf_shared_salt_grid_stride():
    """600000 keys over the 1024 x 256-lane grid: lanes derive 2 or 3 keys."""
    import torch
    from reticulum_amd import device
    n = 600000
    g = torch.Generator(device="cuda").manual_seed(5)
    ikm = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device="cuda", generator=g)
    salt = torch.randint(0, 256, (1, 16), dtype=torch.uint8, device="cuda", generator=g)
    out = torch.zeros((n, 64), dtype=torch.uint8, device="cuda")
    ref = torch.zeros((n, 64), dtype=torch.uint8, device="cuda")
    device.hkdf(ikm, out, salt.expand(n, 16))
    device.hkdf(ikm, ref, salt.repeat(n, 1))          # per-row instance, same salt in every row
    assert torch.equal(out, ref)
    ih, sh, oh = ikm.cpu().numpy(), salt.cpu().numpy(), out.cpu().numpy()
    for i in (0, 262143, 262144, 524288, n - 1):
        assert oh[i].tobytes() == ctoken.hkdf(64, ih[i].tobytes(), sh[0].tobytes(), None), i

@pytest.mark.gpu
def test_gpu_derived_keyset_identity_kat(golden_hkdf, golden):
    """Identity.__decrypt's derivation + Token on the device: the keyset
    derived from the reference KAT's shared key and identity-hash salt opens
    the reference's fixed_token."""
    k = golden_hkdf["identity_kat"]
    ks = rt.derive_keyset([b(k["ikm"])], [b(k["salt"])], key_len=64)
    pts, st = ks.decrypt_batch([b(golden["kat"]["fixed_token"]["token"])])
    assert int(st[0]) == 0 and pts[0].hex() == golden["kat"]["fixed_token"]["pt"]


@pytest.mark.gpu
@pytest.mark.parametrize("key_len", [64, 32])
def test_gpu_derived_keyset_per_packet_tokens(key_len):
    """Per-packet keying at batch scale: key i = hkdf(key_len, ikm_i, salt_i);
    tokens with key_idx = i match the oracle with the oracle's derived keys."""
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(key_len))
    n, L = 4096, 383                        # Packet.ENCRYPTED_MDU
    ikm = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    salt = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    ks = device.derive_keyset(torch.from_numpy(ikm).cuda(), torch.from_numpy(salt).cuda(), key_len=key_len)
    pt = rng.integers(0, 256, (n, L), dtype=np.uint8)
    iv = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    tl = rt.token_len(L)
    tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
    kidx = torch.arange(n, dtype=torch.int32, device="cuda")
    device.encrypt_uniform(ks, torch.from_numpy(pt).cuda(), L, torch.from_numpy(iv).cuda(), tok, key_idx=kidx)
    th = tok.cpu().numpy()
    for i in range(0, n, 61):
        key = ctoken.hkdf(key_len, ikm[i].tobytes(), salt[i].tobytes())
        assert th[i].tobytes() == ctoken.encrypt(key, iv[i].tobytes(), pt[i].tobytes()), i


@pytest.mark.gpu
def test_gpu_keyset_record_buffer_reuse():
    """Per-batch key sets: destroying a key set returns its record buffer to
    the context's cache and the next key set of a similar size reuses it.
    Every reused set must be fully rewritten: tokens of batch k match the
    oracle under batch k's own keys (never a previous batch's), for sizes
    that hit the cache (equal, slightly smaller) and one that does not."""
    import gc
    import torch
    from reticulum_amd import device
    L = 100
    tl = rt.token_len(L)
    for step, n in enumerate([3000, 3000, 2900, 3000, 700, 3000]):
        rng = np.random.Generator(np.random.PCG64(100 + step))
        ikm = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        salt = rng.integers(0, 256, (n, 16), dtype=np.uint8)
        ks = device.derive_keyset(torch.from_numpy(ikm).cuda(), torch.from_numpy(salt).cuda(), key_len=64)
        pt = rng.integers(0, 256, (n, L), dtype=np.uint8)
        iv = rng.integers(0, 256, (n, 16), dtype=np.uint8)
        tok = torch.empty((n, tl), dtype=torch.uint8, device="cuda")
        device.encrypt_uniform(ks, torch.from_numpy(pt).cuda(), L, torch.from_numpy(iv).cuda(), tok,
                               key_idx=torch.arange(n, dtype=torch.int32, device="cuda"))
        th = tok.cpu().numpy()
        for i in list(range(0, n, 97)) + [n - 1]:
            key = ctoken.hkdf(64, ikm[i].tobytes(), salt[i].tobytes())
            assert th[i].tobytes() == ctoken.encrypt(key, iv[i].tobytes(), pt[i].tobytes()), (step, i)
        del ks
        gc.collect()
