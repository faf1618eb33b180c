"""Resource hashmap (RNS/Resource.py:426-468, get_map_hash :505-506).

CPU: the oracle against fixtures made by the reference itself
(tests/golden/gen_resource.py: real RNS.Resource constructions over a stub
link, and the reference's hashmap loop over streams with repeated parts);
the host layer's loop through the fake library.  GPU (-m gpu): the
k_map_hashes / k_map_collisions kernels through the C-ABI, bit-exact.
"""
import json
import os

import numpy as np
import pytest

import reticulum_amd as rt
from oracle import ctoken
from tests_helpers import b, collision_stream

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def rv():
    with open(os.path.join(HERE, "golden", "resource_vectors.json")) as f:
        d = json.load(f)
    for c in d["collisions"]:          # inputs are stored as (seed, length, dup)
        c["stream"] = collision_stream(c["seed"], c["stream_len"], c["dup"], d["sdu_default"]).hex()
    return d


@pytest.fixture
def fake(monkeypatch):
    import fake_native
    return fake_native.install(monkeypatch)


def test_constants_match_reference(rv):
    from reticulum_amd import resource
    assert (resource.SDU, resource.MAPHASH_LEN, resource.RANDOM_HASH_SIZE, resource.COLLISION_GUARD_SIZE) == (
        rv["sdu_default"], rv["maphash_len"], rv["random_hash_size"], rv["collision_guard_size"])


def test_oracle_reference_resources(rv):
    for r in rv["resources"]:
        assert ctoken.map_hashes(b(r["stream"]), b(r["random_hash"]), r["sdu"]).hex() == r["hashmap"], r["size"]


def test_oracle_collision_guard(rv):
    g = rv["collision_guard_size"]
    for c in rv["collisions"]:
        hm = ctoken.map_hashes(b(c["stream"]), b(c["random_hash"]), rv["sdu_default"])
        assert hm.hex() == c["map_hashes"]
        col = ctoken.first_collision(hm, g)
        assert col == c["first_collision"], c["dup"]
        if col is not None:
            assert hm[:4 * col].hex() == c["hashmap_until_break"]


def test_host_layer_loop(rv, fake):
    """build_hashmap re-rolls on a collision exactly where the reference
    loop breaks, and returns the accepted hashmap."""
    r = rv["resources"][-1]
    assert rt.resource_hashmap(b(r["stream"]), b(r["random_hash"]))[0].hex() == r["hashmap"]
    draws = iter([b(r["random_hash"]), b"\x01\x02\x03\x04"])
    rh, hm = rt.build_hashmap(b(r["stream"]), random_hash=lambda: next(draws))
    assert rh == b(r["random_hash"]) and hm.hex() == r["hashmap"]      # accepted on the first draw
    c = [c for c in rv["collisions"] if c["first_collision"] is not None][0]
    _, col = rt.resource_hashmap(b(c["stream"]), b(c["random_hash"]))
    assert col == c["first_collision"]
    with pytest.raises(RuntimeError):
        rt.build_hashmap(b(c["stream"]), max_rounds=3)
    with pytest.raises(TypeError):
        rt.resource_hashmap("text", b"1234")


@pytest.mark.gpu
def test_gpu_reference_resources(rv):
    for r in rv["resources"]:
        hm, col = rt.resource_hashmap(b(r["stream"]), b(r["random_hash"]), sdu=r["sdu"])
        assert hm.hex() == r["hashmap"] and col is None, r["size"]
    st = b(rv["resources"][2]["stream"])
    rh = b(rv["resources"][2]["random_hash"])
    assert rt.get_map_hash(st[:464], rh) == ctoken.sha256(st[:464] + rh)[:4]
    assert rt.get_map_hash(b"", rh) == ctoken.sha256(rh)[:4]


@pytest.mark.gpu
def test_gpu_collision_guard(rv):
    for c in rv["collisions"]:
        hm, col = rt.resource_hashmap(b(c["stream"]), b(c["random_hash"]))
        assert hm.hex() == c["map_hashes"] and col == c["first_collision"], c["dup"]


@pytest.mark.gpu
def test_gpu_many_resources_one_launch():
    """Parts of 300 resources of ragged sizes (unaligned offsets, last parts
    short, one empty-salt resource) in one launch, vs the oracle; a repeated
    part planted in two resources is found per resource."""
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(506))
    sizes = rng.integers(1, 20000, 300)
    sizes[7] = 464 * 5
    streams = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in sizes]
    s11 = bytearray(rng.integers(0, 256, 464 * 12, dtype=np.uint8).tobytes())
    s11[464 * 9:464 * 10] = s11[464 * 2:464 * 3]
    streams[11] = bytes(s11)
    salts = rng.integers(0, 256, (300, 4), dtype=np.uint8)
    buf, off, ln, res = bytearray(), [], [], []
    for r, st in enumerate(streams):
        base = len(buf) + int(rng.integers(0, 7))
        buf += bytes(base - len(buf)) + st
        for j in range(-(-len(st) // 464)):
            off.append(base + 464 * j)
            ln.append(min(464, len(st) - 464 * j))
            res.append(r)
    n = len(off)
    d = torch.frombuffer(bytearray(buf), dtype=torch.uint8).cuda()
    out = torch.zeros(4 * n, dtype=torch.uint8, device="cuda")
    fc = torch.zeros(300, dtype=torch.int32, device="cuda")
    device.map_hashes(d, out, torch.from_numpy(salts).cuda(), torch.tensor(off, dtype=torch.int64).cuda(),
                      torch.tensor(ln, dtype=torch.int32).cuda(), torch.tensor(res, dtype=torch.int32).cuda(),
                      guard=224, first_collision=fc)
    got = out.cpu().numpy().tobytes()
    exp = b"".join(ctoken.map_hashes(st, salts[r].tobytes(), 464) for r, st in enumerate(streams))
    assert got == exp
    fch = fc.cpu().numpy()                    # global part index of the first collision, -1 if none
    start = np.searchsorted(np.array(res), np.arange(300))
    for r, st in enumerate(streams):
        col = ctoken.first_collision(ctoken.map_hashes(st, salts[r].tobytes(), 464), 224)
        assert fch[r] == (-1 if col is None else start[r] + col), r
    assert fch[11] == start[11] + 9
