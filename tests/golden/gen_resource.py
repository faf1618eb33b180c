"""Generate tests/golden/resource_vectors.json from the reference Resource.

Runs only in the build container (imports /root/reference).  Two kinds of
fixture for the Resource hashmap row (RNS/Resource.py:426-468, 505-506):

* real constructions: RNS.Resource(data, link, advertise=False) with a stub
  link whose encrypt is a reference Token (Link.encrypt, Link.py:1161-1173)
  and a stand-in Packet class (only .pack() and .map_hash are touched on
  this path, :464-466).  Recorded: the encrypted stream the hashmap is
  computed over, the resource's random_hash, sdu, and its hashmap.
* collision-guard cases: the reference's get_map_hash (:505-506) over
  streams with repeated parts, and the index where the reference loop
  (:446-462, guard list of COLLISION_GUARD_SIZE entries) breaks to re-roll.
  Identical parts collide under every random_hash, so these cannot go
  through Resource() itself (it would re-roll forever); the loop is run here
  verbatim over the reference's own get_map_hash.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_resource.py
"""
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))          # tests/ (tests_helpers)
REF = os.environ.get("RNS_REFERENCE", "/root/reference")


def main():
    sys.path.insert(0, REF)
    import RNS
    from RNS.Cryptography.Token import Token

    rng = np.random.Generator(np.random.PCG64(449))
    key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    tok = Token(key)

    class StubLink:
        mtu = None
        mdu = None
        rtt = 0.5
        traffic_timeout_factor = 6
        link_id = bytes(16)

        def __init__(self):
            self.streams = []

        def encrypt(self, plaintext):
            ct = tok.encrypt(plaintext)
            self.streams.append(ct)
            return ct

    class StubPacket:
        RESOURCE = RNS.Packet.RESOURCE

        def __init__(self, link, data, context=None):
            self.data = data

        def pack(self):
            pass

    real_packet = RNS.Packet
    out = {"reference": "RNS/Resource.py:426-468,505-506", "generator": "tests/golden/gen_resource.py",
           "sdu_default": RNS.Resource.SDU, "maphash_len": RNS.Resource.MAPHASH_LEN,
           "random_hash_size": RNS.Resource.RANDOM_HASH_SIZE,
           "collision_guard_size": RNS.ResourceAdvertisement.COLLISION_GUARD_SIZE,
           "resources": [], "collisions": []}
    RNS.Packet = StubPacket
    try:
        for size in (1, 200, 431, 1000, 5000, 12000):
            link = StubLink()
            data = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
            res = RNS.Resource(data, link, advertise=False, auto_compress=False)
            stream = link.streams[-1]
            assert len(res.hashmap) == 4 * len(res.parts)
            out["resources"].append({"size": size, "sdu": res.sdu, "stream": stream.hex(),
                                     "random_hash": res.random_hash.hex(), "hashmap": res.hashmap.hex()})
    finally:
        RNS.Packet = real_packet

    # collision guard: the reference loop over the reference's get_map_hash
    guard = RNS.ResourceAdvertisement.COLLISION_GUARD_SIZE
    sdu = RNS.Resource.SDU

    def ref_loop(stream, random_hash):
        stub = types.SimpleNamespace(random_hash=random_hash)
        parts = -(-len(stream) // sdu)
        hashmap, guard_list = b"", []
        for i in range(parts):
            mh = RNS.Resource.get_map_hash(stub, stream[i * sdu:(i + 1) * sdu])
            if mh in guard_list:
                return hashmap, i
            guard_list.append(mh)
            if len(guard_list) > guard:
                guard_list.pop(0)
            hashmap += mh
        return hashmap, None

    # The streams are inputs we make, so they are stored as (seed, length,
    # dup) and rebuilt by tests_helpers.collision_stream; the reference's
    # outputs (map hashes, the break index) are stored in full.
    from tests_helpers import collision_stream
    for k, (n_parts, dup) in enumerate(((40, (5, 30)), (400, (10, 10 + guard)), (400, (10, 11 + guard)),
                                        (300, (299, 299)), (300, None))):
        seed = 4490 + k
        stream = collision_stream(seed, n_parts * sdu - 17, dup, sdu)
        rh = rng.integers(0, 256, 4, dtype=np.uint8).tobytes()
        hm, col = ref_loop(bytes(stream), rh)
        full = b"".join(RNS.Resource.get_map_hash(types.SimpleNamespace(random_hash=rh), bytes(stream[i * sdu:(i + 1) * sdu]))
                        for i in range(-(-len(stream) // sdu)))
        out["collisions"].append({"n_parts": n_parts, "dup": dup, "seed": seed, "stream_len": len(stream),
                                  "random_hash": rh.hex(), "first_collision": col,
                                  "hashmap_until_break": hm.hex(), "map_hashes": full.hex()})

    path = os.path.join(HERE, "resource_vectors.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
