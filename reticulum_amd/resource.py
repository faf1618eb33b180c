"""Resource hashmap on the GPU (RNS/Resource.py:426-468, 505-506).

A Resource's encrypted stream is cut into SDU-sized parts; each part is
advertised by ``SHA-256(part || random_hash)[:4]`` and the sender draws a new
random_hash while any map hash repeats one of the previous
COLLISION_GUARD_SIZE map hashes.  ``build_hashmap`` is that loop with the
map hashes and the collision scan computed by librnstok's k_map_hashes /
k_map_collisions; ``get_map_hash`` is the single-part form used by the
receiver (receive_part, Resource.py:865-866).  No CPU fallback.
"""
import ctypes
import os

import numpy as np

from . import _native

SDU = 464                    # Resource.SDU = Packet.MDU for the default MTU
MAPHASH_LEN = 4              # Resource.MAPHASH_LEN
RANDOM_HASH_SIZE = 4         # Resource.RANDOM_HASH_SIZE
COLLISION_GUARD_SIZE = 224   # ResourceAdvertisement.COLLISION_GUARD_SIZE = 2*WINDOW_MAX + HASHMAP_MAX_LEN
_NONE = 0xFFFFFFFF


def _bytes(x, what):
    if not isinstance(x, (bytes, bytearray, memoryview)):
        raise TypeError(f"{what} must be bytes")
    return bytes(x)


def resource_hashmap(stream, random_hash, sdu=SDU, guard=COLLISION_GUARD_SIZE, device=None):
    """Map hashes of every part of ``stream`` and the index of the first part
    whose map hash repeats one of the previous ``guard`` ones (None if the
    hashmap would be accepted).  Returns (hashmap_bytes, first_collision)."""
    stream = _bytes(stream, "stream")
    random_hash = _bytes(random_hash, "random_hash")
    if sdu < 1:
        raise ValueError("sdu must be positive")
    parts = -(-len(stream) // sdu)
    if parts == 0:
        return b"", None
    lib = _native.load()
    ctx = _native.context(device)
    data = np.frombuffer(stream, np.uint8)
    rh = np.frombuffer(random_hash, np.uint8) if random_hash else None
    out = np.zeros(4 * parts, np.uint8)
    col = ctypes.c_uint32(_NONE)
    _native.check(lib.rt_resource_hashmap_host(ctx, data.ctypes.data_as(ctypes.c_void_p), len(stream), sdu,
                                               None if rh is None else rh.ctypes.data_as(ctypes.c_void_p),
                                               len(random_hash), guard, out.ctypes.data_as(ctypes.c_void_p),
                                               ctypes.byref(col)))
    return out.tobytes(), (None if col.value == _NONE else int(col.value))


def build_hashmap(stream, sdu=SDU, guard=COLLISION_GUARD_SIZE, random_hash=None, device=None, max_rounds=64):
    """The sender's loop (Resource.py:431-468): draw random_hash
    (Identity.get_random_hash()[:4], i.e. os.urandom-backed) until no map hash
    collides inside the guard window.  Returns (random_hash, hashmap).
    ``random_hash`` may be a callable returning the next candidate (tests)."""
    draw = random_hash if callable(random_hash) else (lambda: os.urandom(RANDOM_HASH_SIZE))
    for _ in range(max_rounds):
        rh = draw()
        hashmap, col = resource_hashmap(stream, rh, sdu, guard, device)
        if col is None:
            return rh, hashmap
    raise RuntimeError("resource hashmap kept colliding (repeated parts inside the guard window)")


def get_map_hash(data, random_hash, device=None):
    """Resource.get_map_hash (Resource.py:505-506) for one part:
    SHA-256(data || random_hash)[:4]."""
    data = _bytes(data, "data")
    random_hash = _bytes(random_hash, "random_hash")
    if data:
        return resource_hashmap(data, random_hash, sdu=len(data), guard=0, device=device)[0]
    if random_hash:      # SHA-256(b"" || rh) is the one-part hash of rh with an empty salt
        return resource_hashmap(random_hash, b"", sdu=len(random_hash), guard=0, device=device)[0]
    raise ValueError("get_map_hash of an empty part with an empty random_hash")
