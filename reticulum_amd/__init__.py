"""reticulum_amd — MI355X-native engine for Reticulum's encrypted-token path.

Drop-in for ``RNS.Cryptography.Token`` (AES-256/128-CBC + PKCS7 +
HMAC-SHA256), computed by hand-written gfx950 HIP kernels in librnstok.so.

    from reticulum_amd import Token
    t = Token(Token.generate_key())
    assert t.decrypt(t.encrypt(b"hello")) == b"hello"

Batch use: ``KeySet.encrypt_batch`` / ``decrypt_batch`` over host buffers,
``reticulum_amd.device`` over device-resident (torch) buffers, and
``reticulum_amd.shard`` for one-process-per-GPU sharding.  Key derivation:
``hkdf`` (drop-in for RNS.Cryptography.hkdf), ``hkdf_batch`` and
``derive_keyset`` (Identity's per-packet keys, derived and expanded on the
device).  Resource hashmaps: ``resource_hashmap`` / ``build_hashmap`` /
``get_map_hash`` (Resource.py:426-468, 505-506).  Wire-side neighbours
(HDLC framing, IFAC masking, packet header unpack/pack): ``reticulum_amd.wire``.

``available()`` tells whether the library and a gfx950 device are usable;
``reticulum_amd.dropin`` is the import for the reference's one-line swap,
which raises ImportError when they are not.
"""
from ._native import NativeError, NativeUnavailable, LIB_PATH, available  # noqa: F401
from ._native import RT_ST_OK, RT_ST_TOO_SHORT, RT_ST_BAD_HMAC, RT_ST_BAD_CT_LEN, RT_ST_BAD_PAD  # noqa: F401
from .hkdf import derive_keyset, hkdf, hkdf_batch  # noqa: F401
from .resource import build_hashmap, get_map_hash, resource_hashmap  # noqa: F401
from . import wire  # noqa: F401
from .token import AES, AES_128_CBC, AES_256_CBC, KeySet, Packed, Token, TOKEN_OVERHEAD, token_len  # noqa: F401

__version__ = "0.1.0"
