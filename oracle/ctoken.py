"""ctypes wrapper over oracle/liboracle_token.so — TEST INFRASTRUCTURE ONLY.

See oracle/token_oracle.c for the reference file:line each function restates.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle_token.so")
_lib = None

_u8p = ctypes.POINTER(ctypes.c_uint8)


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp = ctypes.c_void_p
        L.oracle_token_encrypt.restype = ctypes.c_int64
        L.oracle_token_encrypt.argtypes = [vp, ctypes.c_uint32, vp, vp, ctypes.c_uint32, vp]
        L.oracle_token_decrypt.restype = ctypes.c_int
        L.oracle_token_decrypt.argtypes = [vp, ctypes.c_uint32, vp, ctypes.c_uint64, vp, ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_encrypt_batch.restype = ctypes.c_int
        L.oracle_encrypt_batch.argtypes = [vp, ctypes.c_uint32, vp, vp, vp, vp, vp, vp, vp, ctypes.c_uint64, ctypes.c_int]
        L.oracle_decrypt_batch.restype = ctypes.c_int
        L.oracle_decrypt_batch.argtypes = [vp, ctypes.c_uint32, vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_uint64, ctypes.c_int]
        L.oracle_sha256.argtypes = [vp, ctypes.c_uint64, vp]
        L.oracle_hmac_sha256.argtypes = [vp, ctypes.c_uint32, vp, ctypes.c_uint64, vp]
        L.oracle_aes_encrypt_block.argtypes = [vp, ctypes.c_uint32, vp, vp]
        L.oracle_aes_decrypt_block.argtypes = [vp, ctypes.c_uint32, vp, vp]
        L.oracle_sbox.argtypes = [vp]
        L.oracle_hkdf.argtypes = [vp, ctypes.c_uint64, vp, ctypes.c_uint32, vp, ctypes.c_uint32, ctypes.c_uint64, vp]
        _lib = L
    return _lib


def _buf(b):
    return ctypes.create_string_buffer(bytes(b), max(len(b), 1))


def token_len(pt_len):
    return 16 + 16 * (pt_len // 16 + 1) + 32


def encrypt(key, iv, pt):
    out = ctypes.create_string_buffer(token_len(len(pt)))
    n = lib().oracle_token_encrypt(_buf(key), len(key), _buf(iv), _buf(pt), len(pt), out)
    if n < 0:
        raise ValueError("bad key")
    return out.raw[:n]


def decrypt(key, tok):
    """Returns (status, plaintext_or_None)."""
    out = ctypes.create_string_buffer(max(len(tok), 1))
    pl = ctypes.c_uint64(0)
    st = lib().oracle_token_decrypt(_buf(key), len(key), _buf(tok), len(tok), out, ctypes.byref(pl))
    return st, (out.raw[:pl.value] if st == 0 else None)


def sha256(msg):
    out = ctypes.create_string_buffer(32)
    lib().oracle_sha256(_buf(msg), len(msg), out)
    return out.raw


def hmac_sha256(key, msg):
    out = ctypes.create_string_buffer(32)
    lib().oracle_hmac_sha256(_buf(key), len(key), _buf(msg), len(msg), out)
    return out.raw


def aes_encrypt_block(key, blk):
    out = ctypes.create_string_buffer(16)
    lib().oracle_aes_encrypt_block(_buf(key), len(key), _buf(blk), out)
    return out.raw


def sbox():
    out = ctypes.create_string_buffer(256)
    lib().oracle_sbox(out)
    return out.raw


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def encrypt_batch(keys, pt, pt_off, pt_len, key_idx, iv, tok, tok_off, threads=1):
    """Batch encrypt over host numpy arrays (same meaning as rt_encrypt)."""
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    klen = keys.shape[1]
    rc = lib().oracle_encrypt_batch(_p(keys), klen, _p(pt), _p(pt_off), _p(pt_len), _p(key_idx), _p(iv),
                                    _p(tok), _p(tok_off), len(pt_off), threads)
    if rc:
        raise ValueError("oracle_encrypt_batch rc=%d" % rc)


def decrypt_batch(keys, tok, tok_off, tok_len, key_idx, pt, pt_off, pt_len, status, threads=1):
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    klen = keys.shape[1]
    rc = lib().oracle_decrypt_batch(_p(keys), klen, _p(tok), _p(tok_off), _p(tok_len), _p(key_idx), _p(pt),
                                    _p(pt_off), _p(pt_len), _p(status), len(tok_off), threads)
    if rc:
        raise ValueError("oracle_decrypt_batch rc=%d" % rc)


def hkdf(length, derive_from, salt=None, context=None):
    """RNS/Cryptography/HKDF.py:35-62 (argument checks :40-44 included)."""
    if length is None or length < 1:
        raise ValueError("Invalid output key length")
    if derive_from is None or derive_from == "":
        raise ValueError("Cannot derive key from empty input material")
    out = ctypes.create_string_buffer(length)
    lib().oracle_hkdf(_buf(derive_from), len(derive_from), None if salt is None else _buf(salt),
                      0 if salt is None else len(salt), None if context is None else _buf(context),
                      0 if context is None else len(context), length, out)
    return out.raw


def map_hashes(stream, random_hash, sdu):
    """Resource map hashes, RNS/Resource.py:505-506 (get_map_hash) over the
    sender's segmentation :449-451: SHA-256(part || random_hash)[:4] each."""
    n = -(-len(stream) // sdu)
    return b"".join(sha256(stream[i * sdu:(i + 1) * sdu] + random_hash)[:4] for i in range(n))


def first_collision(hashes, guard):
    """Index where the hashmap loop of RNS/Resource.py:446-462 breaks: the
    first map hash equal to one of the previous `guard` map hashes; None if
    the hashmap is accepted."""
    window = []
    for i in range(len(hashes) // 4):
        mh = hashes[4 * i:4 * i + 4]
        if mh in window:
            return i
        window.append(mh)
        if len(window) > guard:
            window.pop(0)
    return None
