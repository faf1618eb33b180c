"""HKDF-SHA256 on the GPU: drop-in for ``RNS.Cryptography.hkdf``
(RNS/Cryptography/HKDF.py:35-62) plus the batched per-packet keying that
Identity.encrypt / __decrypt perform (Identity.py:837-846: a fresh 64-byte
token key per packet, salt = the identity hash, context None).

Every derivation runs in librnstok's ``k_hkdf`` kernel (one lane per key);
there is no CPU fallback.
"""
import ctypes

import numpy as np

from . import _native
from .token import KeySet


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None and a.size else None


def _check_args(length, derive_from):
    # HKDF.py:40-44, same messages and exception class
    if length is None or length < 1:
        raise ValueError("Invalid output key length")
    if derive_from is None or (isinstance(derive_from, str) and derive_from == ""):
        raise ValueError("Cannot derive key from empty input material")


def _as_items(x, n=None, what="derive_from"):
    """bytes -> [bytes]; list of bytes kept; (n, L) uint8 array kept."""
    if x is None:
        return None
    if isinstance(x, (bytes, bytearray, memoryview)):
        return [bytes(x)] if n is None else [bytes(x)] * n
    if isinstance(x, np.ndarray):
        if x.ndim != 2 or x.dtype != np.uint8:
            raise ValueError(f"{what} array must be (n, L) uint8")
        return x
    items = list(x)
    for it in items:
        if it is None and what == "salt":
            continue
        if what == "derive_from" and (it is None or (isinstance(it, str) and it == "")):
            raise ValueError("Cannot derive key from empty input material")     # HKDF.py:43-44, per item
        if not isinstance(it, (bytes, bytearray, memoryview)):
            raise TypeError(f"{what} items must be bytes")
    return items


def _stack(items):
    """list of equal-length bytes -> (n, L) uint8 C array."""
    L = len(items[0]) if items else 0
    if L == 0:
        return np.zeros((len(items), 0), np.uint8)
    return np.frombuffer(b"".join(bytes(i) for i in items), np.uint8).reshape(len(items), L)


def _groups(ikm, salt):
    """Index groups with one (ikm_len, salt_len) each (the kernel takes uniform
    lengths per launch)."""
    n = len(ikm)
    il = [ikm.shape[1]] * n if isinstance(ikm, np.ndarray) else [len(i) for i in ikm]
    if salt is None:
        sl = [0] * n
    elif isinstance(salt, np.ndarray):
        sl = [salt.shape[1]] * n
    else:
        sl = [0 if s is None else len(s) for s in salt]
    g = {}
    for i in range(n):
        g.setdefault((il[i], sl[i]), []).append(i)
    return g


def _pick(items, idx):
    if isinstance(items, np.ndarray):
        return np.ascontiguousarray(items[idx])
    return _stack([items[i] for i in idx])


def _pick_salt(salt, idx, slen):
    if salt is None or slen == 0:
        return None
    if isinstance(salt, np.ndarray):
        return np.ascontiguousarray(salt[idx])
    return _stack([salt[i] for i in idx])


def _context_bytes(context):
    if context is None:
        return b""
    if not isinstance(context, (bytes, bytearray, memoryview)):
        # the reference concatenates bytes + context (HKDF.py:57)
        raise TypeError(f"can't concat {type(context).__name__} to bytes")
    return bytes(context)


def hkdf_batch(length, derive_from, salt=None, context=None, device=None):
    """n derivations at once: ``derive_from`` is a list of bytes or an (n, L)
    uint8 array, ``salt`` None, one bytes for all, a list (items may be None)
    or an (n, S) array; ``context`` one bytes object shared by all.  Returns
    an (n, length) uint8 array whose row i is
    ``RNS.Cryptography.hkdf(length, derive_from[i], salt[i], context)``."""
    _check_args(length, derive_from)
    ikm = _as_items(derive_from)
    n = len(ikm)
    sal = _as_items(salt, n, "salt")
    if sal is not None and len(sal) != n:
        raise ValueError("need one salt per item")
    ctxb = _context_bytes(context)
    out = np.zeros((n, length), np.uint8)
    if n == 0:
        return out
    lib = _native.load()
    ctx = _native.context(device)
    cbuf = np.frombuffer(ctxb, np.uint8) if ctxb else None
    for (ilen, slen), idx in _groups(ikm, sal).items():
        a = _pick(ikm, idx)
        s = _pick_salt(sal, idx, slen)
        o = np.zeros((len(idx), length), np.uint8)
        _native.check(lib.rt_hkdf_host(ctx, _ptr(a), ilen, ilen, _ptr(s), slen, slen if s is not None else 0,
                                       _ptr(cbuf), len(ctxb), _ptr(o), length, length, len(idx)))
        out[idx] = o
    return out


def hkdf(length=None, derive_from=None, salt=None, context=None, device=None):
    """Same signature, result and errors as RNS.Cryptography.hkdf
    (HKDF.py:35-62), computed by the k_hkdf kernel."""
    _check_args(length, derive_from)
    if not isinstance(derive_from, (bytes, bytearray, memoryview)):
        raise TypeError("derive_from must be bytes")
    if salt is not None and not isinstance(salt, (bytes, bytearray, memoryview)):
        raise TypeError("salt must be bytes")
    return hkdf_batch(length, [bytes(derive_from)], None if salt is None else [bytes(salt)], context,
                      device)[0].tobytes()


def derive_keyset(derive_from, salt=None, context=None, key_len=64, device=None):
    """Per-packet keying (Identity.py:837-846): a :class:`KeySet` whose key i
    is ``Token(hkdf(key_len, derive_from[i], salt[i], context))``.  The
    derived keys are produced and expanded on the device and never copied
    back.  Items must share the ikm length and the salt length."""
    if key_len not in (32, 64):
        raise ValueError("Token key must be 128 or 256 bits, not " + str(key_len * 8))
    _check_args(key_len, derive_from)
    ikm = _as_items(derive_from)
    n = len(ikm)
    sal = _as_items(salt, n, "salt")
    groups = _groups(ikm, sal)
    if len(groups) != 1:
        raise ValueError("derive_keyset needs equal-length ikm and salt items")
    (ilen, slen), = groups.keys()
    a = _pick(ikm, list(range(n)))
    s = _pick_salt(sal, list(range(n)), slen)
    ctxb = _context_bytes(context)
    lib = _native.load()
    ctx = _native.context(device)
    bufs = []
    try:
        def up(arr):
            if arr is None or arr.size == 0:
                return None
            d = lib.rt_device_alloc(ctx, arr.nbytes)
            if not d:
                raise _native.NativeError(_native.RT_E_NOMEM, _native.last_error())
            bufs.append(d)
            _native.check(lib.rt_memcpy_h2d(ctx, d, _ptr(arr), arr.nbytes, None))
            return d
        d_ikm = up(a)
        d_salt = up(s)
        d_ctx = up(np.frombuffer(ctxb, np.uint8) if ctxb else None)
        h = lib.rt_keyset_create_hkdf(ctx, d_ikm, ilen, ilen, d_salt, slen, slen if s is not None else 0,
                                      d_ctx, len(ctxb), key_len, n, None)
        if not h:
            raise _native.NativeError(-1, _native.last_error())
        _native.check(lib.rt_stream_sync(ctx, None))
    finally:
        for d in bufs:
            lib.rt_device_free(ctx, d)
    return KeySet._adopt(h, key_len, n, lib, ctx)
