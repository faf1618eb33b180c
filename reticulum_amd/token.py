"""Drop-in ``Token`` for Reticulum's encrypted-token path, backed by HIP kernels.

Mirrors ``RNS.Cryptography.Token`` (markqvist/Reticulum 1.4.2,
RNS/Cryptography/Token.py:40-114): same constructor, key split, methods,
constants, exception classes and messages.  The per-item calls run the same
gfx950 kernels as the batch calls (a batch of one, through the host-staging
entry points of librnstok); ``encrypt_batch`` / ``decrypt_batch`` take many
packets per call, and ``reticulum_amd.device`` drives device-resident
buffers.  There is no CPU fallback: without librnstok.so and a gfx950 device
every call raises ``NativeUnavailable``.
"""
import ctypes
import os

import numpy as np

from . import _native
from ._native import RT_ST_OK, RT_ST_TOO_SHORT, RT_ST_BAD_HMAC, RT_ST_BAD_CT_LEN, RT_ST_BAD_PAD


class _Mode:
    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return self.name


# Mode sentinels standing in for the reference's RNS.Cryptography.AES module
# and its AES_128_CBC / AES_256_CBC classes (Token.py:36-38,53-74).
AES = _Mode("AES")
AES_128_CBC = _Mode("AES_128_CBC")
AES_256_CBC = _Mode("AES_256_CBC")

TOKEN_OVERHEAD = 48

_OFF0 = ctypes.byref(ctypes.c_uint64(0))   # the offset array of a one-record call (read-only)


def token_len(pt_len):
    """len(token) for a plaintext of pt_len bytes (Token.py:96-97, PKCS7.py:35-39)."""
    return 16 + 16 * (pt_len // 16 + 1) + 32


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class Packed:
    """Variable-length records packed in one uint8 buffer: record i is
    ``buf[off[i] : off[i] + length[i]]``."""

    __slots__ = ("buf", "off", "length")

    def __init__(self, buf, off, length):
        self.buf = np.ascontiguousarray(buf, dtype=np.uint8)
        self.off = np.ascontiguousarray(off, dtype=np.uint64)
        self.length = np.ascontiguousarray(length, dtype=np.uint32)

    @classmethod
    def from_list(cls, items):
        lens = np.fromiter((len(b) for b in items), dtype=np.uint32, count=len(items))
        off = np.zeros(len(items), dtype=np.uint64)
        if len(items) > 1:
            np.cumsum(lens[:-1], out=off[1:])
        buf = np.frombuffer(b"".join(items), dtype=np.uint8) if items else np.zeros(0, np.uint8)
        return cls(buf, off, lens)

    @classmethod
    def empty_like_lengths(cls, lengths):
        lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
        off = np.zeros(len(lengths), dtype=np.uint64)
        if len(lengths) > 1:
            np.cumsum(lengths[:-1].astype(np.uint64), out=off[1:])
        total = int(lengths.astype(np.uint64).sum())
        return cls(np.zeros(max(total, 1), dtype=np.uint8), off, lengths)

    def __len__(self):
        return len(self.off)

    def __getitem__(self, i):
        o = int(self.off[i])
        return self.buf[o:o + int(self.length[i])].tobytes()

    def to_list(self):
        return [self[i] for i in range(len(self))]


class KeySet:
    """Device key table: n keys of one length (64 B AES-256 or 32 B AES-128),
    expanded on the GPU into round keys and HMAC midstates (Token.py:58-74)."""

    def __init__(self, keys, device=None):
        if isinstance(keys, (bytes, bytearray)):
            keys = [bytes(keys)]
        if isinstance(keys, (list, tuple)):
            if not keys:
                raise ValueError("KeySet needs at least one key")
            klen = len(keys[0])
            if any(len(k) != klen for k in keys):
                raise ValueError("all keys of a KeySet must have the same length")
            arr = np.frombuffer(b"".join(bytes(k) for k in keys), dtype=np.uint8).reshape(len(keys), klen)
        else:
            arr = np.ascontiguousarray(keys, dtype=np.uint8)
            if arr.ndim != 2:
                raise ValueError("keys array must be (n_keys, key_len)")
        n, klen = arr.shape
        if klen not in (32, 64):
            raise ValueError("Token key must be 128 or 256 bits, not " + str(klen * 8))
        self.key_len = klen
        self.n_keys = n
        self._lib = _native.load()
        self._ctx = _native.context(device)
        arr = np.ascontiguousarray(arr)
        self._ptr = self._lib.rt_keyset_create(self._ctx, _ptr(arr), klen, n)
        if not self._ptr:
            raise _native.NativeError(-1, _native.last_error())

    @classmethod
    def _adopt(cls, handle, key_len, n_keys, lib, ctx):
        """Wrap a keyset handle built by the library (e.g. rt_keyset_create_hkdf)."""
        ks = cls.__new__(cls)
        ks.key_len, ks.n_keys, ks._lib, ks._ctx, ks._ptr = key_len, n_keys, lib, ctx, handle
        return ks

    @property
    def handle(self):
        return self._ptr

    def __del__(self):
        p = getattr(self, "_ptr", None)
        if p:
            try:
                self._lib.rt_keyset_destroy(p)
            except Exception:
                pass
            self._ptr = None

    # ---------------------------------------------------------------- batch
    def encrypt_batch(self, plaintexts, ivs=None, key_idx=None):
        """Token.encrypt over many packets.  ``plaintexts``: list of bytes or
        :class:`Packed`; ``ivs``: (n,16) uint8 or None (fresh os.urandom,
        Token.py:89); ``key_idx``: per-packet key index or None (key 0).
        Returns a :class:`Packed` of tokens."""
        pts = plaintexts if isinstance(plaintexts, Packed) else Packed.from_list(list(plaintexts))
        n = len(pts)
        if ivs is None:
            ivs = np.frombuffer(os.urandom(16 * n), dtype=np.uint8) if n else np.zeros(0, np.uint8)
        ivs = np.ascontiguousarray(ivs, dtype=np.uint8).reshape(-1)
        if ivs.size != 16 * n:
            raise ValueError("need 16 IV bytes per packet")
        kidx = self._key_idx(key_idx, n)
        tl = (16 + 16 * (pts.length.astype(np.uint64) // 16 + 1) + 32).astype(np.uint32)
        out = Packed.empty_like_lengths(tl)
        if n:
            _native.check(self._lib.rt_encrypt_host(self._ptr, _ptr(pts.buf), _ptr(pts.off), _ptr(pts.length),
                                                    _ptr(kidx), _ptr(ivs), _ptr(out.buf), _ptr(out.off), n))
        return out

    def decrypt_batch(self, tokens, key_idx=None):
        """Token.verify_hmac + Token.decrypt over many tokens.  Returns
        ``(plaintexts: Packed, status: int32 array)``; status values are
        RT_ST_* (0 = OK) and failed packets have length 0."""
        out, status, _ = self._decrypt_raw(tokens, key_idx)
        return out, status

    def verify_batch(self, tokens, key_idx=None):
        """Token.verify_hmac over many tokens (no AES, no plaintext written):
        an int32 status array, RT_ST_OK where the tag verifies, RT_ST_BAD_HMAC
        where it does not, RT_ST_TOO_SHORT for tokens of <= 32 bytes."""
        toks = tokens if isinstance(tokens, Packed) else Packed.from_list(list(tokens))
        n = len(toks)
        kidx = self._key_idx(key_idx, n)
        status = np.zeros(n, dtype=np.int32)
        if n:
            _native.check(self._lib.rt_verify_host(self._ptr, _ptr(toks.buf), _ptr(toks.off), _ptr(toks.length),
                                                   _ptr(kidx), _ptr(status), n))
        return status

    def verify_trials(self, tokens, candidates):
        """Identity.decrypt's ratchet loop (Identity.py:865-878) over a batch:
        ``candidates[t]`` lists key indices of this key set to try on token t,
        in ratchet order.  Returns an int64 array: the first candidate key
        index whose HMAC verifies over well-formed token t, or -1."""
        toks = tokens if isinstance(tokens, Packed) else Packed.from_list(list(tokens))
        n = len(toks)
        if len(candidates) != n:
            raise ValueError("need one candidate list per token")
        counts = np.fromiter((len(c) for c in candidates), dtype=np.uint32, count=n)
        pair_off = np.zeros(n + 1, dtype=np.uint32)
        np.cumsum(counts, out=pair_off[1:])
        pair_key = np.fromiter((k for c in candidates for k in c), dtype=np.int64, count=int(pair_off[-1]))
        if pair_key.size and (pair_key.min() < 0 or pair_key.max() >= self.n_keys):
            raise ValueError("candidate key index out of range")
        pair_key = pair_key.astype(np.uint32)
        first = np.zeros(n, dtype=np.uint32)
        if n:
            _native.check(self._lib.rt_verify_trials_host(self._ptr, _ptr(toks.buf), _ptr(toks.off),
                                                          _ptr(toks.length), _ptr(pair_off), _ptr(pair_key),
                                                          _ptr(first), n, int(pair_off[-1])))
        out = np.full(n, -1, dtype=np.int64)
        hit = first != 0xFFFFFFFF
        out[hit] = pair_key[pair_off[:-1][hit].astype(np.int64) + first[hit]]
        return out

    def decrypt_trials(self, tokens, candidates):
        """verify_trials, then each opened token decrypted with its key.
        Returns ``(plaintexts: Packed, status, key_used)``: key_used is -1 and
        status RT_ST_BAD_HMAC where no candidate opens the token (the
        reference's loop ends with plaintext None, Identity.py:880-886)."""
        toks = tokens if isinstance(tokens, Packed) else Packed.from_list(list(tokens))
        key_used = self.verify_trials(toks, candidates)
        n = len(toks)
        opened = np.nonzero(key_used >= 0)[0]
        status = np.full(n, RT_ST_BAD_HMAC, dtype=np.int32)
        lengths = np.zeros(n, dtype=np.uint32)
        bufs = [b""] * n
        if opened.size:
            sub = Packed.from_list([toks[int(i)] for i in opened])
            pts, st, _ = self._decrypt_raw(sub, key_idx=key_used[opened])
            status[opened] = st
            for j, i in enumerate(opened):
                bufs[int(i)] = pts[j]
        out = Packed.from_list(bufs)
        return out, status, np.where(status == RT_ST_OK, key_used, -1)

    def _decrypt_raw(self, tokens, key_idx=None):
        toks = tokens if isinstance(tokens, Packed) else Packed.from_list(list(tokens))
        n = len(toks)
        kidx = self._key_idx(key_idx, n)
        cap = np.where(toks.length > 48, toks.length.astype(np.int64) - 48, 0).astype(np.uint32)
        out = Packed.empty_like_lengths(cap)
        status = np.zeros(n, dtype=np.int32)
        if n:
            _native.check(self._lib.rt_decrypt_host(self._ptr, _ptr(toks.buf), _ptr(toks.off), _ptr(toks.length),
                                                    _ptr(kidx), _ptr(out.buf), _ptr(out.off), _ptr(out.length),
                                                    _ptr(status), n))
        detail = out.length.copy()           # BAD_PAD reports the pad byte here
        out.length[status != RT_ST_OK] = 0
        return out, status, detail

    def _key_idx(self, key_idx, n):
        if key_idx is None:
            return None
        k = np.ascontiguousarray(key_idx, dtype=np.uint32).reshape(-1)
        if k.size != n:
            raise ValueError("need one key index per packet")
        if n and int(k.max()) >= self.n_keys:
            raise ValueError("key index out of range")
        return k


class Token:
    """Drop-in for ``RNS.Cryptography.Token`` (Token.py:40-114).

    Fernet-derived token without version/timestamp:
    ``iv(16) || AES-CBC(ek, iv, PKCS7(pt)) || HMAC-SHA256(sk, iv||ct)``.
    """

    TOKEN_OVERHEAD = TOKEN_OVERHEAD

    @staticmethod
    def generate_key(mode=AES_256_CBC):                       # Token.py:53-56
        if mode == AES_128_CBC:
            return os.urandom(32)
        elif mode == AES_256_CBC:
            return os.urandom(64)
        else:
            raise TypeError(f"Invalid token mode: {mode}")

    def __init__(self, key=None, mode=AES, device=None):       # Token.py:58-74
        if key == None:  # noqa: E711  (same test as the reference)
            raise ValueError("Token key cannot be None")
        if mode == AES:
            if len(key) == 32:
                self.mode = AES_128_CBC
                self._signing_key = key[:16]
                self._encryption_key = key[16:]
            elif len(key) == 64:
                self.mode = AES_256_CBC
                self._signing_key = key[:32]
                self._encryption_key = key[32:]
            else:
                raise ValueError("Token key must be 128 or 256 bits, not " + str(len(key) * 8))
        else:
            raise TypeError(f"Invalid token mode: {mode}")
        self._key = bytes(key)
        self._device = device
        self._keyset = None

    @property
    def keyset(self):
        if self._keyset is None:
            self._keyset = KeySet(self._key, device=self._device)
        return self._keyset

    # One packet per call, as Identity/Link call Token: the host entry points
    # with n = 1 on ctypes scalars and the caller's bytes (no Packed arrays:
    # building them cost ≈30-40 µs of Python per call).
    def _decrypt_one(self, token):
        ks = self.keyset
        L = len(token)
        out = ctypes.create_string_buffer(max(L - 48, 1))
        olen, st = ctypes.c_uint32(0), ctypes.c_int32(0)
        _native.check(ks._lib.rt_decrypt_host(ks._ptr, token, _OFF0, ctypes.byref(ctypes.c_uint32(L)), None, out,
                                              _OFF0, ctypes.byref(olen), ctypes.byref(st), 1))
        return st.value, out, olen.value

    def verify_hmac(self, token):                               # Token.py:77-84
        if len(token) <= 32:
            raise ValueError("Cannot verify HMAC on token of only " + str(len(token)) + " bytes")
        # the verify-only kernel: HMAC over token[:-32], no AES, no plaintext
        ks = self.keyset
        token = bytes(token)
        st = ctypes.c_int32(-1)
        _native.check(ks._lib.rt_verify_host(ks._ptr, token, _OFF0, ctypes.byref(ctypes.c_uint32(len(token))), None,
                                             ctypes.byref(st), 1))
        return st.value == RT_ST_OK

    def encrypt(self, data=None):                               # Token.py:87-97
        if not isinstance(data, bytes):
            raise TypeError("Token plaintext input must be bytes")
        ks = self.keyset
        n = len(data)
        out = ctypes.create_string_buffer(token_len(n))
        _native.check(ks._lib.rt_encrypt_host(ks._ptr, data, _OFF0, ctypes.byref(ctypes.c_uint32(n)), None,
                                              os.urandom(16), out, _OFF0, 1))      # fresh IV, Token.py:89
        return out.raw

    def decrypt(self, token=None):                              # Token.py:100-114
        if not isinstance(token, bytes):
            raise TypeError("Token must be bytes")
        if len(token) <= 32:
            raise ValueError("Cannot verify HMAC on token of only " + str(len(token)) + " bytes")
        st, out, n = self._decrypt_one(token)
        if st == RT_ST_OK:
            return out.raw[:n]
        raise ValueError(status_message(st, len(token), n))

    # batch extensions ---------------------------------------------------
    def encrypt_batch(self, plaintexts, ivs=None):
        return self.keyset.encrypt_batch(plaintexts, ivs=ivs)

    def decrypt_batch(self, tokens):
        return self.keyset.decrypt_batch(tokens)


def status_message(status, token_len_, detail=0):
    """The reference's exception message for a non-OK decrypt status
    (Token.py:78,102,114; PKCS7.py:44-46; aes256.py:136)."""
    if status == RT_ST_TOO_SHORT:
        return "Cannot verify HMAC on token of only " + str(token_len_) + " bytes"
    if status == RT_ST_BAD_HMAC:
        return "Token HMAC was invalid"
    if status == RT_ST_BAD_CT_LEN:
        if token_len_ <= 48:          # empty ciphertext -> PKCS7.unpad IndexError
            return "Could not decrypt token: index out of range"
        return "Could not decrypt token: "   # split_blocks assertion
    if status == RT_ST_BAD_PAD:
        return f"Could not decrypt token: Cannot unpad, invalid padding length of {detail} bytes"
    return f"Could not decrypt token: status {status}"
