"""CPU stand-in for librnstok's host-staging entry points — TEST ONLY.

Implements rt_create / rt_keyset_* / rt_encrypt_host / rt_decrypt_host with
the C oracle so the Python host layer (reticulum_amd.token: argument
marshalling, key split, error mapping, Packed layout) can be unit-tested in
the CPU suite.  It is installed only by tests (``install(monkeypatch)``); the
product has no path to it, and the real kernels are covered by ``-m gpu``.
"""
import ctypes

import numpy as np

from oracle import ctoken


def _arr(p, dtype, n):
    if p is None:
        return None
    if isinstance(p, bytes):                      # Token's one-packet calls pass bytes,
        return np.frombuffer(p, dtype=dtype)      # ctypes buffers and byref() scalars
    if isinstance(p, ctypes.Array):
        return np.frombuffer(p, dtype=dtype)
    if type(p).__name__ == "CArgObject":
        return np.frombuffer(p._obj, dtype=dtype)
    addr = p.value if isinstance(p, ctypes.c_void_p) else int(p)
    if not addr or n == 0:
        return np.zeros(0, dtype=dtype)
    nbytes = np.dtype(dtype).itemsize * n
    return np.frombuffer((ctypes.c_uint8 * nbytes).from_address(addr), dtype=dtype)


class FakeLib:
    def __init__(self):
        self._keysets = {}
        self._next = 1000
        self.calls = []

    def rt_last_error(self):
        return b""

    def rt_device_count(self):
        return 1

    def rt_create(self, device):
        return 1

    def rt_keyset_create(self, ctx, keys, klen, n):
        if klen not in (32, 64):
            return None
        self._next += 1
        self._keysets[self._next] = _arr(keys, np.uint8, klen * n).copy().reshape(n, klen)
        return self._next

    def rt_keyset_destroy(self, h):
        self._keysets.pop(h, None)

    def rt_encrypt_host(self, ks, pt, pt_off, pt_len, key_idx, iv, tok, tok_off, n):
        self.calls.append(("encrypt", n))
        keys = self._keysets[ks]
        po, pl, to = _arr(pt_off, np.uint64, n), _arr(pt_len, np.uint32, n), _arr(tok_off, np.uint64, n)
        ki = _arr(key_idx, np.uint32, n)
        ivs = _arr(iv, np.uint8, 16 * n)
        pext = int(max((po + pl).max(), 1))
        text = int(max(to + 16 + 16 * (pl // 16 + 1) + 32))
        pbuf, tbuf = _arr(pt, np.uint8, pext), _arr(tok, np.uint8, text)
        for i in range(n):
            k = keys[ki[i] if ki is not None else 0].tobytes()
            t = ctoken.encrypt(k, ivs[16 * i:16 * i + 16].tobytes(), pbuf[po[i]:po[i] + pl[i]].tobytes())
            tbuf[to[i]:to[i] + len(t)] = np.frombuffer(t, np.uint8)
        return 0

    def rt_decrypt_host(self, ks, tok, tok_off, tok_len, key_idx, pt, pt_off, pt_len, status, n):
        self.calls.append(("decrypt", n))
        keys = self._keysets[ks]
        to, tl, po = _arr(tok_off, np.uint64, n), _arr(tok_len, np.uint32, n), _arr(pt_off, np.uint64, n)
        ki = _arr(key_idx, np.uint32, n)
        text = int(max((to + tl).max(), 1))
        cap = np.where(tl > 48, tl.astype(np.int64) - 48, 0)
        pext = int(max((po + cap).max(), 1))
        tbuf, pbuf = _arr(tok, np.uint8, text), _arr(pt, np.uint8, pext)
        ol, st = _arr(pt_len, np.uint32, n), _arr(status, np.int32, n)
        for i in range(n):
            k = keys[ki[i] if ki is not None else 0].tobytes()
            t = tbuf[to[i]:to[i] + tl[i]].tobytes()
            s, p = ctoken.decrypt(k, t)
            st[i] = s
            region = slice(int(po[i]), int(po[i] + cap[i]))
            if s == 0:
                pbuf[int(po[i]):int(po[i]) + len(p)] = np.frombuffer(p, np.uint8)
                ol[i] = len(p)
            else:
                ol[i] = 0
                if s == 4:          # the kernel reports the authenticated pad byte
                    raw = _raw_last_byte(k, t)
                    ol[i] = raw
                pbuf[region] = 0
        return 0

    def rt_verify_host(self, ks, tok, tok_off, tok_len, key_idx, status, n):
        """Token.verify_hmac per token: hashlib HMAC over token[:-32]."""
        import hashlib
        import hmac
        self.calls.append(("verify", n))
        keys = self._keysets[ks]
        to, tl = _arr(tok_off, np.uint64, n), _arr(tok_len, np.uint32, n)
        ki = _arr(key_idx, np.uint32, n)
        tbuf, st = _arr(tok, np.uint8, int(max((to + tl).max(), 1))), _arr(status, np.int32, n)
        for i in range(n):
            k = keys[ki[i] if ki is not None else 0].tobytes()
            t = tbuf[to[i]:to[i] + tl[i]].tobytes()
            if len(t) <= 32:
                st[i] = 1
            else:
                st[i] = 0 if hmac.new(k[:len(k) // 2], t[:-32], hashlib.sha256).digest() == t[-32:] else 2
        return 0

    def rt_verify_trials_host(self, ks, tok, tok_off, tok_len, pair_off, pair_key, first, n_tok, n_pairs):
        """first[t] = rank of the first candidate key that opens token t
        (oracle status OK or BAD_PAD: tag verified over a well-formed token)."""
        self.calls.append(("rt_verify_trials_host", n_tok, n_pairs))
        keys = self._keysets[ks]
        to, tl = _arr(tok_off, np.uint64, n_tok), _arr(tok_len, np.uint32, n_tok)
        po, pk = _arr(pair_off, np.uint32, n_tok + 1), _arr(pair_key, np.uint32, n_pairs)
        tbuf = _arr(tok, np.uint8, int(max((to + tl).max(), 1)))
        out = _arr(first, np.uint32, n_tok)
        for t in range(n_tok):
            out[t] = 0xFFFFFFFF
            token = tbuf[to[t]:to[t] + tl[t]].tobytes()
            for r, j in enumerate(range(int(po[t]), int(po[t + 1]))):
                if ctoken.decrypt(keys[pk[j]].tobytes(), token)[0] in (0, 4):
                    out[t] = r
                    break
        return 0

    def rt_resource_hashmap_host(self, ctx, data, size, sdu, rh, rh_len, guard, hashmap, first_collision):
        self.calls.append(("rt_resource_hashmap_host", size, sdu, guard))
        stream = _arr(data, np.uint8, size).tobytes()
        salt = _arr(rh, np.uint8, rh_len).tobytes() if rh_len else b""
        hm = ctoken.map_hashes(stream, salt, sdu)
        _arr(hashmap, np.uint8, len(hm))[:] = np.frombuffer(hm, np.uint8)
        col = ctoken.first_collision(hm, guard) if guard else None
        first_collision._obj.value = 0xFFFFFFFF if col is None else col
        return 0

    def rt_hkdf_host(self, ctx, ikm, ikm_stride, ikm_len, salt, salt_stride, salt_len, context, context_len, out,
                     out_stride, length, n):
        self.calls.append(("rt_hkdf_host", ikm_len, salt_len, n))
        if length < 1:
            return -1
        a = _arr(ikm, np.uint8, ikm_stride * (n - 1) + ikm_len) if ikm_len else None
        s = _arr(salt, np.uint8, salt_stride * (n - 1) + salt_len) if salt_len and salt else None
        c = _arr(context, np.uint8, context_len).tobytes() if context_len else None
        o = _arr(out, np.uint8, out_stride * (n - 1) + length)
        for i in range(n):
            k = a[i * ikm_stride:i * ikm_stride + ikm_len].tobytes() if ikm_len else b""
            sl = s[i * salt_stride:i * salt_stride + salt_len].tobytes() if s is not None else None
            o[i * out_stride:i * out_stride + length] = np.frombuffer(ctoken.hkdf(length, k, sl, c), np.uint8)
        return 0


def _raw_last_byte(key, tok):
    """Last byte of the CBC-decrypted body (for BAD_PAD detail)."""
    ek = key[len(key) // 2:]
    last_ct, prev = tok[-48:-32], tok[-64:-48]
    blk = ctoken.lib()
    out = ctypes.create_string_buffer(16)
    blk.oracle_aes_decrypt_block(ctypes.create_string_buffer(ek, len(ek)), len(ek),
                                 ctypes.create_string_buffer(last_ct, 16), out)
    return out.raw[15] ^ prev[15]


def install(monkeypatch):
    from reticulum_amd import _native
    fake = FakeLib()
    monkeypatch.setattr(_native, "_lib", fake)
    monkeypatch.setattr(_native, "_contexts", {})
    return fake
