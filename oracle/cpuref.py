"""Pure-Python restatement of the reference token path — TEST INFRASTRUCTURE.

Used as (1) a second, independent checker of the golden vectors and (2) the
"reference pure-Python CPU path" baseline timed on the GPU box, where the
reference itself may not run.  It keeps the reference's per-call *work
shape* so its speed tracks the reference's:

  * a fresh AES key schedule on every encrypt/decrypt call
    (RNS/Cryptography/AES.py:83,100 constructs AES256(key) per call);
  * byte-oriented AES rounds over a 16-byte state list
    (RNS/Cryptography/aes/aes256.py:177-213), CBC chaining per block
    (aes256.py:215-235);
  * HMAC-SHA256 through hashlib with the ipad/opad contexts rebuilt per
    call (RNS/Cryptography/HMAC.py:47-125);
  * PKCS7 pad / lenient unpad (RNS/Cryptography/PKCS7.py:35-48) and the
    Token framing and error order of RNS/Cryptography/Token.py:77-114.

Written from FIPS-197; the S-box is derived, not transcribed.
"""
import hashlib


def _xt(b):
    b <<= 1
    return (b ^ 0x11B) if b & 0x100 else b


def _gmul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a = _xt(a)
        b >>= 1
    return r


def _derive_sbox():
    sbox = [0] * 256
    for x in range(256):
        inv = 0
        if x:
            for y in range(1, 256):
                if _gmul(x, y) == 1:
                    inv = y
                    break
        s = inv
        for k in range(1, 5):
            s ^= ((inv << k) | (inv >> (8 - k))) & 0xFF
        sbox[x] = s ^ 0x63
    inv_sbox = [0] * 256
    for i, s in enumerate(sbox):
        inv_sbox[s] = i
    return sbox, inv_sbox


SBOX, INV_SBOX = _derive_sbox()
M2 = [_gmul(i, 2) for i in range(256)]
M3 = [_gmul(i, 3) for i in range(256)]
M9 = [_gmul(i, 9) for i in range(256)]
M11 = [_gmul(i, 11) for i in range(256)]
M13 = [_gmul(i, 13) for i in range(256)]
M14 = [_gmul(i, 14) for i in range(256)]


def key_schedule(key):
    """FIPS-197 §5.2; returns a list of Nr+1 round keys of 16 ints."""
    nk = len(key) // 4
    nr = nk + 6
    words = [list(key[4 * i:4 * i + 4]) for i in range(nk)]
    rcon = 1
    while len(words) < 4 * (nr + 1):
        t = list(words[-1])
        i = len(words)
        if i % nk == 0:
            t = [SBOX[t[1]] ^ rcon, SBOX[t[2]], SBOX[t[3]], SBOX[t[0]]]
            rcon = _xt(rcon)
        elif nk > 6 and i % nk == 4:
            t = [SBOX[b] for b in t]
        words.append([a ^ b for a, b in zip(words[i - nk], t)])
    return [sum(words[4 * r:4 * r + 4], []) for r in range(nr + 1)]


def _enc_block(st, rks):
    # state index = 4*col + row
    s = [a ^ b for a, b in zip(st, rks[0])]
    nr = len(rks) - 1
    for r in range(1, nr + 1):
        t = [SBOX[s[(4 * (c + row) + row) % 16]] for c in range(4) for row in range(4)]
        if r < nr:
            m = []
            for c in range(4):
                a0, a1, a2, a3 = t[4 * c:4 * c + 4]
                m += [M2[a0] ^ M3[a1] ^ a2 ^ a3, a0 ^ M2[a1] ^ M3[a2] ^ a3,
                      a0 ^ a1 ^ M2[a2] ^ M3[a3], M3[a0] ^ a1 ^ a2 ^ M2[a3]]
            t = m
        k = rks[r]
        s = [t[i] ^ k[i] for i in range(16)]
    return s


def _dec_block(st, rks):
    nr = len(rks) - 1
    s = [a ^ b for a, b in zip(st, rks[nr])]
    for r in range(nr - 1, -1, -1):
        t = [0] * 16
        for c in range(4):
            for row in range(4):
                t[(4 * (c + row) + row) % 16] = INV_SBOX[s[4 * c + row]]
        k = rks[r]
        t = [t[i] ^ k[i] for i in range(16)]
        if r > 0:
            m = []
            for c in range(4):
                a0, a1, a2, a3 = t[4 * c:4 * c + 4]
                m += [M14[a0] ^ M11[a1] ^ M13[a2] ^ M9[a3], M9[a0] ^ M14[a1] ^ M11[a2] ^ M13[a3],
                      M13[a0] ^ M9[a1] ^ M14[a2] ^ M11[a3], M11[a0] ^ M13[a1] ^ M9[a2] ^ M14[a3]]
            t = m
        s = t
    return s


def hmac_sha256(key, msg):
    if len(key) > 64:
        key = hashlib.sha256(key).digest()
    key = key.ljust(64, b"\0")
    inner = hashlib.sha256(bytes(b ^ 0x36 for b in key))
    outer = hashlib.sha256(bytes(b ^ 0x5C for b in key))
    inner.update(msg)
    outer.update(inner.digest())
    return outer.digest()


def _split(key):
    if len(key) not in (32, 64):
        raise ValueError("Token key must be 128 or 256 bits, not " + str(len(key) * 8))
    h = len(key) // 2
    return key[:h], key[h:]


def encrypt(key, iv, pt):
    sk, ek = _split(key)
    rks = key_schedule(ek)                      # per call, like AES.py:83
    n = 16 - len(pt) % 16
    data = pt + bytes([n]) * n
    prev = list(iv)
    out = bytearray(iv)
    for i in range(0, len(data), 16):
        prev = _enc_block([a ^ b for a, b in zip(data[i:i + 16], prev)], rks)
        out += bytes(prev)
    return bytes(out) + hmac_sha256(sk, bytes(out))


def decrypt(key, tok):
    """Returns (status, plaintext or None); status as include/rnstok.h RT_ST_*."""
    sk, ek = _split(key)
    if len(tok) <= 32:
        return 1, None
    if hmac_sha256(sk, tok[:-32]) != tok[-32:]:
        return 2, None
    ct = tok[16:-32]
    if len(tok) < 48 or len(ct) == 0 or len(ct) % 16:
        return 3, None
    rks = key_schedule(ek)                      # per call, like AES.py:100
    prev = list(tok[:16])
    out = bytearray()
    for i in range(0, len(ct), 16):
        blk = list(ct[i:i + 16])
        out += bytes(a ^ b for a, b in zip(_dec_block(blk, rks), prev))
        prev = blk
    n = out[-1]
    if n > 16:
        return 4, None
    return 0, bytes(out[:len(out) - n])
