"""Generate the committed golden fixtures from the reference implementation.

Runs ONLY in the build container, where the reference checkout exists at
/root/reference (markqvist/Reticulum 1.4.2).  It imports the reference's own
RNS.Cryptography and records (key, iv, plaintext, token) and negative decrypt
cases as JSON under tests/golden/.  Nothing here travels to the GPU box except
the JSON data it writes.

Deterministic IVs: Token.encrypt draws its IV from the module-global
``os.urandom`` (RNS/Cryptography/Token.py:31,89); the module object is fetched
through sys.modules because the package attribute ``RNS.Cryptography.Token`` is
shadowed by the class (RNS/Cryptography/__init__.py:38).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py
"""
import ast
import hashlib
import json
import os
import sys

import numpy as np

REF = os.environ.get("RETICULUM_REF", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))

LENGTHS = [0, 1, 15, 16, 17, 31, 32, 63, 64, 100, 383, 431, 464, 499, 500, 501, 1024, 4095, 4096, 16384]


def load_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import RNS  # noqa: F401  (imports modules only; starts no instance)
    import RNS.Cryptography
    tokmod = sys.modules["RNS.Cryptography.Token"]
    return RNS, tokmod


class FixedUrandom:
    """Stand-in for os.urandom inside the reference Token module only."""

    def __init__(self, real):
        self.real = real
        self.queue = []

    def push(self, b):
        self.queue.append(b)

    def __getattr__(self, name):
        return getattr(self.real, name)

    def urandom(self, n):
        if self.queue:
            b = self.queue.pop(0)
            assert len(b) == n
            return b
        return self.real.urandom(n)


def ref_decrypt(Token, key, tok):
    """Run the reference decrypt; return (status, plaintext_hex, exc_class, message)."""
    try:
        pt = Token(key).decrypt(tok)
        return 0, pt.hex(), None, None
    except Exception as e:  # record class and message exactly
        msg = str(e)
        if "Cannot verify HMAC" in msg:
            st = 1
        elif "HMAC was invalid" in msg:
            st = 2
        elif "invalid padding length" in msg:
            st = 4
        elif "Could not decrypt token" in msg:
            st = 3
        else:
            st = -1
        return st, None, type(e).__name__, msg


def main():
    RNS, tokmod = load_reference()
    Token = tokmod.Token
    fake = FixedUrandom(os)
    tokmod.os = fake
    from RNS.Cryptography import HMAC as RHMAC

    rng = np.random.Generator(np.random.PCG64(20261015))
    out = {"reference": "markqvist/Reticulum " + RNS._version.__version__ if hasattr(RNS, "_version") else "markqvist/Reticulum",
           "backend": RNS.Cryptography.backend(),
           "generator": "tests/golden/gen_golden.py", "encrypt": [], "decrypt": [], "kat": {}}

    keys64 = [rng.integers(0, 256, 64, dtype=np.uint8).tobytes() for _ in range(8)]
    keys32 = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(2)]

    # Positive encrypt vectors: every length x several keys (AES-256), AES-128 on a subset.
    for ki, key in enumerate(keys64 + keys32):
        lens = LENGTHS if ki < 3 or ki >= 8 else [0, 17, 500, 4095]
        for L in lens:
            if len(key) == 32 and L > 4096:
                continue
            pt = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
            iv = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
            fake.push(iv)
            tok = Token(key).encrypt(pt)
            back = Token(key).decrypt(tok)
            assert back == pt
            out["encrypt"].append({"key": key.hex(), "iv": iv.hex(), "pt": pt.hex(), "token": tok.hex()})

    # Negative / edge decrypt vectors.  Tokens with a *valid* tag but malformed
    # body are forged with the signing key, exactly as a key holder could.
    key = keys64[0]
    sk = key[:32]

    def sign(body):
        return body + RHMAC.new(sk, body).digest()

    fake.push(bytes(16))
    good = Token(key).encrypt(b"reticulum golden vector")
    iv = os.urandom(16)
    cases = []
    cases.append(("empty", b""))
    cases.append(("len1", b"\x01"))
    cases.append(("len32", bytes(32)))
    cases.append(("len33_badtag", bytes(33)))
    cases.append(("len47_badtag", bytes(range(47))))
    cases.append(("len40_validtag", sign(bytes(range(8)))))          # iv shorter than 16
    cases.append(("len48_validtag_empty_ct", sign(iv)))              # empty ct
    cases.append(("ct_not_mult16_validtag", sign(iv + bytes(20))))
    cases.append(("flipped_tag", good[:-1] + bytes([good[-1] ^ 1])))
    cases.append(("flipped_ct", good[:20] + bytes([good[20] ^ 0x80]) + good[21:]))
    cases.append(("flipped_iv", bytes([good[0] ^ 1]) + good[1:]))
    cases.append(("truncated", good[:-16]))
    cases.append(("good", good))
    # Valid tag, chosen last plaintext byte: build ct by encrypting a chosen
    # padded block with the reference AES, then sign.
    from RNS.Cryptography.AES import AES_256_CBC
    ek = key[32:]
    for last in (0, 1, 16, 17, 0xFF):
        blk = bytes(rng.integers(0, 256, 31, dtype=np.uint8).tobytes()) + bytes([last])
        ct = AES_256_CBC.encrypt(blk, ek, iv)
        cases.append((f"pad_last_{last}", sign(iv + ct)))
    # inconsistent pad bytes but last byte in range -> accepted (lenient unpad)
    blk = bytes(range(14)) + bytes([7, 2])
    cases.append(("pad_inconsistent", sign(iv + AES_256_CBC.encrypt(blk, ek, iv))))

    for name, tok in cases:
        st, pt_hex, exc, msg = ref_decrypt(Token, key, tok)
        out["decrypt"].append({"name": name, "key": key.hex(), "token": tok.hex(), "status": st,
                               "pt": pt_hex, "exc": exc, "msg": msg})
    # type errors on the single-item surface (Token.py:88,101)
    for meth, arg in (("encrypt", bytearray(b"x")), ("decrypt", bytearray(64)), ("encrypt", "str")):
        try:
            getattr(Token(key), meth)(arg)
            raise AssertionError("expected TypeError")
        except TypeError as e:
            out["kat"].setdefault("type_errors", []).append({"method": meth, "arg_type": type(arg).__name__, "msg": str(e)})
    for bad in (None, bytes(16), bytes(48), bytes(65)):
        try:
            Token(bad)
            raise AssertionError("expected error")
        except (ValueError, TypeError) as e:
            out["kat"].setdefault("key_errors", []).append(
                {"key_len": None if bad is None else len(bad), "exc": type(e).__name__, "msg": str(e)})

    # Reference KAT (tests/identity.py:11-19,148-158): the fixed identity
    # decrypts fixed_token.  Capture the HKDF-derived 64-B token key the
    # reference computes on the way (Identity.py:837-846).
    ti = {}
    src = open(os.path.join(REF, "tests", "identity.py")).read()
    ns = {}
    for line in src.splitlines():
        s = line.strip()
        if s.startswith("encrypted_message =") or s.startswith("fixed_token ="):
            name, rhs = s.split("=", 1)            # a literal only: never executed
            ns[name.strip()] = ast.literal_eval(rhs.strip())
    fixed_key0 = src.split('fixed_keys = [')[1].split('("')[1].split('"')[0]
    captured = []
    orig_init = Token.__init__

    def spy(self, key=None, mode=tokmod.AES):
        captured.append(bytes(key))
        return orig_init(self, key, mode)

    Token.__init__ = spy
    try:
        fid = RNS.Identity.from_bytes(bytes.fromhex(fixed_key0))
        pt = fid.decrypt(bytes.fromhex(ns["fixed_token"]))
    finally:
        Token.__init__ = orig_init
    assert pt == bytes.fromhex(ns["encrypted_message"])
    ftok = bytes.fromhex(ns["fixed_token"])[32:]   # strip 32 B ephemeral pub (Identity.py:831)
    ti = {"source": "tests/identity.py:11-19,148-158", "derived_key": captured[-1].hex(),
          "token": ftok.hex(), "pt": ns["encrypted_message"]}
    out["kat"]["fixed_token"] = ti

    # SHA-256 / HMAC KATs used by the token MAC (tests/hashes.py:12-30 vectors).
    out["kat"]["sha256"] = [
        {"msg": "", "digest": hashlib.sha256(b"").hexdigest()},
        {"msg": b"abc".hex(), "digest": hashlib.sha256(b"abc").hexdigest()},
        {"msg": (b"a" * 64).hex(), "digest": hashlib.sha256(b"a" * 64).hexdigest()},
        {"msg_repeat": ["61", 1000000], "digest": hashlib.sha256(b"a" * 1000000).hexdigest()},
    ]
    hm = []
    for klen in (16, 32, 64, 65, 100):
        k = rng.integers(0, 256, klen, dtype=np.uint8).tobytes()
        m = rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
        hm.append({"key": k.hex(), "msg": m.hex(), "mac": RHMAC.new(k, m).digest().hex()})
    out["kat"]["hmac_sha256"] = hm

    # HKDF vectors (RNS/Cryptography/HKDF.py:35-62) for the ranked-next key-derivation row.
    from RNS.Cryptography import hkdf
    hk = []
    for i in range(4):
        ikm = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        salt = rng.integers(0, 256, 16, dtype=np.uint8).tobytes() if i % 2 == 0 else None
        hk.append({"ikm": ikm.hex(), "salt": None if salt is None else salt.hex(), "length": 64,
                   "okm": hkdf(length=64, derive_from=ikm, salt=salt, context=None).hex()})
    out["kat"]["hkdf"] = hk

    path = os.path.join(HERE, "token_vectors.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", path, os.path.getsize(path), "bytes;", len(out["encrypt"]), "encrypt,", len(out["decrypt"]), "decrypt cases")


if __name__ == "__main__":
    main()
