"""Generate tests/golden/hkdf_vectors.json from the reference HKDF.

Runs only in the build container (it imports /root/reference, which never
travels to the GPU box).  Covers RNS/Cryptography/HKDF.py:35-62 as called by
Identity.encrypt/__decrypt (Identity.py:837-846: 64-byte key, salt = the
identity hash, context None) and Link.handshake, plus the edges of the
function itself: salt None / empty / <=64 / >64 bytes (HMAC.py:73-82 hashes
long keys), empty and long contexts (multi-block expand messages), empty and
long input material, output lengths that truncate the last block and lengths
past 255 blocks (the counter byte wraps, HKDF.py:60), and the argument
errors.  The fixed_token identity KAT's own derivation (tests/identity.py) is
captured by spying on the reference's hkdf while it decrypts.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_hkdf.py
"""
import ast
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("RNS_REFERENCE", "/root/reference")


def main():
    sys.path.insert(0, REF)
    import RNS
    import RNS.Cryptography as C
    from RNS.Cryptography import hkdf

    rng = np.random.Generator(np.random.PCG64(35))

    def rb(n):
        return rng.integers(0, 256, n, dtype=np.uint8).tobytes()

    vec = []

    def add(length, ikm, salt, context, note):
        okm = hkdf(length=length, derive_from=ikm, salt=salt, context=context)
        vec.append({"length": length, "ikm": ikm.hex(), "salt": None if salt is None else salt.hex(),
                    "context": None if context is None else context.hex(), "okm": okm.hex(), "note": note})

    for length in (1, 16, 31, 32, 33, 64, 100):
        add(length, rb(32), rb(16), None, "identity-shaped")
    for slen in (0, 1, 16, 32, 63, 64, 65, 100, 200):
        add(64, rb(32), rb(slen), None, f"salt {slen} B")
    add(64, rb(32), None, None, "salt None")
    for clen in (0, 1, 5, 22, 23, 31, 55, 56, 64, 120, 300):
        add(64, rb(32), rb(16), rb(clen), f"context {clen} B")
    for ilen in (0, 1, 31, 55, 56, 63, 64, 65, 119, 120, 200, 1000):
        add(32, rb(ilen), rb(16), None, f"ikm {ilen} B")
    add(8192, rb(32), rb(16), b"ctx", "counter wraps after 255 blocks")
    add(8161, rb(32), None, None, "counter wraps, truncated")

    # batch-shaped sample: one salt per item, as Identity.encrypt over many destinations
    batch = {"length": 64, "ikm": [], "salt": [], "okm": []}
    for _ in range(64):
        ikm, salt = rb(32), rb(16)
        batch["ikm"].append(ikm.hex())
        batch["salt"].append(salt.hex())
        batch["okm"].append(hkdf(length=64, derive_from=ikm, salt=salt, context=None).hex())

    errors = []
    for args in ({"length": 0, "derive_from": b"x"}, {"length": None, "derive_from": b"x"},
                 {"length": -3, "derive_from": b"x"}, {"length": 5, "derive_from": None},
                 {"length": 5, "derive_from": ""}):
        try:
            hkdf(**args)
            raise AssertionError("expected an error")
        except ValueError as e:
            errors.append({"length": args["length"],
                           "derive_from": None if args["derive_from"] is None else
                           (args["derive_from"].hex() if isinstance(args["derive_from"], bytes) else "str:"),
                           "exc": type(e).__name__, "msg": str(e)})

    # the reference identity KAT: capture the hkdf call made while decrypting fixed_token
    src = open(os.path.join(REF, "tests", "identity.py")).read()
    fixed_key0 = src.split('fixed_keys = [')[1].split('("')[1].split('"')[0]
    ns = {}
    for line in src.splitlines():
        s = line.strip()
        if s.startswith("fixed_token ="):
            ns["fixed_token"] = ast.literal_eval(s.split("=", 1)[1].strip())   # a literal only: never executed
    calls = []
    orig = C.hkdf

    def spy(length=None, derive_from=None, salt=None, context=None):
        out = orig(length=length, derive_from=derive_from, salt=salt, context=context)
        calls.append({"length": length, "ikm": derive_from.hex(), "salt": None if salt is None else salt.hex(),
                      "context": None if context is None else context.hex(), "okm": out.hex()})
        return out

    C.hkdf = spy
    try:
        fid = RNS.Identity.from_bytes(bytes.fromhex(fixed_key0))
        assert fid.decrypt(bytes.fromhex(ns["fixed_token"])) is not None
    finally:
        C.hkdf = orig
    kat = dict(calls[-1])
    kat["source"] = "tests/identity.py:11-19,148-158 via Identity.py:837-846"
    kat["identity_hash"] = fid.hash.hex()
    assert kat["salt"] == fid.hash.hex()

    out = {"reference": "RNS/Cryptography/HKDF.py:35-62", "generator": "tests/golden/gen_hkdf.py",
           "sha256_empty": hashlib.sha256(b"").hexdigest(), "vectors": vec, "batch": batch,
           "errors": errors, "identity_kat": kat}
    path = os.path.join(HERE, "hkdf_vectors.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", path, os.path.getsize(path), "bytes;", len(vec), "vectors")


if __name__ == "__main__":
    main()
