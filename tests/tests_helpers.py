"""Small helpers shared by the test modules."""


def b(h):
    return bytes.fromhex(h)


def trial_case(seed, n_tok=40, n_keys=12):
    """Tokens under random keys of a key set and candidate lists in which the
    right key sits at a random rank, is missing, or appears twice; plus
    malformed and too-short tokens that no key opens."""
    import numpy as np
    from oracle import ctoken
    rng = np.random.Generator(np.random.PCG64(seed))
    keys = rng.integers(0, 256, (n_keys, 64), dtype=np.uint8)
    toks, cands, expect = [], [], []
    for t in range(n_tok):
        k = int(rng.integers(0, n_keys))
        pt = rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
        tok = ctoken.encrypt(keys[k].tobytes(), rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), pt)
        others = [i for i in rng.permutation(n_keys).tolist() if i != k][: int(rng.integers(0, 6))]
        mode = t % 5
        if mode == 0:                      # right key missing
            cand, exp = others, -1
        elif mode == 1:                    # right key twice
            cand = others + [k, k]
            exp = k
        elif mode == 2:                    # malformed: ciphertext not whole blocks
            tok, cand, exp = tok[:-33] + tok[-32:], others + [k], -1
        elif mode == 3:                    # too short
            tok, cand, exp = tok[:32], [k], -1
        else:
            pos = int(rng.integers(0, len(others) + 1))
            cand = others[:pos] + [k] + others[pos:]
            exp = k
        toks.append(tok)
        cands.append(cand)
        expect.append(exp)
    return keys, toks, cands, np.array(expect)


def collision_stream(seed, length, dup, sdu=464):
    """The input stream of a Resource collision-guard fixture
    (tests/golden/gen_resource.py): `length` seeded random bytes with part
    dup[1] overwritten by a copy of part dup[0] (no copy when dup is None or
    names one part)."""
    import numpy as np
    stream = bytearray(np.random.Generator(np.random.PCG64(seed)).integers(0, 256, length, dtype=np.uint8).tobytes())
    if dup and dup[0] != dup[1]:
        a, c = dup
        stream[c * sdu:(c + 1) * sdu] = stream[a * sdu:(a + 1) * sdu]
    return bytes(stream)
