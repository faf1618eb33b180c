"""Where a coalesced batch's time goes: Coalescer._execute on batches of k
encrypts / decrypts with k distinct keys (the key table already built), and
the same k packets as one key's batch, vs k plain Token calls."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import reticulum_amd as rt
    from reticulum_amd import coalesce
    out = {}
    for k in (1, 2, 8, 32):
        co = coalesce.Coalescer()
        toks = [coalesce.CoalescingToken(os.urandom(64)) for _ in range(k)]
        one = coalesce.CoalescingToken(os.urandom(64))
        pts = [os.urandom(383) for _ in range(k)]
        enc = lambda ts: [coalesce._Call(coalesce._ENC, t, p) for t, p in zip(ts, pts)]   # noqa: E731
        calls = enc(toks)
        co._execute(calls * 1 if k > 1 else calls + enc(toks))            # builds the table
        tokens = [c.result for c in enc(toks)]
        co._execute(calls2 := enc(toks))
        tokens = [c.result for c in calls2]
        res = {}
        for name, make in (("enc_k_keys", lambda: enc(toks)),
                           ("dec_k_keys", lambda: [coalesce._Call(coalesce._DEC, t, x) for t, x in zip(toks, tokens)]),
                           ("enc_one_key", lambda: enc([one] * k))):
            reps = 60
            t0 = time.perf_counter()
            for _ in range(reps):
                b = make()
                if len(b) == 1:
                    b = b + make()[:0]
                co._execute(b)
                assert all(c.error is None for c in b), [c.error for c in b][:2]
            res[name + "_us"] = (time.perf_counter() - t0) / reps * 1e6
        t0 = time.perf_counter()
        for _ in range(20):
            for t, p in zip(toks, pts):
                rt.Token.encrypt(t, p)
        res["plain_token_enc_k_calls_us"] = (time.perf_counter() - t0) / 20 * 1e6
        out[k] = res
        print(k, json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
