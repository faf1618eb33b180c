"""The latency kernels on one packet per launch (Token's call shape): per
plaintext length, k_encrypt_long4 / k_decrypt_long2 launched one at a time
(synchronised after each, as a Token call is), with their own cycles, clock
and workgroup span from the launch clock (rt_clock_stamps).  With a probe
build (RNSTOK_L4_PROBE_AES_ONLY / _SHA_ONLY, RNSTOK_DL2_PROBE_*) it times
one side of the kernel alone (the tokens are then wrong; nothing is checked).

  RNSTOK_LIB=... python tools/one_packet_probe.py [--calls 300] [--lengths 100,383,1000]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=300)
    ap.add_argument("--lengths", default="100,383,1000")
    args = ap.parse_args()
    import torch
    import reticulum_amd as rt
    from reticulum_amd import device
    dev = torch.device("cuda", 0)
    ks = rt.KeySet(os.urandom(64), device=0)
    out = {"lib": os.environ.get("RNSTOK_LIB", "reticulum_amd/librnstok.so")}
    for L in (int(x) for x in args.lengths.split(",")):
        tl = rt.token_len(L)
        pt = torch.randint(0, 256, (1, L), dtype=torch.uint8, device=dev)
        iv = torch.randint(0, 256, (1, 16), dtype=torch.uint8, device=dev)
        tok = torch.zeros(1, tl, dtype=torch.uint8, device=dev)
        back = torch.zeros(1, tl - 48, dtype=torch.uint8, device=dev)
        ol = torch.zeros(1, dtype=torch.int32, device=dev)
        st = torch.zeros(1, dtype=torch.int32, device=dev)
        res = {}
        for name, f in (("encrypt", lambda: device.encrypt_uniform(ks, pt, L, iv, tok)),
                        ("decrypt", lambda: device.decrypt_uniform(ks, tok, tl, back, ol, st))):
            for _ in range(30):
                f()
                torch.cuda.synchronize()
            with device.LaunchClock(dev) as lc:
                for _ in range(args.calls):
                    f()
                    torch.cuda.synchronize()
            s = lc.summary().get(name)
            if s is None:           # (the DL2 AES-only probe does not stamp)
                continue
            res[name] = {"us": round(s["wg_span_ms"] * 1e3, 2), "kcycles": round(s["cycles_per_launch"] / 1e3, 2),
                         "clock_ghz": round(s["clock_ghz"], 3)}
        res["round_trip_ok"] = bool(int(st[0]) == 0 and torch.equal(back[0, :L], pt[0]))
        # the same kernels behind Token (rt_*_host, n = 1: inputs and outputs in the mapped pinned staging buffer)
        tk, msg = rt.Token(os.urandom(64)), os.urandom(L)
        for name, f in (("token_encrypt", lambda: tk.encrypt(msg)), ("token_decrypt", None)):
            if f is None:
                t0 = tk.encrypt(msg)
                f = lambda: tk.decrypt(t0)      # noqa: E731
            for _ in range(30):
                f()
            with device.LaunchClock(dev) as lc:
                for _ in range(args.calls):
                    f()
            s = lc.summary().get(name.split("_")[1])
            if s is not None:
                res[name] = {"us": round(s["wg_span_ms"] * 1e3, 2), "kcycles": round(s["cycles_per_launch"] / 1e3, 2),
                             "clock_ghz": round(s["clock_ghz"], 3)}
        out[L] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
