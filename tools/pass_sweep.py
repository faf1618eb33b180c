"""Fixed cost per launch of the c2 kernels: encrypt/decrypt time against the
number of packets per lane (passes), device-resident, one key, 500 B.

  python tools/pass_sweep.py [--rounds R]

For k passes of the 768-thread decrypt (n = 256 CUs x 768 x k) and the same
n for encrypt, the median HIP-event time and the in-run launch clock's mean
workgroup span; a least-squares line time = fixed + k x per_pass separates
the per-launch cost from the per-packet one.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--length", type=int, default=500)
    args = ap.parse_args()
    import torch
    import bench
    import reticulum_amd as rt
    from reticulum_amd import _native, device
    dev = torch.device("cuda", 0)
    n_cu = _native.load().rt_num_cus(_native.context(0))
    L, tl = args.length, rt.token_len(args.length)
    per_pass = n_cu * 768
    ks = rt.KeySet(bytes(range(64)), device=0)
    nmax = per_pass * 8
    g = torch.Generator(device=dev).manual_seed(9)
    pt_all = torch.randint(0, 256, (nmax, L), dtype=torch.uint8, device=dev, generator=g)
    iv_all = torch.randint(0, 256, (nmax, 16), dtype=torch.uint8, device=dev, generator=g)
    tok_all = torch.empty((nmax, tl), dtype=torch.uint8, device=dev)
    back_all = torch.empty((nmax, tl - 48), dtype=torch.uint8, device=dev)
    ol_all = torch.empty(nmax, dtype=torch.int32, device=dev)
    st_all = torch.empty(nmax, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    out = {"per_pass_packets": per_pass, "points": []}
    shapes = [(k, per_pass * k) for k in (1, 2, 3, 4, 5, 6, 8)] + [(round((1 << 20) / per_pass, 3), 1 << 20)]
    for k, n in shapes:
        pt, iv, tok, back, ol, st = pt_all[:n], iv_all[:n], tok_all[:n], back_all[:n], ol_all[:n], st_all[:n]

        def step(ev=None):
            if ev:
                ev[0].record(s)
            device.encrypt_uniform(ks, pt, L, iv, tok)
            if ev:
                ev[1].record(s)
            device.decrypt_uniform(ks, tok, tl, back, ol, st)
            if ev:
                ev[2].record(s)
        bench.warmup(step, s, 3, 0.3)
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.rounds)]
        with device.LaunchClock(dev) as lc:
            for e in evs:
                step(e)
            torch.cuda.synchronize()
        ok = bool((st == 0).all()) and torch.equal(back[:, :L], pt)
        summ = lc.summary()
        e_ms = statistics.median(e[0].elapsed_time(e[1]) for e in evs)
        d_ms = statistics.median(e[1].elapsed_time(e[2]) for e in evs)
        pnt = {"passes": k, "n": n, "ok": ok, "encrypt_ms": e_ms, "decrypt_ms": d_ms,
               "encrypt_span_ms": summ["encrypt"]["wg_span_ms"], "decrypt_span_ms": summ["decrypt"]["wg_span_ms"],
               "encrypt_ghz": summ["encrypt"]["clock_ghz"], "decrypt_ghz": summ["decrypt"]["clock_ghz"],
               "encrypt_cycles": summ["encrypt"]["cycles_per_launch"],
               "decrypt_cycles": summ["decrypt"]["cycles_per_launch"]}
        out["points"].append(pnt)
        print(json.dumps(pnt), flush=True)
    for key in ("encrypt_ms", "decrypt_ms", "encrypt_cycles", "decrypt_cycles"):
        xs = [p["passes"] for p in out["points"] if float(p["passes"]).is_integer()]
        ys = [p[key] for p in out["points"] if float(p["passes"]).is_integer()]
        mx, my = sum(xs) / len(xs), sum(ys) / len(ys)
        b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
        out[key + "_fit"] = {"fixed": my - b * mx, "per_pass": b}
    print(json.dumps({k: v for k, v in out.items() if k.endswith("_fit")}))


if __name__ == "__main__":
    main()
