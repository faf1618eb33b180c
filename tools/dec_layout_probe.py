"""Decrypt (or encrypt, --kernel encrypt) alone on two token layouts of the same c2 packets: packed rows (560-B
stride) and each token's ciphertext on a 128-B line (640-B stride, +112).
Runs of back-to-back decrypts, the layouts alternated; per layout the median
HIP-event time, and the kernel's own clock and cycles (rt_clock_stamps).

  python tools/dec_layout_probe.py [--runs 8] [--per-run 20] [--length 500]
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
    ap.add_argument("--runs", type=int, default=8)
    ap.add_argument("--per-run", type=int, default=20)
    ap.add_argument("--packets", type=int, default=1 << 20)
    ap.add_argument("--length", type=int, default=500)
    ap.add_argument("--kernel", choices=["decrypt", "encrypt"], default="decrypt")
    ap.add_argument("--back-stride", type=int, default=0, help="decrypt output row stride (0: tl - 48)")
    ap.add_argument("--pt-stride", type=int, default=0, help="encrypt input row stride (0: packed, the length)")
    ap.add_argument("--extra", default="", help="more token layouts, e.g. 576+0,640+0 (stride+first offset)")
    args = ap.parse_args()
    import torch
    import reticulum_amd as rt
    from reticulum_amd import device
    n, L = args.packets, args.length
    tl = rt.token_len(L)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    ps = args.pt_stride or L
    pt_buf = torch.empty(n * ps + 256, dtype=torch.uint8, device=dev)
    pt = pt_buf[(-pt_buf.data_ptr()) % 256:].as_strided((n, L), (ps, 1))
    pt.copy_(torch.randint(0, 256, (n, L), dtype=torch.uint8, device=dev, generator=g))
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device=dev, generator=g)
    ks = rt.KeySet(os.urandom(64), device=0)
    def rows(stride, off):
        """(n, tl) token rows at `stride`, the first at byte `off` of a 256-B-aligned buffer"""
        buf = torch.empty(n * stride + 512, dtype=torch.uint8, device=dev)
        base = (-buf.data_ptr()) % 256 + off
        return buf[base:].as_strided((n, tl), (stride, 1))
    layouts = {"packed": rows(tl, 0), "ct_on_line": device.aligned_rows(n, tl, 16, dev)}
    for spec in args.extra.split(",") if args.extra else []:
        stride, off = (int(x) for x in spec.split("+"))
        layouts[f"stride{stride}+{off}"] = rows(stride, off)
    bs = args.back_stride or tl - 48
    back = torch.empty(n * bs + 256, dtype=torch.uint8, device=dev)
    back = back[(-back.data_ptr()) % 256:].as_strided((n, tl - 48), (bs, 1))
    ol = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    for tok in layouts.values():
        device.encrypt_uniform(ks, pt, L, iv, tok, stream=stream)
        device.decrypt_uniform(ks, tok, tl, back, ol, st, stream=stream)
        torch.cuda.synchronize()
        assert bool((st == 0).all()) and torch.equal(back[:, :L], pt)
    for tok in layouts.values():
        assert torch.equal(layouts["packed"], tok)
    res = {k: {"ms": [], "clock": [], "cycles": []} for k in layouts}

    def run(tok):
        if args.kernel == "decrypt":
            device.decrypt_uniform(ks, tok, tl, back, ol, st, stream=stream)
        else:
            device.encrypt_uniform(ks, pt, L, iv, tok, stream=stream)
    for r in range(args.runs):
        names = list(layouts)
        for name in names[r % len(names):] + names[:r % len(names)]:
            tok = layouts[name]
            for _ in range(args.per_run):           # clock settles on this layout
                run(tok)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.per_run)]
            for a, b in ev:
                a.record(stream)
                run(tok)
                b.record(stream)
            torch.cuda.synchronize()
            with device.LaunchClock(dev) as lc:
                for _ in range(args.per_run):
                    run(tok)
            c = lc.summary()[args.kernel]
            res[name]["ms"].append(statistics.median(a.elapsed_time(b) for a, b in ev))
            res[name]["clock"].append(c["clock_ghz"])
            res[name]["cycles"].append(c["cycles_per_launch"])
    out = {k: {"ms": statistics.median(v["ms"]), "clock_ghz": statistics.median(v["clock"]),
               "cycles_per_launch": statistics.median(v["cycles"])} for k, v in res.items()}
    out["workload"] = {"packets": n, "length": L, "kernel": args.kernel, "back_stride": bs, "pt_stride": ps}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
