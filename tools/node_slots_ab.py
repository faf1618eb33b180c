"""A/B in one process: the composed interface path (reticulum_amd.pipeline)
with its packet buffers in 128-B-aligned slots (aligned=True, the default)
against packets packed end to end (aligned=False); bench.node_rate's workload
(2^20 DATA packets of 383 B, 16-B IFAC).  Rounds interleave the variants;
prints one JSON line with the median HIP-event ms per direction and variant,
and the in-run clock of the token kernels in each."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(rounds=15, n=1 << 20, L=383, isz=16):
    import torch
    import reticulum_amd as rt
    from reticulum_amd import device, pipeline
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(6)
    r = lambda *s: torch.randint(0, 256, s, dtype=torch.uint8, device=dev, generator=g)
    pt, iv, dh, ctx, ifac, ikey = r(n, L), r(n, 16), r(n, 16), r(n), r(n, isz), r(64)
    ks = rt.KeySet(bytes(range(64)), device=0)
    framed, foff = pipeline.outbound(ks, pt, iv, dh, ctx, ifac, ikey)
    torch.cuda.synchronize()
    buf = framed[:int(foff[-1])].clone()
    del framed
    st = torch.cuda.current_stream()
    out = {}
    ref = None
    for al in (True, False):
        f2, o2 = pipeline.outbound(ks, pt, iv, dh, ctx, ifac, ikey, aligned=al)
        res = pipeline.inbound(ks, buf, ikey, isz, 2 * n, aligned=al)
        torch.cuda.synchronize()
        ok = torch.equal(f2[:buf.numel()], buf) and bool((res["status"][:n] == 0).all())
        rows = torch.arange(0, n, 997, device=dev)
        idx = res["pt_off"][rows].unsqueeze(1) + torch.arange(L, device=dev)
        ok = ok and torch.equal(res["pt"][idx], pt[rows])
        if not ok:
            raise SystemExit(f"aligned={al}: wrong results")
        del f2, res
    only = os.environ.get("ONLY")           # "aligned" / "packed": one variant (for a per-kernel trace)
    variants = (True, False) if not only else ((only == "aligned"),)
    times = {(d, al): [] for d in ("outbound", "inbound") for al in variants}
    clocks = {}
    for k in range(rounds + 2):
        for al in (variants if k % 2 == 0 else variants[::-1]):
            for d in ("outbound", "inbound"):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                clk = device.LaunchClock(dev) if k == rounds + 1 else None
                if clk is not None:
                    clk.__enter__()
                a.record(st)
                if d == "outbound":
                    pipeline.outbound(ks, pt, iv, dh, ctx, ifac, ikey, aligned=al)
                else:
                    pipeline.inbound(ks, buf, ikey, isz, 2 * n, aligned=al)
                b.record(st)
                torch.cuda.synchronize()
                if clk is not None:
                    clk.__exit__(None, None, None)
                    clocks[f"{d}_{'aligned' if al else 'packed'}"] = clk.summary()
                if k >= 2:
                    times[(d, al)].append(a.elapsed_time(b))
    for (d, al), v in times.items():
        v.sort()
        out[f"{d}_{'aligned' if al else 'packed'}_ms"] = v[len(v) // 2]
    out["clock"] = clocks
    out["workload"] = f"{n} x {L} B DATA packets, {isz}-B IFAC, one link key"
    print(json.dumps(out))


if __name__ == "__main__":
    main()
