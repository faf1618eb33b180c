"""Throwaway: IFAC unmask time with its input frames at stream offsets vs
copied into 128-B-aligned slots at several phases (kernel only, HIP events)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
    max_pairs = 2 * n
    out = torch.empty(buf.numel(), dtype=torch.uint8, device=dev)
    d_off = torch.empty(max_pairs, dtype=torch.int64, device=dev)
    d_len = torch.empty(max_pairs, dtype=torch.int32, device=dev)
    d_st = torch.full((max_pairs,), -1, dtype=torch.int32, device=dev)
    counts = torch.empty(2, dtype=torch.int64, device=dev)
    device.hdlc_deframe(buf, out, d_off, d_len, d_st, counts, ifac_size=isz)
    f_off = torch.empty(max_pairs, dtype=torch.int64, device=dev)
    f_len = torch.empty(max_pairs, dtype=torch.int32, device=dev)
    fp = torch.empty(max_pairs, dtype=torch.int64, device=dev)
    nf = torch.empty((), dtype=torch.int64, device=dev)
    device.frames_compact(d_off, d_len, d_st, counts, f_off, f_len, fp, nf)
    torch.cuda.synchronize()
    m = int(nf)
    fo, fl = f_off[:m], f_len[:m]
    ml = int(fl.max())
    stride = -(-ml // 128) * 128
    variants = {"stream": (out, fo)}
    for ph in (0, 16, 35, 93):
        sl = device.aligned_rows(m, ml, ph, dev)
        s_flat = sl.as_strided((m * sl.stride(0),), (1,))
        idx = fo.unsqueeze(1) + torch.arange(ml, device=dev)
        sl.copy_(out[idx.clamp(max=out.numel() - 1)])
        so = torch.arange(m, dtype=torch.int64, device=dev) * sl.stride(0)
        variants[f"slot_phase{ph}"] = (s_flat, so)
    ifc = torch.empty((m, isz), dtype=torch.uint8, device=dev)
    st = torch.empty(m, dtype=torch.int32, device=dev)
    pl = torch.empty(m, dtype=torch.int32, device=dev)
    un = torch.empty(buf.numel(), dtype=torch.uint8, device=dev)
    res = {}
    ref = None
    for v, (src, so) in variants.items():
        device.ifac_unmask(src, so, fl, ikey, ifc, un, fo, st, out_len=pl)
        torch.cuda.synchronize()
        got = un.clone()
        if ref is None:
            ref = got
        assert torch.equal(got, ref) and bool((st == 0).all()), v
    t = {v: [] for v in variants}
    s = torch.cuda.current_stream()
    names = list(variants)
    for k in range(rounds + 2):
        for v in (names if k % 2 == 0 else names[::-1]):
            src, so = variants[v]
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            device.ifac_unmask(src, so, fl, ikey, ifc, un, fo, st, out_len=pl)
            b.record(s)
            torch.cuda.synchronize()
            if k >= 2:
                t[v].append(a.elapsed_time(b))
    print(json.dumps({v: sorted(x)[len(x) // 2] for v, x in t.items()}))


if __name__ == "__main__":
    main()
