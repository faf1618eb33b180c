"""A/B in one process of pipeline.outbound's slot layouts (through a pipeline._SLOTS knob, removed
after this A/B; the tool no longer runs against the product):
where each packet sits in its 128-B line (the token ciphertext's phase, or the
IFAC size so the IFAC mask's 32-B payload loads are aligned) and whether the
masked packets get line-aligned slots too; packed rows as the baseline.
bench.node_rate's workload; interleaved rounds, median HIP-event ms."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

VARIANTS = {
    "packed": None,
    "ct": {"raw_base": None, "masked_slots": False},
    "ct_mslots": {"raw_base": None, "masked_slots": True},
    "ifac": {"raw_base": "ifac", "masked_slots": False},
    "ifac_mslots": {"raw_base": "ifac", "masked_slots": True},
}


def main(rounds=15, n=1 << 20, L=383, isz=16):
    import torch
    import reticulum_amd as rt
    from reticulum_amd import pipeline
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(6)
    r = lambda *s: torch.randint(0, 256, s, dtype=torch.uint8, device=dev, generator=g)
    pt, iv, dh, ctx, ifac, ikey = r(n, L), r(n, 16), r(n, 16), r(n), r(n, isz), r(64)
    ks = rt.KeySet(bytes(range(64)), device=0)
    st = torch.cuda.current_stream()

    def run(v):
        if VARIANTS[v] is None:
            return pipeline.outbound(ks, pt, iv, dh, ctx, ifac, ikey, aligned=False)
        pipeline._SLOTS.update(VARIANTS[v])
        return pipeline.outbound(ks, pt, iv, dh, ctx, ifac, ikey, aligned=True)

    ref, roff = run("packed")
    total = int(roff[-1])
    for v in VARIANTS:
        f, o = run(v)
        if not (torch.equal(o, roff) and torch.equal(f[:total], ref[:total])):
            raise SystemExit(f"{v}: stream differs")
    del ref
    times = {v: [] for v in VARIANTS}
    names = list(VARIANTS)
    for k in range(rounds + 2):
        for v in (names if k % 2 == 0 else names[::-1]):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            run(v)
            b.record(st)
            torch.cuda.synchronize()
            if k >= 2:
                times[v].append(a.elapsed_time(b))
    out = {f"{v}_ms": sorted(t)[len(t) // 2] for v, t in times.items()}
    out["workload"] = f"{n} x {L} B DATA packets, {isz}-B IFAC, one link key; outbound"
    print(json.dumps(out))


if __name__ == "__main__":
    main()
