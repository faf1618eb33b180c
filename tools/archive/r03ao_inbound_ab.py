"""Same-process A/B of the inbound pipeline: the round-3 r03ac version
(tools/archive/pipeline_r03ac.py: frame compaction and token spans as torch
ops) against reticulum_amd.pipeline (rt_frames_compact, rt_token_spans), on
one 2^20-packet stream (bench.node_rate's shape), alternating, HIP events on
the current stream; both results compared entry by entry."""
import importlib.util
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import reticulum_amd as rt                      # noqa: E402
from reticulum_amd import pipeline as new       # noqa: E402

spec = importlib.util.spec_from_file_location("reticulum_amd._pipeline_r03ac",
                                              os.path.join(ROOT, "tools/archive/pipeline_r03ac.py"))
old = importlib.util.module_from_spec(spec)
spec.loader.exec_module(old)

dev = torch.device("cuda", 0)
n, L, isz = 1 << 20, 383, 16
g = torch.Generator(device=dev).manual_seed(6)
r = lambda *s: torch.randint(0, 256, s, dtype=torch.uint8, device=dev, generator=g)
pt, iv, dh, ctx, ifac, ikey = r(n, L), r(n, 16), r(n, 16), r(n), r(n, isz), r(64)
ks = rt.KeySet(bytes(range(64)), device=0)
framed, foff = new.outbound(ks, pt, iv, dh, ctx, ifac, ikey)
torch.cuda.synchronize()
buf = framed[:int(foff[-1])].clone()
ra, rb = old.inbound(ks, buf, ikey, isz, 2 * n), new.inbound(ks, buf, ikey, isz, 2 * n)
torch.cuda.synchronize()
same = all(torch.equal(ra[k], rb[k]) for k in ("status", "pt_len", "pt_off", "frame_pair", "n_frames", "ifac_status",
                                                "frame_status", "counts"))
same = same and int(rb["n_frames"]) == n and torch.equal(ra["fields"][:n], rb["fields"][:n])
s = torch.cuda.current_stream()
times = {"r03ac_torch_glue": [], "device_glue": []}
for rep in range(6):
    for name, mod in (("r03ac_torch_glue", old), ("device_glue", new)):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for a, b in ev:
            a.record(s)
            mod.inbound(ks, buf, ikey, isz, 2 * n)
            b.record(s)
        torch.cuda.synchronize()
        if rep:                                  # rep 0 warms the clock
            times[name] += [a.elapsed_time(b) for a, b in ev]
med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
print(json.dumps({"same_results": same, "inbound_ms_median": med,
                  "packets_s": {k: n / (v * 1e-3) for k, v in med.items()}}))
