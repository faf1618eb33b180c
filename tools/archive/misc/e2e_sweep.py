"""Sweep of the PCIe-inclusive (pinned host memory in and out) pipeline shape:
slices x streams x D2H mechanism (GPU stores / copy engine), c2 batch (2^20 x 500 B, one key).  Prints one JSON line per
shape with encrypt / decrypt packets/s (bench.e2e_rate, best of 3).

  python tools/e2e_sweep.py [--chunks 8,16,32,64] [--streams 2,3,4,8]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="8,16,32,64")
    ap.add_argument("--streams", default="2,3,4,8")
    ap.add_argument("--packets", type=int, default=1 << 20)
    ap.add_argument("--length", type=int, default=500)
    args = ap.parse_args()
    import torch
    import bench
    import reticulum_amd as rt
    n, L = args.packets, args.length
    tl = rt.token_len(L)
    g = torch.Generator(device="cuda").manual_seed(9)
    pt = torch.randint(0, 256, (n, L), dtype=torch.uint8, device="cuda", generator=g)
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    ks = rt.KeySet(bytes(range(64)), device=0)
    stream = torch.cuda.current_stream()
    for c in map(int, args.chunks.split(",")):
        for s in map(int, args.streams.split(",")):
            res = bench.e2e_rate(ks, pt, iv, L, tl, n, stream, chunks=c, n_streams=s)
            for d2h, key in (("stores", "pipelined"), ("copy_engine", "pipelined_copy_engine")):
                r = res[key]
                print(json.dumps({"chunks": c, "streams": s, "d2h": d2h, "enc_Mpkt_s": r["encrypt_packets_s"] / 1e6,
                                  "dec_Mpkt_s": r["decrypt_packets_s"] / 1e6, "pcie_gb_s": r["encrypt_pcie_gb_s"],
                                  "ok": r["ok"]}), flush=True)


if __name__ == "__main__":
    main()
