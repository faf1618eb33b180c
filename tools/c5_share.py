"""One rank's share of c5 at 8 GPUs (bench.c5_share_rate) on its own, for
kernel traces and PMC passes of the ragged per-key kernels.

  python tools/c5_share.py [--steps K]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--packets", type=int, default=1 << 20)
    ap.add_argument("--align", action="store_true", help="packets in 128-B-aligned slots")
    ap.add_argument("--align-sides", default="", help="only these buffers in slots: enc_in,enc_out,dec_in,dec_out")
    args = ap.parse_args()
    import torch
    import bench
    from reticulum_amd import _native
    dev = torch.device("cuda", 0)
    n_cu = _native.load().rt_num_cus(_native.context(0))
    print(json.dumps(bench.c5_share_rate(dev, n_cu, n=args.packets, steps=args.steps,
                                          align=True if args.align else set(filter(None, args.align_sides.split(","))))), flush=True)


if __name__ == "__main__":
    main()
