"""PCIe ceiling on this box with pinned host buffers: H2D alone, D2H alone,
and both directions at once on two streams (512 MiB each way), best of 5.
The reference point for bench.py's PCIe-inclusive rows.

  python tools/pcie_ceiling.py
"""
import json
import time

import torch


def main():
    n = 512 << 20
    h_src = torch.empty(n, dtype=torch.uint8).pin_memory()
    h_dst = torch.empty(n, dtype=torch.uint8).pin_memory()
    d_a = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_b = torch.empty(n, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(fn):
        best = float("inf")
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best

    def h2d():
        with torch.cuda.stream(s1):
            d_a.copy_(h_src, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            h_dst.copy_(d_b, non_blocking=True)

    def both():
        h2d()
        d2h()

    t1, t2, t3 = timed(h2d), timed(d2h), timed(both)
    print(json.dumps({"bytes_each_way": n, "h2d_gb_s": n / t1 / 1e9, "d2h_gb_s": n / t2 / 1e9,
                      "bidirectional_gb_s": 2 * n / t3 / 1e9}))


if __name__ == "__main__":
    main()
