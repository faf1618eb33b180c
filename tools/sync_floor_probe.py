"""The synchronous-call floor under the HIP runtime's wait policies:
hipSetDeviceFlags(<flags>) before anything initialises the device, then
tools/single_call_latency.py's measurements (Token calls, host ABI, device
entry points, a one-element op + synchronize).

  python tools/sync_floor_probe.py --flags 0|1|2|4 [--calls N] [--length B]
      0 auto (the default), 1 spin, 2 yield, 4 blocking sync
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags", type=int, default=0)
    args, rest = ap.parse_known_args()
    import torch        # its HIP runtime (loading another copy of the runtime aborts the process)
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    if args.flags:
        rc = hip.hipSetDeviceFlags(ctypes.c_uint(args.flags))
        print("hipSetDeviceFlags(%d) -> %d" % (args.flags, rc), file=sys.stderr)
    import single_call_latency
    sys.argv = [sys.argv[0]] + rest
    single_call_latency.main()


if __name__ == "__main__":
    main()
