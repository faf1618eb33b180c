"""bench.per_call_rate at several thread counts (Token vs CoalescingToken)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    for th in (1, 4, 16, 64):
        print(json.dumps(bench.per_call_rate(threads=th, calls=400 if th < 64 else 200)), flush=True)


if __name__ == "__main__":
    main()
