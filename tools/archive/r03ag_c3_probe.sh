#!/bin/bash
# c3 (2^20 x 500 B, 65 536 per-packet keys): how much do the per-packet key
# record gathers cost?  The same per-key kernels with key_idx random (the
# config), sorted (lanes of a wave share keys), all zero, and sequential, in
# both layouts; product library only.
set -o pipefail
O=gpurun_out/r03ag; mkdir -p $O
export TMPDIR=/tmp
for ilv in "" "--ilv"; do
  for k in random sorted zero seq; do
    echo "== kidx=$k $ilv" >> $O/c3_probe.txt
    timeout -k 10 200 python3 tools/exp_bench.py reticulum_amd/librnstok.so --keys 65536 --kidx $k $ilv --rounds 15 >> $O/c3_probe.txt 2>&1 || { echo probe failed; tail $O/c3_probe.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/c3_probe.txt
