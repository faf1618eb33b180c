#!/bin/bash
# Coalesced-layout experiment: time (A/B in one process) and HBM traffic (PMC) of k_encrypt with 16-B units
# interleaved across packets (fully coalesced loads/stores) vs the packed-row layout.
O=gpurun_out/r02o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/exp_bench.py build_exp/v2/librnstok.so build_exp/base2/librnstok.so build_exp/coal/librnstok.so --rounds 20 --probe > $O/ab.txt 2>&1 || exit 1
for V in base2 coal; do
  for PASS in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $PASS --output-format csv -d $O/pmc_${V}_$PASS -o run -- python3 tools/exp_bench.py build_exp/$V/librnstok.so --rounds 4 --probe > $O/pmc_${V}_$PASS.log 2>&1 || { echo "pmc $V $PASS failed"; exit 1; }
  done
done
echo done
