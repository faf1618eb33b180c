#!/bin/bash
# A/B (one process, interleaved): round keys as VGPR copies shared by a decrypt
# quad's 4 blocks (RNSTOK_DEC_VRK) and per-round LDS broadcast reads in
# single-key encrypt (RNSTOK_ENC_LDSRK) against the product build.
set -o pipefail
O=gpurun_out/r02ar_ab; mkdir -p $O
timeout -k 10 300 python -u tools/exp_bench.py build_exp/base/librnstok.so build_exp/decvrk/librnstok.so \
  build_exp/encldsrk/librnstok.so --rounds 20 > $O/ab.txt 2>&1 || { echo ab failed; tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
