#!/bin/bash
# One-pass HDLC framing (decoupled look-back; tiles of 16 x PASSES packets)
# vs the two-pass count/scan/write.
set -o pipefail
mkdir -p gpurun_out
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -Wno-unused-value"
mkdir -p build_exp/f2 build_exp/p2 build_exp/p4 build_exp/p8
make -s -C reticulum_amd/csrc OUT=$PWD/build_exp/f2/librnstok.so FLAGS="$F -DRNSTOK_FRAME_TWO_PASS" 2>/dev/null || exit 1
for P in 2 4 8; do
  make -s -C reticulum_amd/csrc OUT=$PWD/build_exp/p$P/librnstok.so FLAGS="$F -DRNSTOK_FR_PASSES=$P" 2>/dev/null || exit 1
done
timeout -k 10 120 python -u -m pytest tests/test_wire.py -x -q -m gpu --timeout 100 --timeout-method thread || exit 1
for r in 1 2; do
  for V in p16 two p2 p4 p8; do
    case $V in p16) unset RNSTOK_LIB;; two) export RNSTOK_LIB=$PWD/build_exp/f2/librnstok.so;; *) export RNSTOK_LIB=$PWD/build_exp/$V/librnstok.so;; esac
    echo -n "$V run $r: "
    timeout -k 10 120 python3 tools/bench_configs.py --config wire --steps 10 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ok'], round(d['stages']['hdlc_frame']['ms'], 4), 'ms frame')" || exit 1
  done
done
