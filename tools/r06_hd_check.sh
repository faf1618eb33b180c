#!/bin/bash
# the one-packet direct host path (exp_ship/hd1): host-path GPU tests on it, then the per-call A/B against base
set -o pipefail
mkdir -p gpurun_out/r06at
RNSTOK_LIB=exp_ship/hd1/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_token_gpu.py tests/test_threads_gpu.py tests/test_dropin_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r06at/tests_hd1.log 2>&1 || { tail -30 gpurun_out/r06at/tests_hd1.log; exit 1; }
tail -2 gpurun_out/r06at/tests_hd1.log
bash tools/r06_h2d_ab.sh r06at 3 base hd1
