#!/bin/bash
# After removing the rejected experiment variants from the kernels: the c4
# shard (k_encrypt_long4, whose ring loop was simplified) and c2 A/B against
# the previous build, alternating processes, then the whole GPU suite and
# the smoke on the product build.
set -o pipefail
O=gpurun_out/r03z; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in prev cur; do
    RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 200 python -u tools/bench_configs.py --config c4s8 --steps 20 >> $O/c4s8_$v.jsonl 2>> $O/c4s8_$v.err || { echo "$v failed"; tail -5 $O/c4s8_$v.err; exit 1; }
  done
done
for v in prev cur; do echo == $v; python3 -c "
import json
for l in open('$O/c4s8_$v.jsonl'):
    d=json.loads(l); print({k: v for k, v in d.items() if 'ms' in k or k == 'ok'})
"; done
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -20 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
