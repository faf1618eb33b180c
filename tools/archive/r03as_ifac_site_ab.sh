#!/bin/bash
# IFAC code size: build_exp/site (PRK, its outer hash and PRK's key midstates
# through one inlined compression, RNSTOK_IFAC_ONE_SITE, capped at 4
# waves/SIMD) and build_exp/sitex (+ each expand block's inner and outer hash
# through one, RNSTOK_IFAC_ONE_SITE_X) vs build_exp/base (the product), then
# the wire and pipeline tests on both variants.
set -o pipefail
O=gpurun_out/r03as; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in site sitex base; do
    RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 200 python -u tools/bench_configs.py --config wire --steps 20 >> $O/wire_$v.jsonl 2>> $O/wire_$v.err || { echo "$v failed"; tail -5 $O/wire_$v.err; exit 1; }
  done
done
for v in site sitex base; do
  RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python3 tools/bench_configs.py --config wire --steps 20 > $O/trace_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
done
for v in site sitex; do
  RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_wire.py tests/test_pipeline_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/${v}_tests.log 2>&1 || { echo $v tests failed; tail -20 $O/${v}_tests.log; exit 1; }
  tail -1 $O/${v}_tests.log
done
for v in site sitex base; do python3 -c "
import json
for l in open('$O/wire_$v.jsonl'):
    d=json.loads(l); print('$v', d['ok'], {k: round(s.get('ms', 0),4) for k, s in d['stages'].items() if 'ifac' in k})
"; done
