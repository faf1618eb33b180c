#!/bin/bash
# IFAC: build_exp/rot (the ifac_key midstates computed by wave blockIdx % 4,
# RNSTOK_IFAC_ROTATE_KEYWAVE) vs build_exp/base (always wave 0; the product),
# then the wire and pipeline tests on rot.
set -o pipefail
O=gpurun_out/r03ar; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in rot base; do
    RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 200 python -u tools/bench_configs.py --config wire --steps 20 >> $O/wire_$v.jsonl 2>> $O/wire_$v.err || { echo "$v failed"; tail -5 $O/wire_$v.err; exit 1; }
  done
done
for v in rot base; do
  RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python3 tools/bench_configs.py --config wire --steps 20 > $O/trace_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
  f=$(find $O/trace_$v -name "*kernel_stats.csv"); grep -h "ifac" $f | cut -d, -f1-4
done
RNSTOK_LIB=build_exp/rot/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_wire.py tests/test_pipeline_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/rot_tests.log 2>&1 || { echo rot tests failed; tail -20 $O/rot_tests.log; exit 1; }
tail -1 $O/rot_tests.log
