# quick GPU check: token parity tests + the given bench_configs configs
set -o pipefail
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 300 python -u -m pytest tests/test_token_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for c in "$@"; do timeout -k 10 200 python tools/bench_configs.py --config $c 2>/dev/null | tee -a gpurun_out/${TAG}_configs.jsonl | cut -c1-300 || exit 1; done
