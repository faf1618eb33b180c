#!/bin/bash
# Round 3: c4 sharded in both directions and c3's key setup timing (SURVEY
# §8(d)): the bench GPU tests, the c3 and c4 lines at N = 1, then bench.py's
# N > 1 path rehearsed on one GPU over gloo at 2 ranks.
set -o pipefail
O=gpurun_out/r03m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_rank_shapes_gpu.py tests/test_bench_gpu.py -x -v -s -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
RNSTOK_BENCH_REHEARSE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29621 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-seconds 4 > $O/rehearse_n2.json 2> $O/rehearse_n2.err || { echo rehearse n2 failed; tail -30 $O/rehearse_n2.err; exit 1; }
cut -c1-400 $O/rehearse_n2.json
timeout -k 10 300 python -u bench.py --config c3 --cpu-seconds 0 --no-e2e > $O/bench_c3.json 2> $O/bench_c3.err || { echo c3 failed; tail $O/bench_c3.err; exit 1; }
cut -c1-300 $O/bench_c3.json
timeout -k 10 300 python -u bench.py --config c4 > $O/bench_c4.json 2> $O/bench_c4.err || { echo c4 failed; tail $O/bench_c4.err; exit 1; }
cut -c1-300 $O/bench_c4.json
echo all ok
