#!/bin/bash
# Round 3: new GPU tests (8-GPU per-rank shapes, side-stream key setup), then
# bench.py's N > 1 path rehearsed on one GPU over gloo at 2 and 4 ranks
# (e2e on every rank, CPU baseline at N > 1, the pipelined sharded c4 pass).
set -o pipefail
O=gpurun_out/r03f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_rank_shapes_gpu.py tests/test_bench_gpu.py tests/test_interleaved_gpu.py tests/test_runtime_gpu.py -x -v -s -m gpu -k "rank_shape or 8gpu or sharded_config or side_stream or device_keyset or interleaved or counter_ring" --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
RNSTOK_BENCH_REHEARSE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-seconds 4 > $O/rehearse_n2.json 2> $O/rehearse_n2.err || { echo rehearse n2 failed; tail -30 $O/rehearse_n2.err; exit 1; }
cut -c1-400 $O/rehearse_n2.json
RNSTOK_BENCH_REHEARSE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 4 --steps 5 --warmup 2 --cpu-seconds 4 > $O/rehearse_n4.json 2> $O/rehearse_n4.err || { echo rehearse n4 failed; tail -30 $O/rehearse_n4.err; exit 1; }
cut -c1-400 $O/rehearse_n4.json
echo all ok
