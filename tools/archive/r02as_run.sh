#!/bin/bash
# Key-table broadcast (shard.broadcast_keyset) on the GPU: the device.keyset
# test, then bench.py's N > 1 path rehearsed on one GPU over gloo (default
# run with the sharded c4 pass, and --config c5 at 3 ranks with 300 001
# packets), every round trip checked.
set -o pipefail
O=gpurun_out/r02as; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_runtime_gpu.py -x -v -m gpu -k "device_keyset" --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -20 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
RNSTOK_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-seconds 0 > $O/rehearse_n2.json 2> $O/rehearse_n2.err || { echo rehearse n2 failed; tail -30 $O/rehearse_n2.err; exit 1; }
cut -c1-300 $O/rehearse_n2.json
RNSTOK_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 3 --config c5 --packets 300001 > $O/rehearse_c5_n3.json 2> $O/rehearse_c5_n3.err || { echo rehearse c5 failed; tail -30 $O/rehearse_c5_n3.err; exit 1; }
cut -c1-300 $O/rehearse_c5_n3.json
echo all ok
