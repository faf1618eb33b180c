#!/bin/bash
# round 4: the one-rank RCCL script's self send/recv outcome, bench tests, default bench line
set -o pipefail
mkdir -p gpurun_out
WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 timeout -k 10 180 python -u tests/rccl_one_rank.py > gpurun_out/r04n_rccl1.json 2> gpurun_out/r04n_rccl1.err &&
python -c "import json;d=json.loads(open('gpurun_out/r04n_rccl1.json').read().splitlines()[-1]);d.pop('tokens');print(json.dumps(d))" &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_bench_gpu.py > gpurun_out/r04n_bench_tests.log 2>&1 &&
tail -3 gpurun_out/r04n_bench_tests.log &&
timeout -k 10 600 python -u bench.py > gpurun_out/r04n_bench.json 2> gpurun_out/r04n_bench.err &&
tail -c 600 gpurun_out/r04n_bench.json
