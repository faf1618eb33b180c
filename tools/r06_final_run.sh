#!/bin/bash
# Round 6 final build: full GPU suite, smoke, default bench line (in-run clock),
# the headline's kernel trace + PMC passes, c3/c4/c5 config lines, and the
# N = 2 gloo rehearsal (both ranks on the one GPU) of the default bench and
# --config c4|c5.  Usage: tools/r06_final_run.sh <tag>
set -o pipefail
TAG=${1:-r06z}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
bash tools/profile.sh $TAG > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
tail -2 $O/profile.log
timeout -k 10 300 python -u bench.py --config c3 --cpu-seconds 0 --no-e2e --no-node > $O/bench_c3.json 2> $O/bench_c3.err || { tail $O/bench_c3.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c4 > $O/bench_c4.json 2> $O/bench_c4.err || { tail $O/bench_c4.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c5 > $O/bench_c5.json 2> $O/bench_c5.err || { tail $O/bench_c5.err; exit 1; }
RNSTOK_BENCH_REHEARSE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29621 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-seconds 4 > $O/rehearse_n2.json 2> $O/rehearse_n2.err || { echo rehearse n2 failed; tail -30 $O/rehearse_n2.err; exit 1; }
RNSTOK_BENCH_REHEARSE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29622 bench.py --gpus 2 --config c5 > $O/rehearse_n2_c5.json 2> $O/rehearse_n2_c5.err || { echo rehearse n2 c5 failed; tail -30 $O/rehearse_n2_c5.err; exit 1; }
RNSTOK_BENCH_REHEARSE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29623 bench.py --gpus 2 --config c4 > $O/rehearse_n2_c4.json 2> $O/rehearse_n2_c4.err || { echo rehearse n2 c4 failed; tail -30 $O/rehearse_n2_c4.err; exit 1; }
cut -c1-200 $O/rehearse_n2.json $O/rehearse_n2_c5.json $O/rehearse_n2_c4.json
echo final run done
