#!/bin/bash
# Round 3: the headline bench line as the driver runs it (default flags), c3, and the c4/c5 configs at N = 1.
set -o pipefail
O=gpurun_out/r03l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
timeout -k 10 300 python -u bench.py --config c3 --cpu-seconds 0 --no-e2e > $O/bench_c3.json 2> $O/bench_c3.err || { echo c3 failed; tail $O/bench_c3.err; exit 1; }
cut -c1-300 $O/bench_c3.json
timeout -k 10 300 python -u bench.py --config c4 > $O/bench_c4.json 2> $O/bench_c4.err || { echo c4 failed; tail $O/bench_c4.err; exit 1; }
cut -c1-300 $O/bench_c4.json
timeout -k 10 300 python -u bench.py --config c5 > $O/bench_c5.json 2> $O/bench_c5.err || { echo c5 failed; tail $O/bench_c5.err; exit 1; }
cut -c1-300 $O/bench_c5.json
echo all ok
