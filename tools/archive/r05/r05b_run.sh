#!/bin/bash
# Round 5: full GPU suite + smoke + default bench line (in-run launch clock),
# the clock cross-checked against GRBM_GUI_ACTIVE, and an A/B of the build
# against round 4's product (stamps off) at c2.
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc_clk -o run -- python3 bench.py --steps 30 --warmup 2 --cpu-seconds 0 --no-e2e --no-node --one-layout > $O/bench_pmc.json 2> $O/bench_pmc.err || { tail -20 $O/bench_pmc.err; exit 1; }
python3 tools/clock_check.py $O/pmc_clk $O/bench_pmc.json 30 > $O/clock_check.json && cat $O/clock_check.json
for args in "" "--ilv"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py build_exp/base/librnstok.so reticulum_amd/librnstok.so --rounds 20 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt | grep -v round-trip
