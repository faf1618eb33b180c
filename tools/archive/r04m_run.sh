#!/bin/bash
# GPU suite + smoke + default bench line; c5 share trace + PMC on the split
# kernels; the bare coalescing-gather cost at c5's share.
set -o pipefail
O=gpurun_out/r04m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-200 $O/bench.json
timeout -k 10 200 python tools/c5_gather_cost.py > $O/c5_gather_cost.json 2> $O/c5_gather_cost.err || { tail -5 $O/c5_gather_cost.err; exit 1; }
cat $O/c5_gather_cost.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5/trace -o run -- python3 tools/c5_share.py > $O/c5_trace.log 2>&1 || { tail -20 $O/c5_trace.log; exit 1; }
for PASS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_ACTIVE_INST_VALU2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM" \
            "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT" "TCC_HIT_sum TCC_MISS_sum"; do
  N=$(echo $PASS | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 200 rocprofv3 --pmc $PASS --output-format csv -d $O/c5/pmc_$N -o run -- python3 tools/c5_share.py --steps 3 > $O/c5/pmc_$N.log 2>&1 || { echo "pmc pass $N failed rc=$?"; tail -5 $O/c5/pmc_$N.log; exit 1; }
done
python3 tools/pmc_summary.py $O/c5 --json $O/c5/pmc.json > $O/c5/pmc_summary.txt 2>&1
cp $O/c5/trace/run_kernel_stats.csv $O/c5/kernel_stats.csv
echo r04m done
