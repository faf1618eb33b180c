#!/bin/bash
# Kernel trace + PMC passes of any python command (run on the GPU box via gpurun).
# Usage: tools/profile_cmd.sh <out_dir> <workload p,l,k or -> <python script> [args...]
# Each rocprofv3 run holds one pass (separate --pmc runs; no trace domains mixed with counters).
set -o pipefail
OUT=$1; WL=$2; shift 2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 "$@" > $OUT/trace.log 2>&1 || { echo "trace failed rc=$?"; tail -5 $OUT/trace.log; exit 1; }
for PASS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
            "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  N=$(echo $PASS | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 300 rocprofv3 --pmc $PASS --output-format csv -d $OUT/pmc_$N -o run -- python3 "$@" > $OUT/pmc_$N.log 2>&1 || { echo "pmc pass $N failed rc=$?"; tail -5 $OUT/pmc_$N.log; exit 1; }
done
if [ "$WL" != "-" ]; then W="--workload $WL"; else W=""; fi
python3 tools/pmc_summary.py $OUT --json $OUT/pmc.json $W > $OUT/pmc_summary.txt
cp $OUT/trace/run_kernel_stats.csv $OUT/kernel_stats.csv
echo profile done $OUT
