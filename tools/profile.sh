#!/bin/bash
# Kernel-trace + PMC profile of bench.py on one GPU (run on the GPU box via gpurun).
# Usage: tools/profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
ARGS="--steps 30 --warmup 2 --cpu-seconds 0 --no-e2e --no-node --one-layout $@"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit $?
for PASS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
            "SQ_IFETCH SQ_IFETCH_LEVEL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_LEVEL_LDS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_SMEM" \
            "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  N=$(echo $PASS | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --pmc $PASS --output-format csv -d $OUT/pmc_$N -o run -- python3 bench.py $ARGS > $OUT/pmc_$N.log 2>&1 || { echo "pmc pass $N failed rc=$?"; tail -5 $OUT/pmc_$N.log; exit 1; }
done
WL=$(python3 -c "
import sys; a=sys.argv[1:]
g=lambda f,d: a[a.index(f)+1] if f in a else d
print(','.join([g('--packets','1048576'), g('--length','500'), g('--keys','1')]))" $ARGS)
python3 tools/pmc_summary.py $OUT --json $OUT/pmc.json --workload $WL > $OUT/pmc_summary.txt
cp $OUT/trace/run_kernel_stats.csv $OUT/kernel_stats.csv
echo profile done
