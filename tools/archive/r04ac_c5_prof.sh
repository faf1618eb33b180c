#!/bin/bash
# c5 per-rank share on the round's final build: kernel trace + traffic/clock passes
set -o pipefail
O=gpurun_out/r04ac/c5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/c5_share.py > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
for PASS in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_ACTIVE_INST_VALU2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU"; do
  N=$(echo $PASS | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 200 rocprofv3 --pmc $PASS --output-format csv -d $O/pmc_$N -o run -- python3 tools/c5_share.py --steps 3 > $O/pmc_$N.log 2>&1 || { echo "pmc pass $N failed rc=$?"; tail -5 $O/pmc_$N.log; exit 1; }
done
python3 tools/pmc_summary.py $O --json $O/pmc.json > $O/pmc_summary.txt 2>&1
cp $O/trace/run_kernel_stats.csv $O/kernel_stats.csv
tail -1 $O/trace.log | cut -c1-400
grep -E "^[a-z_]|hbm_bytes_per_launch " $O/pmc_summary.txt | head -30
