#!/bin/bash
# Issue-slot accounting of the wire kernels (tools/bench_configs.py --config
# wire): kernel trace, then instruction / dual-issue / clock / HBM passes, one
# counter group per run.  Summary per kernel (template argument kept, so IFAC
# mask and unmask stay apart): tools/archive/r03am_wire_pmc_summary.py.
set -o pipefail
O=gpurun_out/r03am; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_configs.py --config wire --steps 5 > $O/trace.log 2>&1 || { echo trace failed; tail -5 $O/trace.log; exit 1; }
for PASS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU2 SQ_BUSY_CYCLES" \
            "GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  N=$(echo $PASS | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $PASS --output-format csv -d $O/pmc_$N -o run -- python3 tools/bench_configs.py --config wire --steps 5 > $O/pmc_$N.log 2>&1 || { echo "pmc pass $N failed"; tail -5 $O/pmc_$N.log; exit 1; }
done
python3 tools/archive/r03am_wire_pmc_summary.py $O > $O/summary.txt && cat $O/summary.txt
