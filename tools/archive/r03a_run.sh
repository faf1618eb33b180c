#!/bin/bash
# Round 3: the issue-model probe (tools/gen_issue_model_probe.py) timed, then two PMC passes over it.
set -o pipefail
O=gpurun_out/${TAG:-r03a}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 180 build_exp/issue_model_probe "" 2000 > $O/probe.txt 2>&1 || { echo probe failed; tail $O/probe.txt; exit 1; }
cat $O/probe.txt
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_IFETCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc1 -o run -- build_exp/issue_model_probe "" 500 > $O/pmc1.log 2>&1 || { echo pmc1 failed; tail $O/pmc1.log; exit 1; }
echo all ok
