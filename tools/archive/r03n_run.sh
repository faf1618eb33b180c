#!/bin/bash
# Round 3, session 2: sanity of the restored tree (GPU suite, smoke, default
# bench line) and the PCIe ceiling by copy mechanism (tools/pcie_probe.hip:
# copy engines vs blit kernels vs zero-copy kernels, one and both directions).
set -o pipefail
O=gpurun_out/r03n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 tools/_bin/pcie_probe > $O/pcie_default.json 2>&1 || { echo probe failed; cat $O/pcie_default.json; exit 1; }
cat $O/pcie_default.json
HSA_ENABLE_SDMA=0 timeout -k 10 60 tools/_bin/pcie_probe > $O/pcie_nosdma.json 2>&1 || { echo probe nosdma failed; cat $O/pcie_nosdma.json; exit 1; }
cat $O/pcie_nosdma.json
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=10 > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
echo all ok
