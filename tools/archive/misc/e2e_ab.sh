#!/bin/bash
# PCIe-inclusive bench rows for the current build and tools/_ab/prev.so, alternated.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/e2e_ab.jsonl
for i in 1 2; do
  for lib in reticulum_amd/librnstok.so tools/_ab/prev.so; do
    [ -f "$lib" ] || continue
    RNSTOK_LIB=$PWD/$lib timeout -k 10 180 python -u bench.py --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/e2e_one.json 2>>gpurun_out/e2e_ab.err || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/e2e_one.json')); print(json.dumps({'lib':sys.argv[1],'value':d['value'],'e2e':d['e2e_pcie']}))" "$lib" | tee -a gpurun_out/e2e_ab.jsonl
  done
done
