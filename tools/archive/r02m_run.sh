#!/bin/bash
set -e
bash tools/profile_cmd.sh gpurun_out/r02m_c4s8 - tools/bench_configs.py --config c4s8 --steps 10
echo all done
