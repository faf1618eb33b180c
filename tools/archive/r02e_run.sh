#!/bin/bash
# Round-2 profiles: c2 bench (trace + PMC), c4 per-GPU shard at 8 GPUs (long-token kernels), per-packet keying (fused HKDF + key setup).
set -e
bash tools/profile_cmd.sh gpurun_out/r02e_c2 1048576,500,1 bench.py --steps 30 --warmup 2 --cpu-seconds 0 --no-e2e
bash tools/profile_cmd.sh gpurun_out/r02e_c4s8 - tools/bench_configs.py --config c4s8 --steps 10
bash tools/profile_cmd.sh gpurun_out/r02e_ident - tools/bench_configs.py --config ident --steps 5
echo all done
