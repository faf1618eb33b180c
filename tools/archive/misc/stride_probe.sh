set -o pipefail
for cfg in "0 0" "512 576" "512 640"; do set -- $cfg; timeout -k 10 200 python bench.py --cpu-seconds 0 --no-e2e --steps 30 --pt-stride $1 --tok-stride $2 > gpurun_out/stride_$1_$2.json 2>/dev/null || exit 1; done
bash tools/profile.sh s576 --pt-stride 512 --tok-stride 576 > gpurun_out/s576.log 2>&1 || exit 1
bash tools/profile.sh s640 --pt-stride 512 --tok-stride 640 > gpurun_out/s640.log 2>&1 || exit 1
for cfg in "0 0" "512 576" "512 640"; do set -- $cfg; timeout -k 10 200 python bench.py --cpu-seconds 0 --no-e2e --steps 30 --pt-stride $1 --tok-stride $2 > gpurun_out/stride2_$1_$2.json 2>/dev/null || exit 1; done
