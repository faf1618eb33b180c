#!/bin/bash
# Round 3, session 2: bench.py's N > 1 path after the host-origin change
# (D2H as GPU stores; e2e_pcie has a third leg), rehearsed on one GPU over
# gloo at 2 and 4 ranks, then the default line at N = 1.
set -o pipefail
O=gpurun_out/r03y; mkdir -p $O
export TMPDIR=/tmp
RNSTOK_BENCH_REHEARSE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-seconds 4 > $O/rehearse_n2.json 2> $O/rehearse_n2.err || { echo rehearse n2 failed; tail -30 $O/rehearse_n2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/rehearse_n2.json'));print(d['value'], json.dumps(d['e2e_pcie'].get('aggregate'))[:600]); print(json.dumps(d.get('sharded_c4'))[:300])"
RNSTOK_BENCH_REHEARSE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29642 bench.py --gpus 4 --steps 5 --warmup 2 --cpu-seconds 4 > $O/rehearse_n4.json 2> $O/rehearse_n4.err || { echo rehearse n4 failed; tail -30 $O/rehearse_n4.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/rehearse_n4.json'));print(d['value'], json.dumps(d['e2e_pcie'].get('aggregate'))[:600])"
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['roofline']['frac'], json.dumps(d['e2e_pcie']['pipelined']))"
echo all ok
