#!/bin/bash
# N > 1 control-flow rehearsal of the default bench over gloo with every rank on
# the one GPU (RNSTOK_BENCH_REHEARSE=1; not a measurement): N = 4 and N = 8
set -o pipefail
O=gpurun_out/r06_rehearse
mkdir -p $O
for N in 4 8; do
  RNSTOK_BENCH_REHEARSE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29700 + N)) bench.py --gpus $N --steps 5 --warmup 2 --cpu-seconds 2 \
    > $O/n$N.json 2> $O/n$N.err || { echo "rehearse n$N failed"; tail -30 $O/n$N.err; exit 1; }
  python3 - $O/n$N.json $N <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d.get("sharded_c4") or {}
print("N=%s value %.4g n_gpus %s sharded_c4 ok %s err %s e2e_aggregate %s" % (sys.argv[2], d["value"], d["n_gpus"],
      s.get("ok"), s.get("error"), bool((d.get("e2e_pcie") or {}).get("aggregate"))))
PY
done
