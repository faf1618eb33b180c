#!/bin/bash
# bench.node_rate (the composed interface path) per library
# variant, each its own process, alternated:  tools/r06_node_ab.sh <tag> <rounds> <variant>...
set -o pipefail
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq 1 $R); do
  for v in "$@"; do
    RNSTOK_LIB=exp_ship/$v/librnstok.so timeout -k 10 300 python -c "
import json, torch, bench
d = bench.node_rate(torch.device('cuda', 0), steps=15)
print(json.dumps({k: d[k] for k in ('outbound', 'inbound', 'ok') if k in d}))" > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
    python3 - $O/${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("%-6s outbound %.4f ms  inbound %.4f ms  ok %s" % (sys.argv[2], d["outbound"]["ms"], d["inbound"]["ms"], d.get("ok")))
PY
  done
done | tee $O/summary.txt
