#!/bin/bash
# --config c4|c5 lines per library variant, alternated, each its own process
#   tools/r06_config_ab.sh <tag> <config> <rounds> <variant>...
set -o pipefail
TAG=$1; CFG=$2; R=$3; shift 3
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq 1 $R); do
  for v in "$@"; do
    RNSTOK_LIB=exp_ship/$v/librnstok.so timeout -k 10 300 python bench.py --config $CFG > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
    python3 - $O/${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ph = d.get("phases", {})
print("%-6s value %.4g  %s  ok %s" % (sys.argv[2], d["value"], {k: round(v.get("compute_ms", 0), 3) for k, v in ph.items()}, d.get("ok")))
PY
  done
done | tee $O/summary.txt
