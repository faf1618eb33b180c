#!/bin/bash
# tools/one_packet_probe.py per library variant (exp_ship/<variant>/librnstok.so), R rounds
set -o pipefail
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq 1 $R); do
  for v in "$@"; do
    RNSTOK_LIB=exp_ship/$v/librnstok.so timeout -k 10 200 python tools/one_packet_probe.py > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
    echo "$v $(cat $O/${v}_$r.json)"
  done
done | tee $O/summary.txt
