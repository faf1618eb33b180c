#!/bin/bash
# k_encrypt_split wait probe (build_exp/splitprobe): per role, share of cycles polling the other role
set -o pipefail
O=gpurun_out/r04s
mkdir -p $O
for args in "" "--ilv" "--length 1500" "--keys 65536" "--length 100"; do
  RNSTOK_LIB=build_exp/splitprobe/librnstok.so timeout -k 10 120 python tools/split_wait_probe.py $args >> $O/split_wait.jsonl 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
done
cat $O/split_wait.jsonl
