#!/bin/bash
# derive_keyset timing for the current build (KS_P = 9) and KS_P variants under tools/_ab, alternated.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ks_ab.jsonl
for i in 1 2; do
  for lib in reticulum_amd/librnstok.so tools/_ab/*.so; do
    RNSTOK_LIB=$PWD/$lib timeout -k 10 120 python -u tools/bench_configs.py --config ident > gpurun_out/ks_one.json 2>>gpurun_out/ks_ab.err || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/ks_one.json').read().strip().splitlines()[-1]); print(json.dumps({'lib':sys.argv[1],'derive_keyset_ms':d['derive_keyset_ms'],'derive_keyset_shared_salt_ms':d['derive_keyset_shared_salt_ms'],'ok':d['ok']}))" "$lib" | tee -a gpurun_out/ks_ab.jsonl
  done
done
