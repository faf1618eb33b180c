#!/bin/bash
# GPU tests, then the identity-keying config for the current build and
# tools/_ab/ksdirect.so (direct-store key setup), alternated.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/hkdf_tests.txt 2>&1 || { tail -30 gpurun_out/hkdf_tests.txt; exit 1; }
tail -2 gpurun_out/hkdf_tests.txt
: > gpurun_out/hkdf_ab.jsonl
for i in 1 2 3; do
  for lib in reticulum_amd/librnstok.so tools/_ab/ksdirect.so; do
    RNSTOK_LIB=$PWD/$lib timeout -k 10 120 python -u tools/bench_configs.py --config ident > gpurun_out/hkdf_one.json 2>>gpurun_out/hkdf_ab.err || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/hkdf_one.json').read().strip().splitlines()[-1]); print(json.dumps({'lib':sys.argv[1],'hkdf_ms':d['hkdf_ms'],'derive_keyset_ms':d['derive_keyset_ms'],'hkdf_shared_salt_ms':d['hkdf_shared_salt_ms'],'derive_keyset_shared_salt_ms':d['derive_keyset_shared_salt_ms'],'ok':d['ok']}))" "$lib" | tee -a gpurun_out/hkdf_ab.jsonl
  done
done
