#!/bin/bash
# Per-key decrypt with the round keys streamed from the key record
# (RNSTOK_PERKEY_STREAM = rounds ahead) vs the whole schedule in VGPRs (base5).
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
RNSTOK_LIB=build_exp/ps2/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_token_gpu.py tests/test_large_shapes_gpu.py tests/test_split_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
L="build_exp/base5/librnstok.so build_exp/ps1/librnstok.so build_exp/ps2/librnstok.so build_exp/ps3/librnstok.so build_exp/ps2w/librnstok.so"
for args in "--keys 65536" "--keys 65536 --ilv" "--keys 65536 --packed 64 --length 4096 --packets 524288" "--keys 65536 --length 1500"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py $L --rounds 16 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
for r in 1 2; do for v in base5 ps2 ps2w; do
  echo "== c5 share $v" >> $O/c5.txt
  RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 200 python tools/c5_share.py --steps 10 >> $O/c5.txt 2>&1 || { tail -20 $O/c5.txt; exit 1; }
done; done
grep -v amdgpu.ids $O/ab.txt | grep -v round-trip
python3 - <<'PY'
import json
for l in open("gpurun_out/r05c/c5.txt"):
    if l.startswith("=="): name = l.strip()
    elif l.startswith("{"):
        d = json.loads(l); print(name, {k: (v.get("ms") if isinstance(v, dict) else v) for k, v in d.items() if k in ("encrypt", "decrypt", "frac_of_valu_peak")})
PY
