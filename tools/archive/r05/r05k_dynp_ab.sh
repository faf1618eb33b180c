#!/bin/bash
# Split encrypt batches from a counter with the next index prefetched (sdynp),
# without the prefetch (dynall: + decrypt counter for whole passes), the
# prefetch alone on the product's counter batches (basep: c5's length-ordered
# half) and the round's product (base7).
set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
RNSTOK_LIB=build_exp/sdynp/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py tests/test_token_gpu.py tests/test_large_shapes_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests_sdynp.log 2>&1 || { tail -30 $O/tests_sdynp.log; exit 1; }
tail -1 $O/tests_sdynp.log
L="build_exp/base7/librnstok.so build_exp/basep/librnstok.so build_exp/sdynp/librnstok.so build_exp/dynall/librnstok.so"
for args in "--rounds 30" "--length 100" "--length 1000" "--packets 1500000" "--length 4096 --packets 262144" "--keys 65536" "--rounds 30"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py $L --rounds 20 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt | grep -v round-trip
grep "round-trip" $O/ab.txt | grep -c "ok=True tokens==variant0: True"
for r in 1 2; do for v in base7 basep sdynp; do
  echo "== c5 share $v" >> $O/c5.txt
  RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 200 python tools/c5_share.py --steps 10 >> $O/c5.txt 2>&1 || { tail -20 $O/c5.txt; exit 1; }
done; done
python3 - <<'PY'
import json
for l in open("gpurun_out/r05k/c5.txt"):
    if l.startswith("=="): name = l.strip()
    elif l.startswith("{"):
        d = json.loads(l); print(name, {k: (v.get("ms") if isinstance(v, dict) else v) for k, v in d.items() if k in ("encrypt", "decrypt", "frac_of_valu_peak")})
PY
