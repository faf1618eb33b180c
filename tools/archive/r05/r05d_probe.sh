#!/bin/bash
# (1) Tail of the 768-thread decrypt at c2's 5.33 packets per lane: decrypt
#     time per packet at 5, 5.33 and 6 passes (983 040 / 1 048 576 / 1 179 648).
# (2) Why streamed per-key round keys lost (r05c): FETCH_SIZE of the c3
#     decrypt, schedule in VGPRs (base5) vs streamed 2 rounds ahead (ps2).
# (3) L2->fabric reads of the c2 kernels on rows vs interleaved: all requests
#     vs those destined for DRAM (Infinity-Cache hits are counted in FETCH_SIZE).
set -o pipefail
O=gpurun_out/r05d
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for n in 983040 1048576 1179648; do
  echo "== packets $n" >> $O/tail.txt
  timeout -k 10 200 python tools/exp_bench.py reticulum_amd/librnstok.so --rounds 16 --packets $n >> $O/tail.txt 2>&1 || { tail -20 $O/tail.txt; exit 1; }
done
grep -v amdgpu.ids $O/tail.txt | grep -v round-trip
for v in base5 ps2; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_perkey_$v -o run -- python3 tools/exp_bench.py build_exp/$v/librnstok.so --keys 65536 --rounds 2 > $O/pmc_perkey_$v.log 2>&1 || { tail -20 $O/pmc_perkey_$v.log; exit 1; }
done
for lay in rows interleaved; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d $O/pmc_dram_$lay -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --no-node --one-layout --layout $lay > $O/pmc_dram_$lay.json 2> $O/pmc_dram_$lay.err || { tail -20 $O/pmc_dram_$lay.err; exit 1; }
done
echo probes done
