set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/r01k_tests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r01k_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r01k_bench.json 2> gpurun_out/r01k_bench.err && \
bash tools/profile.sh r01k > gpurun_out/r01k_prof.log 2>&1 && \
for c in c3 c4 c4s8 c5 ident wire resource ratchet; do timeout -k 10 200 python tools/bench_configs.py --config $c >> gpurun_out/r01k_configs.jsonl 2>>gpurun_out/r01k_configs.err || exit 1; done
