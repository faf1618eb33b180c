set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06ar
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r06ar/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/single_call_latency.py --calls 500 --length 383 > $GRAFT_REPO_ROOT/gpurun_out/r06ar/lat.json 2> $GRAFT_REPO_ROOT/gpurun_out/r06ar/lat.err
