#!/bin/bash
# c5 rank share: kernel trace (bucketing passes vs token kernels) and the kernels' stamped clock, packed and slots
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 python tools/c5_share.py > $O/share.json 2> $O/share.err || exit 1
timeout -k 10 200 python tools/c5_share.py --align > $O/share_align.json 2> $O/share_align.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/c5_share.py > $O/trace.log 2>&1 || exit 1
cat $O/share.json $O/share_align.json
find $O/trace -name "*kernel_stats.csv" -exec cat {} \;
