#!/bin/bash
# Round 3, session 3 evidence on the tree with the device-side inbound glue:
# smoke, the default bench line (node_pipeline inbound now on rt_frames_compact
# / rt_token_spans), and the C-host test.
set -o pipefail
O=gpurun_out/r03aq; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['roofline']['frac'], d['kernels']['encrypt']['ms'], d['kernels']['decrypt']['ms'], json.dumps(d.get('node_pipeline'))[:400])"
