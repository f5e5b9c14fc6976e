#!/bin/bash
# the GPU test suite (optional -k filter $K), then one config-2 bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05q}
mkdir -p $O
cd $R
timeout -k 10 ${TLIM:-900} python -u -m pytest $R/tests -m gpu -q -x --timeout 200 --timeout-method thread ${K:+-k "$K"} > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="--no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering --no-file-read"
timeout -k 10 300 python3 $R/bench.py --steps ${STEPS:-600} $B > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('q/s', d['queries_per_sec'], 'frac', d['roofline']['frac'], 'phases', d.get('phase_ms'))"
