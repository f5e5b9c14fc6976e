#!/bin/bash
# the GPU tests of list uploads and file cuts, then the bench's file_read leg
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05fr}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -q -x --timeout 200 --timeout-method thread -k "file or upload or golden or corrupt or msg5 or release" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python3 $R/bench.py --steps 200 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('q/s', d['queries_per_sec'], 'file_read', d.get('file_read'))"
