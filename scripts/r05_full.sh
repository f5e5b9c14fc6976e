#!/bin/bash
# the whole GPU suite, then the default bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05full}
mkdir -p $O
cd $R
timeout -k 10 ${TLIM:-1000} python -u -m pytest $R/tests -m gpu -q -x --timeout 200 --timeout-method thread ${K:+-k "$K"} > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -2 $O/tests.log
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 900 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('q/s', d['queries_per_sec'], 'GB/s', d['value'], 'frac', d['roofline']['frac'], 'clus', d['clustering']['queries_per_sec'], 'c3', d['config3']['queries_per_sec'], 'fr', d['file_read'], 'merge', d['config5_merge']['roofline']['frac'])"
