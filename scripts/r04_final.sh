#!/bin/bash
# Round-4 record: the GPU test suite, smoke(), then the default bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04final}
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('q/s', d['queries_per_sec'], 'file_read', d.get('file_read',{}).get('queries_per_sec'), 'pcie', d.get('pcie_inclusive',{}).get('queries_per_sec'), 'GB/s', d['value'], 'frac', d['roofline']['frac'], 'clus', d['clustering']['queries_per_sec'], 'c3', d.get('config3',{}).get('queries_per_sec'), 'merge', d.get('config5_merge',{}).get('roofline',{}).get('frac'))"
