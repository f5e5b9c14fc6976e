#!/bin/bash
# Round 5: the GPU test suite (optional -k filter in $K), then smoke()
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05t}
mkdir -p $O
cd $R
timeout -k 10 ${TLIM:-900} python -u -m pytest $R/tests -m gpu -q --timeout 200 --timeout-method thread ${K:+-k "$K"} > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
