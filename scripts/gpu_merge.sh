#!/bin/bash
# merge (config 5) job: GPU parity tests, then a timing probe
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests/test_merge.py ${MERGE_FULL:+$R/tests/test_fullsize.py} -m gpu ${K:+-k "$K"} -x -v --timeout 120 --timeout-method thread > $O/merge_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/merge_tests.log; exit 1; }
tail -3 $O/merge_tests.log
timeout -k 10 300 python -u $R/scripts/merge_time.py ${MERGE_KEYS:-400000000} > $O/merge_time.log 2>&1 || { echo "timing failed"; tail -30 $O/merge_time.log; exit 1; }
cat $O/merge_time.log
exit 0
