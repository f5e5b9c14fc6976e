#!/bin/bash
# Round-3 baseline: GPU parity tests, the driver's bench command, a kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r03a_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/r03a_tests.log; exit 1; }
tail -2 $O/r03a_tests.log
timeout -k 10 500 python $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/r03a_bench.json 2> $O/r03a_bench.err || { echo "bench failed"; tail -30 $O/r03a_bench.err; exit 1; }
cat $O/r03a_bench.json
