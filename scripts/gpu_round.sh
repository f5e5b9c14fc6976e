#!/bin/bash
# GPU job: parity tests, bench, rocprofv3 kernel trace of the config-2 rotation.
# Each GPU step has its own time limit; the chain stops at the first failure.
# ($K: pytest -k filter, $BENCH_ARGS, $NOPROF=1 skips the profile)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/gpu_tests.log | head -20; tail -5 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 900 python $R/bench.py ${BENCH_ARGS:---steps 400 --warmup 5} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
[ -n "$NOPROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 64 --warmup 2 --no-cpu-baseline --no-config3 --no-merge --no-ceiling > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $O/prof.log; exit 1; }
find $O/prof -name "*stats*"
