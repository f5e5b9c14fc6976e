#!/bin/bash
# Iteration job: GPU parity tests (optional -k filter $K), a config-2 bench,
# and a kernel trace of the same bench.  Each GPU step has its own limit and
# the chain stops at the first failure.  $TAG names the outputs.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
T=${TAG:-it}
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -x -q --timeout 200 --timeout-method thread ${K:+-k "$K"} > $O/${T}_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $O/${T}_tests.log | head -20; tail -15 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 400 python $R/bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-config3 --no-merge ${BENCH_ARGS} > $O/${T}_bench.json 2> $O/${T}_bench.err || { echo "bench failed"; tail -30 $O/${T}_bench.err; exit 1; }
cat $O/${T}_bench.json
[ -n "$NOPROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${T}_prof -o run --output-format csv -- python3 $R/bench.py --steps 64 --warmup 2 --no-cpu-baseline --no-config3 --no-merge --no-ceiling > $O/${T}_prof.log 2>&1 || { echo "rocprof failed"; tail -30 $O/${T}_prof.log; exit 1; }
find $O/${T}_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -14 {}'
