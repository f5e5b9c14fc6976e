#!/bin/bash
# kernel trace of a short bench run (no tests)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $O/prof.log; exit 1; }
tail -1 $O/prof.log
