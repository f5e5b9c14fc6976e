#!/bin/bash
# GPU job: parity tests, bench, rocprofv3 kernel trace.  Each GPU step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -m pytest $R/tests -m gpu -x -q > $R/gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/gpu_tests.log; exit 1; }
tail -3 $R/gpurun_out/gpu_tests.log
timeout -k 10 600 python $R/bench.py --steps 20 --warmup 3 > $R/gpurun_out/bench.json 2> $R/gpurun_out/bench.err || { echo "bench failed"; tail -30 $R/gpurun_out/bench.err; exit 1; }
cat $R/gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $R/gpurun_out/prof.log; exit 1; }
find $R/gpurun_out/prof -name "*stats*" | head
