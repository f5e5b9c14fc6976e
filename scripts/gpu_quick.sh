#!/bin/bash
# quick iteration: all GPU parity tests, then the config-2 bench line only
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python $R/bench.py --steps 400 --warmup 5 --no-cpu-baseline --no-merge --no-config3 ${BENCH_ARGS} > $O/quick.json 2> $O/quick.err || { echo "bench failed"; tail -20 $O/quick.err; exit 1; }
python -c "import json;d=json.load(open('$O/quick.json'));print('qps',d['queries_per_sec'],'GB/s',d['value'],'dev',d['device_ms_per_query'],d['phase_ms'],'probe',d['roofline']['achieved'])"
