#!/bin/bash
# k_score staging A/B: 4-unit aligned loads (default) vs load6 (GBGPU_SCORE_MODE=1024);
# parity suites that run k_score first, then a kernel trace of config 2 in each mode
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04sab}
mkdir -p $O
cd $R
[ -n "$NOTEST" ] || timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_golden.py tests/test_gpu_parity.py tests/test_fullsize.py tests/test_scoreinfo.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -5 $O/tests.log; exit 1; }
[ -n "$NOTEST" ] || tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
B="--steps 200 --warmup 5 ${SLOTS:+--slots $SLOTS} --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering --no-file-read"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/new -o run --output-format csv -- python3 $R/bench.py $B > $O/new.json 2> $O/new.err || { echo "new trace failed"; tail -20 $O/new.err; exit 1; }
GBGPU_SCORE_MODE=1024 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/old -o run --output-format csv -- python3 $R/bench.py $B > $O/old.json 2> $O/old.err || { echo "old trace failed"; tail -20 $O/old.err; exit 1; }
for m in new old; do f=$(find $O/$m -name "*kernel_stats.csv" | head -1); echo "== $m"; grep -E "k_score|k_probe" $f | cut -c1-160; done
