#!/bin/bash
# Iteration job: GPU parity tests (optional -k filter $K), a config-2 bench
# (2 queries in flight), and a kernel trace with ONE query in flight (kernel
# durations without the other slot's overlap).  Each GPU step has its own
# limit; the chain stops at the first failure.  $TAG names the outputs.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
T=${TAG:-it}
mkdir -p $O
cd $R
if [ -z "$NOTEST" ]; then
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -x -q --timeout 200 --timeout-method thread ${K:+-k "$K"} > $O/${T}_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $O/${T}_tests.log | head -20; tail -15 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
fi
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 400 python $R/bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-config3 --no-merge ${BENCH_ARGS} > $O/${T}_bench.json 2> $O/${T}_bench.err || { echo "bench failed"; tail -30 $O/${T}_bench.err; exit 1; }
cat $O/${T}_bench.json
[ -n "$NOPROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${T}_prof -o run --output-format csv -- python3 $R/bench.py --steps 64 --warmup 2 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering ${BENCH_ARGS} > $O/${T}_prof.log 2>&1 || { echo "rocprof failed"; tail -30 $O/${T}_prof.log; exit 1; }
f=$(find $O/${T}_prof -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in rows[:22]: print('%-50s %6s %9.1f us  min %9.1f' % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1000, float(r['MinNs'])/1000))
"
