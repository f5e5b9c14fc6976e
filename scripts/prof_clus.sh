#!/bin/bash
# Kernel trace of the clustered config-2 rotation (bench's clustering line)
# with one query in flight; $TAG names the outputs.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
T=${TAG:-clus}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${T}_prof -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 1 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling ${BENCH_ARGS} > $O/${T}_prof.log 2>&1 || { echo "rocprof failed"; tail -30 $O/${T}_prof.log; exit 1; }
f=$(find $O/${T}_prof -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in rows[:22]: print('%-50s %6s %9.1f us  min %9.1f' % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1000, float(r['MinNs'])/1000))
"
