#!/bin/bash
# kernel trace of the config-2 rotation only (short); summary to gpurun_out/prof
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 32 --warmup 2 --queries ${Q:-4} --slots ${SL:-2} --no-cpu-baseline --no-config3 --no-merge --no-ceiling > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows[:25]: print('%-60s %8s %10.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1000))
"
