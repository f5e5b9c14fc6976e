#!/bin/bash
# Round 6: kernel stats of the clustered rotation with one query in flight
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06c1}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/clus1 -o run --output-format csv -- python3 $R/bench.py --steps 8 --warmup 1 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-file-read > $O/clus1.log 2>&1 || { echo "trace failed"; tail -20 $O/clus1.log; exit 1; }
python3 - "$O/clus1/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print('%-40s calls %5s avg %9.1f us' % (r['Name'].split('(')[0].replace('void ','').replace('gbgpu::','')[:40], r['Calls'], float(r['AverageNs'])/1000))
PY
