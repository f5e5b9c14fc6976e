#!/bin/bash
# probe parity tests, phase times, and the k_probe FETCH_SIZE pass
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04pt}
mkdir -p $O
K="probe or golden or config2" PWAVES="${PWAVES:-3072 4096}" TAG=${TAG:-r04pt} bash $R/scripts/r04_probe_iter.sh || exit 1
cd /tmp && export TMPDIR=/tmp
B="--steps 48 --warmup 1 --queries 16 --slots 1 --no-cpu-baseline --no-merge --no-config3 --no-ceiling --no-clustering"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $R/bench.py $B > $O/fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $O/fetch.log; exit 1; }
python3 - <<PY
import csv,collections
tot=collections.defaultdict(float); disp=collections.defaultdict(set)
for r in csv.DictReader(open('$O/fetch/run_counter_collection.csv')):
    k=r['Kernel_Name'].split('(')[0]
    if 'probe' in k: tot[k]+=float(r['Counter_Value']); disp[k].add(r['Dispatch_Id'])
for k in tot: print(k, 'fetch x2', round(2*tot[k]/len(disp[k])*1024/1e6,1), 'MB per launch')
PY
