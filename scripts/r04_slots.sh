#!/bin/bash
# queries in flight: the headline and the clustered rotation per slot count
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-slots}
mkdir -p $O
for s in ${SLOTS:-2 3 4}; do
  timeout -k 10 300 python3 $R/bench.py --steps ${STEPS:-300} --warmup 5 --slots $s --no-cpu-baseline --no-config3 --no-merge --no-ceiling > $O/s$s.json 2> $O/s$s.err || { echo "bench slots $s failed"; tail -20 $O/s$s.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/s$s.json'));print('slots $s q/s', d['queries_per_sec'], 'dev ms', d['device_ms_per_query'], 'clus q/s', d.get('clustering',{}).get('queries_per_sec'), d.get('clustering',{}).get('phase_ms'))"
done
