#!/bin/bash
# bench at several query-slot counts
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for s in ${SLOTS:-1 2 4 8}; do
  timeout -k 10 300 python $R/bench.py --steps 400 --warmup 5 --no-cpu-baseline --slots $s > $O/slots_$s.json 2> $O/slots_$s.err || { echo "slots $s failed"; tail -20 $O/slots_$s.err; exit 1; }
  python -c "import json;d=json.load(open('$O/slots_$s.json'));print('slots',$s,'qps',d['queries_per_sec'],'ms/q',d['ms_per_step'],'dev',d['device_ms_per_query'])"
done
