#!/bin/bash
# config-2 throughput vs queries in flight (bench --slots)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for s in ${SLOTS:-1 2 3 4}; do
  timeout -k 10 200 python3 $R/bench.py --steps 400 --warmup 8 --slots $s --no-cpu-baseline --no-config3 --no-merge --no-ceiling > $O/sl$s.json 2> $O/sl$s.err || { echo "slots $s failed"; tail -20 $O/sl$s.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/sl$s.json'));print('slots $s', d['queries_per_sec'], d['value'])"
done
