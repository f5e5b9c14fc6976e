#!/bin/bash
# Round 6: config-2 throughput (12 queries in flight) against the HIP
# runtime's hardware queues per process (GPU_MAX_HW_QUEUES; 4 by default)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06hwq}
mkdir -p $O
cd $R
X="--steps 400 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-file-read"
for rep in 1 2; do
for Q in ${QS:-4 8 12 16}; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python3 bench.py $X > $O/q$Q.json 2> $O/q$Q.err || { echo "Q=$Q failed"; tail -20 $O/q$Q.err; exit 1; }
  python3 -c "import json;b=json.load(open('$O/q$Q.json'));print('hwq $Q', b['queries_per_sec'], 'clus', b['clustering']['queries_per_sec'])"
done
done
