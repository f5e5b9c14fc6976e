#!/bin/bash
# Round 6: the file_read leg with the upload stream at the greatest priority
# (default) and at the default priority (GBGPU_UPLOAD_PRIO=0), alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06prio}
mkdir -p $O
cd $R
X="--steps 40 --warmup 2 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering"
for rep in 1 2; do
for P in 1 0; do
  GBGPU_UPLOAD_PRIO=$P timeout -k 10 300 python3 bench.py $X > $O/p$P.json 2> $O/p$P.err || { echo "prio $P failed"; tail -20 $O/p$P.err; exit 1; }
  python3 -c "import json;b=json.load(open('$O/p$P.json'));print('prio $P', b['queries_per_sec'], b['file_read']['queries_per_sec'], b['file_read']['in_flight'], b.get('msg5_merge',{}).get('queries_per_sec'))"
done
done
