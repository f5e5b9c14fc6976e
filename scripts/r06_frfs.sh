#!/bin/bash
# Round 6: the file_read leg's queries in flight (GBGPU_FR_INFLIGHT) swept
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06frfs}
mkdir -p $O
cd $R
X="--steps 40 --warmup 2 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering"
for rep in 1 2; do
for F in 1 2 4 8 12; do
  GBGPU_FR_INFLIGHT=$F timeout -k 10 300 python3 bench.py $X > $O/f$F.json 2> $O/f$F.err || { echo "fs $F failed"; tail -20 $O/f$F.err; exit 1; }
  python3 -c "import json;b=json.load(open('$O/f$F.json'));print('fs $F', b['queries_per_sec'], b['file_read']['queries_per_sec'], b['file_read']['in_flight'])"
done
done
