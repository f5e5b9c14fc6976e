#!/bin/bash
# Round 6: the file_read leg (one at a time and 4 in flight) for each library
# in $LIBS (lib/<name>), config-2 part cut short
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06fr}
mkdir -p $O
cd $R
X="--steps 40 --warmup 2 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering"
for rep in 1 2; do
for L in ${LIBS}; do
  n=${L%.so}
  GBGPU_LIB=$L timeout -k 10 300 python3 bench.py $X > $O/f_$n.json 2> $O/f_$n.err || { echo "$L failed"; tail -20 $O/f_$n.err; exit 1; }
  python3 -c "import json;b=json.load(open('$O/f_$n.json'));print('$n', b['queries_per_sec'], b['file_read']['queries_per_sec'], b['file_read']['in_flight'], b.get('msg5_merge',{}).get('queries_per_sec'))"
done
done
