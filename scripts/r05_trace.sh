#!/bin/bash
# kernel trace (stats) of the config-2 rotation, one query in flight, for the
# release library and (AB=1) the A/B build
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05tr}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="--steps 100 --warmup 3 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering --no-file-read"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rel -o run --output-format csv -- python3 $R/bench.py $B > $O/rel.log 2>&1 || { echo "rel trace failed"; tail -20 $O/rel.log; exit 1; }
if [ -n "$AB" ]; then
GBGPU_LIB=alt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/alt -o run --output-format csv -- python3 $R/bench.py $B > $O/alt.log 2>&1 || { echo "alt trace failed"; tail -20 $O/alt.log; exit 1; }
fi
for f in $(find $O -name "*kernel_stats.csv"); do echo "== $f"; head -14 $f | cut -d, -f1-4; done
