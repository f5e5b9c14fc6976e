#!/bin/bash
# FETCH_SIZE of the probe's load-only mode (calibration of the 12-byte-lane
# reads: every loaded word used) and the config-2 kernel trace, one query in flight
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="--steps 48 --warmup 1 --queries 16 --slots 1 --no-cpu-baseline --no-merge --no-config3 --no-ceiling --no-clustering"
GBGPU_PROBE_MODE=9 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch9b -o run --output-format csv -- python3 $R/bench.py $B > $O/fetch9b.log 2>&1 || { echo "fetch9 pass failed"; tail -20 $O/fetch9b.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c2s1 -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 5 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering > $O/c2s1.log 2>&1 || { echo "c2 trace failed"; tail -20 $O/c2s1.log; exit 1; }
echo ok
