#!/bin/bash
# Round-4 profiles: HBM traffic passes (FETCH_SIZE / WRITE_SIZE, separate
# runs, counters only) of the config-2 rotation, a FETCH_SIZE pass of the
# probe's load-only mode (calibrates the 12-byte-lane reads), and kernel
# traces (stats) of config 2 and of the clustered rotation.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="--steps 48 --warmup 1 --queries 16 --slots 1 --no-cpu-baseline --no-merge --no-config3 --no-ceiling --no-clustering"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $R/bench.py $B > $O/fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $O/fetch.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $R/bench.py $B > $O/write.log 2>&1 || { echo "write pass failed"; tail -20 $O/write.log; exit 1; }
GBGPU_PROBE_MODE=9 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch9 -o run --output-format csv -- python3 $R/bench.py $B > $O/fetch9.log 2>&1 || { echo "fetch9 pass failed"; tail -20 $O/fetch9.log; exit 1; }
echo "pmc ok"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c2 -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering > $O/c2.log 2>&1 || { echo "c2 trace failed"; tail -20 $O/c2.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/clus -o run --output-format csv -- python3 $R/bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling > $O/clus.log 2>&1 || { echo "clus trace failed"; tail -20 $O/clus.log; exit 1; }
echo "traces ok"
