#!/bin/bash
# kernel trace of the bench with the file-read leg (where a file cut's device time goes)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04fprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/t -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering > $O/b.json 2> $O/b.err || { echo "trace failed"; tail -20 $O/b.err; exit 1; }
ls $O/t
