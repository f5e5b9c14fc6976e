#!/bin/bash
# merge (config 5) kernel trace: per-kernel averages for one full-size merge
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mprof -o m --output-format csv -- python3 $R/scripts/merge_time.py ${MERGE_KEYS:-400000000} 2 > $O/mprof.log 2>&1 || { echo "rocprof failed"; tail -30 $O/mprof.log; exit 1; }
tail -4 $O/mprof.log
find $O/mprof -name "*stats*"
