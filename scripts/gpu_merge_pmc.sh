#!/bin/bash
# counters for the merge kernels: one rocprofv3 run per pass (counters only)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mprof -o run --output-format csv -- python3 $R/scripts/merge_time.py ${MERGE_KEYS:-100000000} 2 > $O/mprof.log 2>&1 || { echo "kernel trace failed"; tail -20 $O/mprof.log; exit 1; }
i=0
while IFS= read -r pass; do
  [ -z "$pass" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass -d $O/mpmc$i -o run --output-format csv -- python3 $R/scripts/merge_time.py ${MERGE_KEYS:-100000000} 1 > $O/mpmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $O/mpmc$i.log; exit 1; }
  echo "pass $i ok: $pass"
done < $R/scripts/merge_pmc.txt
