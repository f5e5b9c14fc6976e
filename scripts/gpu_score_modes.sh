#!/bin/bash
# diagnostic: kernel trace with the scorer on / off (GBGPU_SCORE_MODE)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for m in ${SMODES:-0 1}; do
  GBGPU_SCORE_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_s$m -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_s$m.log 2>&1 || { echo "mode $m failed"; tail -20 $O/prof_s$m.log; exit 1; }
done
