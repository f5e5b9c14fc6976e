#!/bin/bash
# merge tile-kernel phase costs: GBGPU_MERGE_MODE 1 decode, 2 + compaction,
# 3 + merge rounds, 0 full (timings only; outputs of modes 1-3 are not merges)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for m in 1 2 3 0; do
  GBGPU_MERGE_PATH=tiles GBGPU_MERGE_MODE=$m timeout -k 10 200 python -u $R/scripts/merge_time.py ${MERGE_KEYS:-400000000} 2 > $O/merge_mode$m.log 2>&1 || { echo "mode $m failed"; tail -20 $O/merge_mode$m.log; exit 1; }
  echo "mode $m: $(tail -1 $O/merge_mode$m.log)"
done
