#!/bin/bash
# diagnostic: config-2 phase times with k_probe cut short (GBGPU_PROBE_MODE (diagnostic build)
# 9 chunk loads only, 8 + run-start compaction, 0 full)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for m in ${PMODES:-9 8 0}; do
  GBGPU_DIAG=1 GBGPU_PROBE_MODE=$m timeout -k 10 200 python3 $R/bench.py --steps 60 --warmup 4 --queries 4 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering --no-file-read > $O/pm$m.json 2> $O/pm$m.err || { echo "mode $m failed"; tail -20 $O/pm$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/pm$m.json'));print('probe mode $m', d['phase_ms'])"
done
