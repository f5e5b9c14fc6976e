#!/bin/bash
# diagnostic: config-2 phase times with k_score stopped after each scorer phase
# (GBGPU_SCORE_MODE 1 mini-merge, 3 non-body pairs, 4 single terms, 5 window, 0 all)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for m in ${SMODES:-1 3 4 5 0}; do
  GBGPU_DIAG=1 GBGPU_SCORE_MODE=$m timeout -k 10 200 python3 $R/bench.py --steps 60 --warmup 4 --queries 4 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering --no-file-read > $O/sp$m.json 2> $O/sp$m.err || { echo "mode $m failed"; tail -20 $O/sp$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/sp$m.json'));print('mode $m', d['phase_ms'])"
done
