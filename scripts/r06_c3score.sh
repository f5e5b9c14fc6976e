#!/bin/bash
# Round 6: config-3 score phase with k_score stopped after each part
# (diagnostic build, GBGPU_SCORE_MODE 1 mini-merge, 3 non-body pairs,
# 4 single terms, 5 sliding window, 0 all)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06c3s}
mkdir -p $O
cd $R
F="--steps 100 --warmup 1 --queries 2 --no-cpu-baseline --no-merge --no-ceiling --no-clustering --no-file-read"
for m in ${SMODES:-1 3 4 5 0}; do
  GBGPU_DIAG=1 GBGPU_SCORE_MODE=$m timeout -k 10 300 python3 bench.py $F > $O/m$m.json 2> $O/m$m.err || { echo "m $m failed"; tail -20 $O/m$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/m$m.json'));c=d['config3'];print('mode $m score', c['phase_ms_mean']['score'], 'c2 score', d['phase_ms']['score'])"
done
