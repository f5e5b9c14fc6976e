#!/bin/bash
# Round 6: the GPU tests named by $K, then k_score's per-wave segments
# (score_waves.py, diagnostic build) and the score / probe phase modes
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06d}
mkdir -p $O
cd $R
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest $R/tests -m gpu -q -x --timeout 200 --timeout-method thread -k "$K" > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED" $O/tests.log | head -30; exit 1; }
  tail -1 $O/tests.log
fi
GBGPU_DIAG=1 GBGPU_SCORE_DUMP=$O/sdbg.bin timeout -k 10 300 python3 scripts/score_waves.py > $O/score_waves.txt 2>&1 || { echo "score_waves failed"; tail -20 $O/score_waves.txt; exit 1; }
cat $O/score_waves.txt | head -12
B="--steps 60 --warmup 4 --queries 4 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering --no-file-read"
for m in 1 0; do
  GBGPU_DIAG=1 GBGPU_SCORE_MODE=$m timeout -k 10 200 python3 bench.py $B > $O/sp$m.json 2> $O/sp$m.err || { echo "score mode $m failed"; tail -20 $O/sp$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/sp$m.json'));print('score mode $m', d['phase_ms'])"
done
for m in 9 8 5; do
  GBGPU_DIAG=1 GBGPU_PROBE_MODE=$m timeout -k 10 200 python3 bench.py $B > $O/pm$m.json 2> $O/pm$m.err || { echo "probe mode $m failed"; tail -20 $O/pm$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/pm$m.json'));print('probe mode $m', d['phase_ms'])"
done
