#!/bin/bash
# diagnostic: config-2 bench phases with k_probe split into GBGPU_PROBE_WAVES spans
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for w in ${PWS:-2048 4096 8192 16384}; do
  GBGPU_PROBE_WAVES=$w timeout -k 10 200 python3 $R/bench.py --steps 200 --warmup 4 --no-cpu-baseline --no-config3 --no-merge --no-ceiling > $O/pw$w.json 2> $O/pw$w.err || { echo "waves $w failed"; tail -20 $O/pw$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/pw$w.json'));print('waves $w', d['queries_per_sec'], d['phase_ms'], d['roofline']['frac'])"
done
