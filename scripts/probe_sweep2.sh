#!/bin/bash
# diagnostic sweep: probe spans (GBGPU_PROBE_WAVES x GBGPU_PROBE_RUNSPAN),
# config-2 phase times with one query in flight
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for pw in ${PWS:-4096 3584 3072}; do
  for rs in ${RSS:-1 4}; do
    GBGPU_PROBE_WAVES=$pw GBGPU_PROBE_RUNSPAN=$rs timeout -k 10 200 python3 $R/bench.py --steps 100 --warmup 4 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling > $O/ps_${pw}_${rs}.json 2> $O/ps_${pw}_${rs}.err || { echo "sweep $pw $rs failed"; tail -20 $O/ps_${pw}_${rs}.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ps_${pw}_${rs}.json'));print('waves $pw runspan $rs', d['queries_per_sec'], d['phase_ms'])"
  done
done
