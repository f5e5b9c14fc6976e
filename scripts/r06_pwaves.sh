#!/bin/bash
# Round 6: probe spans (GBGPU_PROBE_WAVES, diagnostic build) vs config-2 probe
# time (one query in flight) and config-3 throughput
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06pw}
mkdir -p $O
cd $R
F="--steps 100 --warmup 2 --queries 8 --slots 1 --no-cpu-baseline --no-merge --no-ceiling --no-clustering --no-file-read"
for w in ${PWS:-3072 2048 4096 6144}; do
  GBGPU_DIAG=1 GBGPU_PROBE_WAVES=$w timeout -k 10 300 python3 bench.py $F > $O/w$w.json 2> $O/w$w.err || { echo "w $w failed"; tail -20 $O/w$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/w$w.json'));c=d['config3'];print('waves $w c2 probe', d['phase_ms']['probe'], 'c3 probe', c['phase_ms_mean']['probe'], 'c3 q/s(1 slot)', c['queries_per_sec'])"
done
