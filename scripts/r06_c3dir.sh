#!/bin/bash
# Round 6: config-3 throughput and phases against the probe-direction
# threshold (diagnostic build, GBGPU_PROBE_DIR_T) and probe waves
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06c3d}
mkdir -p $O
cd $R
F="--steps 200 --warmup 1 --queries 2 --no-cpu-baseline --no-merge --no-ceiling --no-clustering --no-file-read"
for t in ${DIRT:-64 16 32 128 512 100000}; do
  GBGPU_DIAG=1 GBGPU_PROBE_DIR_T=$t timeout -k 10 300 python3 bench.py $F > $O/t$t.json 2> $O/t$t.err || { echo "t $t failed"; tail -20 $O/t$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/t$t.json'));c=d['config3'];print('dir_t $t c3 q/s', c['queries_per_sec'], 'probe', c['phase_ms_mean']['probe'], 'dev', c['device_ms_per_query'])"
done
