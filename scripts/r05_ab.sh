#!/bin/bash
# A/B: the release library against lib/libgbgpu_alt.so (Makefile `alt`) on the
# config-2 rotation: q/s at 12 queries in flight, and the one-query phase times
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05ab}
mkdir -p $O
cd $R
B="--no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering --no-file-read"
for rep in 1 2; do
for lib in rel alt; do
  GBGPU_LIB=$lib timeout -k 10 300 python3 $R/bench.py --steps ${STEPS:-600} $B > $O/$lib$rep.json 2> $O/$lib$rep.err || { echo "$lib failed"; tail -20 $O/$lib$rep.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$lib$rep.json'));print('$lib', 'q/s', d['queries_per_sec'], 'phases', d.get('phase_ms'))"
done
done
