#!/bin/bash
# config-3 / file-read A/B over release libraries of earlier commits
# (scripts/bisect_libs.sh), each run twice, alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05bis}
mkdir -p $O
cd $R
for rep in 1 2; do
  for L in ${LIBS:-libgbgpu_bis_c23ef95.so libgbgpu_bis_22ce5db.so libgbgpu_bis_2109cd3.so default}; do
    E=""; [ "$L" != default ] && E="$L"
    GBGPU_LIB=$E timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --no-merge --no-ceiling --no-clustering > $O/$L.$rep.json 2> $O/$L.$rep.err || { echo "bench $L failed"; tail -20 $O/$L.$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$L.$rep.json'));print('$L', $rep, 'q/s', d['queries_per_sec'], 'c3', d['config3']['queries_per_sec'], 'fr', d['file_read']['queries_per_sec'], d['file_read'].get('in_flight'))"
  done
done
