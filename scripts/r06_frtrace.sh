#!/bin/bash
# Round 6: kernel traces of the file_read leg for two libraries ($LIBS)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06frt}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
X="--steps 20 --warmup 1 --queries 2 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering"
for L in ${LIBS}; do
  n=${L%.so}
  GBGPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace -d $O/$n -o run --output-format csv -- python3 $R/bench.py $X > $O/$n.json 2> $O/$n.err || { echo "$L failed"; tail -20 $O/$n.err; exit 1; }
  python3 -c "import json;b=json.load(open('$O/$n.json'));print('$n', b['file_read']['queries_per_sec'], b['file_read']['in_flight'])"
done
