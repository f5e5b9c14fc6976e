#!/bin/bash
# config-3 A/B: release vs alt build (GBGPU_DEFAULT_POOL=1 or GBGPU_LIST_MALLOC=1:
# the device pool or hipMalloc lists) and the slot count
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05c3}
mkdir -p $O
cd $R
run() {  # name lib slots
  GBGPU_LIB=$2 timeout -k 10 300 python3 $R/bench.py --steps 400 --slots $3 --no-cpu-baseline --no-merge --no-ceiling --no-clustering --no-file-read > $O/$1.json 2> $O/$1.err || { echo "bench $1 failed"; tail -20 $O/$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$1.json'));print('$1', 'q/s', d['queries_per_sec'], 'c3', d['config3']['queries_per_sec'])"
}
run rel_a "" 12 && run dpool_a alt 12 && run rel_b "" 12 && run dpool_b alt 12 && run rel_c "" 12 && run dpool_c alt 12
