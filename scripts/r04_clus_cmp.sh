#!/bin/bash
# clustered q/s: the bench's line at two lengths vs the host-timing script
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-cc}
mkdir -p $O
for st in 300 1200; do
  timeout -k 10 300 python3 $R/bench.py --steps $st --warmup 5 --no-cpu-baseline --no-config3 --no-merge --no-ceiling > $O/b$st.json 2> $O/b$st.err || { echo "bench failed"; tail -20 $O/b$st.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$st.json'));print('steps $st q/s', d['queries_per_sec'], 'clus', d['clustering']['queries_per_sec'], d['clustering']['queries'])"
done
HWQ=16 NQ=16 NQUERY=150 CLUS=1 SLOTS="8" timeout -k 10 300 python3 $R/scripts/r04_clus_host.py
