#!/bin/bash
# Round 6: queries in flight (slots) vs throughput with the runtime's default
# hardware queues, unclustered and clustered, twice each
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06s2}
mkdir -p $O
cd $R
for rep in 1 2; do
for s in ${SLOTS:-12 16 20 24}; do
  timeout -k 10 300 python3 bench.py --slots $s --steps 800 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-file-read > $O/s$s.json 2> $O/s$s.err || { echo "slots $s failed"; tail -20 $O/s$s.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/s$s.json'));print('slots $s q/s', d['queries_per_sec'], 'clus', d['clustering']['queries_per_sec'])"
done
done
