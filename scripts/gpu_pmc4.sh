#!/bin/bash
# PMC passes over a short config-2 bench with ONE query in flight (one
# rocprofv3 run per pass, counters only, no tracing domains); $TAG names
# the outputs, scripts/pmc_agg.py summarises them per kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
T=${TAG:-pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
while IFS= read -r pass; do
  [ -z "$pass" ] && continue
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pass -d $O/${T}$i -o run --output-format csv -- python3 $R/bench.py --steps 16 --warmup 1 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering ${BENCH_ARGS} > $O/${T}$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $O/${T}$i.log; exit 1; }
  echo "pass $i ok: $pass"
done < ${PMC_FILE:-$R/scripts/pmc_passes_r03.txt}
for f in $(find $O -path "*${T}*" -name "*counter_collection.csv"); do python3 $R/scripts/pmc_agg.py $f | head -14; done
