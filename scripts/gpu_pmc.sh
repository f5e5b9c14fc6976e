#!/bin/bash
# PMC passes (one rocprofv3 run per pass, counters-only; no tracing domains)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
while IFS= read -r pass; do
  [ -z "$pass" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass -d $O/pmc$i -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $O/pmc$i.log; exit 1; }
  echo "pass $i ok: $pass"
done < ${PMC_FILE:-$R/scripts/pmc_passes.txt}
