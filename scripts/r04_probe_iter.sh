#!/bin/bash
# Round-4 probe iteration: GPU parity tests (optional -k $K), then config-2
# probe phase times at several span counts (GBGPU_PROBE_WAVES)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04i}
mkdir -p $O
cd $R
if [ -z "$NOTEST" ]; then
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -x -q --timeout 200 --timeout-method thread ${K:+-k "$K"} > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $O/tests.log | head -20; tail -15 $O/tests.log; exit 1; }
tail -2 $O/tests.log
fi
for pw in ${PWAVES:-4096}; do
  GBGPU_PROBE_WAVES=$pw timeout -k 10 200 python3 $R/bench.py --steps 100 --warmup 4 --queries 8 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering > $O/pw$pw.json 2> $O/pw$pw.err || { echo "bench $pw failed"; tail -20 $O/pw$pw.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/pw$pw.json'));print('waves $pw', d['phase_ms'], 'probe frac', d['roofline']['frac'], 'q/s', d['queries_per_sec'])"
done
