#!/bin/bash
# Round-4 iteration: GPU tests, config-2 probe timing per span count, one
# full bench line (clustering included), score-info decline diagnostics
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${TAG:-r04r}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $O/tests.log | head -20; tail -15 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for pw in ${PWAVES:-4096}; do
  GBGPU_PROBE_WAVES=$pw timeout -k 10 200 python3 $R/bench.py --steps 100 --warmup 4 --queries 8 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering > $O/pw$pw.json 2> $O/pw$pw.err || { echo "bench $pw failed"; tail -20 $O/pw$pw.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/pw$pw.json'));print('waves $pw', d['phase_ms'], 'probe frac', d['roofline']['frac'], 'q/s', d['queries_per_sec'])"
done
timeout -k 10 400 python3 $R/bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-config3 --no-merge > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('q/s', d['queries_per_sec'], 'dev ms', d['device_ms_per_query'], d['phase_ms'], 'frac', d['roofline']['frac'], 'clus', d.get('clustering',{}).get('queries_per_sec'), d.get('clustering',{}).get('phase_ms'))"
GBGPU_SI_DEBUG=1 timeout -k 10 300 python -u -m pytest $R/tests/test_scoreinfo.py -m gpu -q -s --timeout 200 --timeout-method thread > $O/si.log 2>&1 || { echo "si tests failed"; tail -30 $O/si.log; exit 1; }
grep -E "decline|declined|passed|failed" $O/si.log | tail -60
