#!/bin/bash
# iteration job: GPU parity tests, then bench per probe mode (0 full, 2 staging only)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for m in ${MODES:-0 2}; do
  GBGPU_PROBE_MODE=$m timeout -k 10 300 python $R/bench.py --steps 200 --warmup 5 --no-cpu-baseline > $O/probe_mode_$m.json 2> $O/probe_mode_$m.err || { echo "mode $m failed"; tail -20 $O/probe_mode_$m.err; exit 1; }
  python -c "import json;d=json.load(open('$O/probe_mode_$m.json'));print('mode',$m,'ms/q',d['ms_per_step'],d['phase_ms'],'probe GB/s',d['roofline']['achieved'])"
done
