#!/bin/bash
# iteration job: GPU parity tests, then bench (modes 0,1,2 for the probe)
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest $R/tests -m gpu -x -q > $R/gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $R/gpurun_out/gpu_tests.log; exit 1; }
tail -2 $R/gpurun_out/gpu_tests.log
for m in ${MODES:-0 1 2}; do
  GBGPU_PROBE_MODE=$m timeout -k 10 300 python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/probe_mode_$m.json 2> $R/gpurun_out/probe_mode_$m.err || { echo "mode $m failed"; tail -20 $R/gpurun_out/probe_mode_$m.err; exit 1; }
  python -c "import json;d=json.load(open('$R/gpurun_out/probe_mode_$m.json'));print('mode',$m,'ms/q',d['ms_per_step'],d['phase_ms'],'probe GB/s',d['roofline']['achieved'])"
done
