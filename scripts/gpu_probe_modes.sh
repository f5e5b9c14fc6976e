#!/bin/bash
# diagnostic: k_probe variants (full / classify-only / load-only)
R=$GRAFT_REPO_ROOT
for m in 0 1 2; do
  GBGPU_PROBE_MODE=$m timeout -k 10 300 python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/probe_mode_$m.json 2> $R/gpurun_out/probe_mode_$m.err || { echo "mode $m failed"; tail -20 $R/gpurun_out/probe_mode_$m.err; exit 1; }
  python -c "import json;d=json.load(open('$R/gpurun_out/probe_mode_$m.json'));print('mode',$m,d['phase_ms'],d['roofline']['achieved'])"
done
