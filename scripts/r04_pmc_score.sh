#!/bin/bash
# k_score SQ counters (one --pmc pass per mode, counters only): full, and
# GBGPU_SCORE_MODE=1 (mini-merge only)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04ps}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="--steps 8 --warmup 1 --queries 4 --slots 1 --no-cpu-baseline --no-merge --no-config3 --no-ceiling --no-clustering"
for m in 0 1; do
  GBGPU_SCORE_MODE=$m timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM -d $O/s$m -o run --output-format csv -- python3 $R/bench.py $B > $O/s$m.log 2>&1 || { echo "pmc s$m failed"; tail -20 $O/s$m.log; exit 1; }
done
echo ok
