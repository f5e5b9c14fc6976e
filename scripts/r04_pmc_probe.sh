#!/bin/bash
# k_probe SQ counters (one --pmc pass each, counters only): the default
# candidate path and GBGPU_PROBE_MODE=$ALT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04p}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="--steps 3 --warmup 1 --queries 2 --slots 1 --no-cpu-baseline --no-merge --no-config3 --no-ceiling --no-clustering"
for m in 0 ${ALT:-4}; do
  GBGPU_PROBE_MODE=$m timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU -d $O/a$m -o run --output-format csv -- python3 $R/bench.py $B > $O/a$m.log 2>&1 || { echo "pmc a$m failed"; tail -20 $O/a$m.log; exit 1; }
  GBGPU_PROBE_MODE=$m timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS GRBM_GUI_ACTIVE -d $O/b$m -o run --output-format csv -- python3 $R/bench.py $B > $O/b$m.log 2>&1 || { echo "pmc b$m failed"; tail -20 $O/b$m.log; exit 1; }
  echo "mode $m ok"
done
