#!/bin/bash
# PMC pass for k_probe under probe modes (counters only, no tracing)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in ${PMODES:-1 0}; do
  GBGPU_PROBE_MODE=$m timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM -d $O/pmcp$m -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --queries 2 --slots 1 --no-cpu-baseline --no-merge --no-config3 --no-ceiling > $O/pmcp$m.log 2>&1 || { echo "pmc mode $m failed"; tail -20 $O/pmcp$m.log; exit 1; }
  echo "mode $m ok"
done
