#!/bin/bash
# Round-4 k_probe diagnosis: phase times per probe mode, then SQ counters of
# the full probe (one rocprofv3 --pmc pass, counters only).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04d
mkdir -p $O
for m in ${PMODES:-2 1 0}; do
  GBGPU_PROBE_MODE=$m timeout -k 10 200 python3 $R/bench.py --steps 60 --warmup 4 --queries 4 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering > $O/pm$m.json 2> $O/pm$m.err || { echo "mode $m failed"; tail -20 $O/pm$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/pm$m.json'));print('probe mode $m', d['phase_ms'], d['roofline'])"
done
[ -n "$NOPMC" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM -d $O/pmc -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --queries 2 --slots 1 --no-cpu-baseline --no-merge --no-config3 --no-ceiling --no-clustering > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
echo pmc ok
