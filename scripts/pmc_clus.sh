#!/bin/bash
# SQ counters over the clustered config-2 rotation (one pass, counters only);
# $TAG names the outputs.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
T=${TAG:-pmcclus}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $O/${T}1 -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 1 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling > $O/${T}1.log 2>&1 || { echo "pass 1 failed"; tail -20 $O/${T}1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES -d $O/${T}2 -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 1 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling > $O/${T}2.log 2>&1 || { echo "pass 2 failed"; tail -20 $O/${T}2.log; exit 1; }
for f in $(find $O -path "*${T}*" -name "*counter_collection.csv"); do python3 $R/scripts/pmc_agg.py $f | grep -E "replay|k_bound|k_rep_sum|k_rank"; done
