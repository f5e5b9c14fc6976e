#!/bin/bash
# Round 6: SQ counters of the config-2 kernels at HEAD (release library), two
# --pmc passes (counters only, each its own run), one query in flight
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06sqc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="--steps 6 --warmup 1 --queries 4 --slots 1 --no-cpu-baseline --no-merge --no-config3 --no-ceiling --no-clustering --no-file-read"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU -d $O/a -o run --output-format csv -- python3 $R/bench.py $B > $O/a.log 2>&1 || { echo "pmc a failed"; tail -20 $O/a.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS GRBM_GUI_ACTIVE -d $O/b -o run --output-format csv -- python3 $R/bench.py $B > $O/b.log 2>&1 || { echo "pmc b failed"; tail -20 $O/b.log; exit 1; }
python3 $R/scripts/pmc_agg.py $O/a/run_counter_collection.csv $O/b/run_counter_collection.csv | head -30
