#!/bin/bash
# diagnostic: k_tree_seq's clocks (time inside TopTree adds, the sequencer's
# share, the filter's) over the clustered config-2 rotation, diagnostic build
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06sq}
mkdir -p $O
GBGPU_DIAG=1 GBGPU_TOPK_DEBUG=1 timeout -k 10 300 python3 $R/bench.py --steps 4 --warmup 1 --queries 16 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-file-read > $O/sq.json 2> $O/sq.err || { tail -20 $O/sq.err; exit 1; }
grep "replay:" $O/sq.err | tail -8
