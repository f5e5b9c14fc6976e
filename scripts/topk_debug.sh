#!/bin/bash
# diagnostic: k_topk phase clocks (GBGPU_TOPK_DEBUG, the diagnostic build)
# over a short config-2 run
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
GBGPU_DIAG=1 GBGPU_TOPK_DEBUG=1 timeout -k 10 200 python3 $R/bench.py --steps 20 --warmup 2 --queries 4 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering --no-file-read > $R/gpurun_out/tkd.json 2> $R/gpurun_out/tkd.err || { tail -20 $R/gpurun_out/tkd.err; exit 1; }
grep "topk us" $R/gpurun_out/tkd.err | tail -8
