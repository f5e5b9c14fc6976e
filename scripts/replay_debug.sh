#!/bin/bash
# diagnostic: site-clustering replay counters (GBGPU_TOPK_DEBUG) over the clustered rotation
R=$GRAFT_REPO_ROOT
GBGPU_TOPK_DEBUG=1 timeout -k 10 300 python3 $R/bench.py --steps 4 --warmup 1 --queries 16 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling > $R/gpurun_out/rpd.json 2> $R/gpurun_out/rpd.err || { tail -20 $R/gpurun_out/rpd.err; exit 1; }
grep "replay:" $R/gpurun_out/rpd.err | tail -6
