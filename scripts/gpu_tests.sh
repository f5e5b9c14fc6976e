#!/bin/bash
# GPU job: parity tests only (optional -k filter in $K)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread ${K:+-k "$K"} > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
