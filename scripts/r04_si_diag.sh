#!/bin/bash
# which score-info fixtures decline on the GPU, and why (GBGPU_SI_DEBUG)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04s}
mkdir -p $O
cd $R
GBGPU_SI_DEBUG=1 timeout -k 10 300 python -u -m pytest $R/tests/test_scoreinfo.py -m gpu -q -s --timeout 200 --timeout-method thread > $O/si.log 2>&1 || { echo "si tests failed"; tail -30 $O/si.log; exit 1; }
grep -E "decline|declined|passed|failed" $O/si.log | tail -60
