#!/bin/bash
# Round 6 A/B of the clustered rotation (Msg39's default request): clustered
# q/s (12 in flight) and device phases for each library in $LIBS, then
# k_tree_seq's clocks (diagnostic build), then the GPU tests ($K / $ALLT)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06cl}
mkdir -p $O
cd $R
X="--no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-file-read"
for rep in 1 2; do
for L in ${LIBS:-libgbgpu_base.so libgbgpu.so}; do
  n=${L%.so}
  GBGPU_LIB=$L timeout -k 10 300 python3 bench.py --steps ${STEPS:-60} --warmup 2 $X > $O/cl_$n.json 2> $O/cl_$n.err || { echo "$L failed"; tail -20 $O/cl_$n.err; exit 1; }
  python3 -c "import json;b=json.load(open('$O/cl_$n.json'))['clustering'];print('$n', 'clus q/s', b['queries_per_sec'], 'dev ms', b.get('device_ms_per_query'), b.get('phase_ms'))"
done
done
TAG=${TAG:-r06cl} bash $R/scripts/r06_seqdbg.sh || exit 1
if [ -n "$K$ALLT" ]; then
  timeout -k 10 900 python -u -m pytest $R/tests -m gpu -q -x --timeout 200 --timeout-method thread ${K:+-k "$K"} > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED" $O/tests.log | head -30; exit 1; }
  tail -1 $O/tests.log
fi
