#!/bin/bash
# Round 6 A/B: config-2 phase times (one query in flight) and 12-in-flight
# throughput for each library named in $LIBS (lib/<name>; "" = libgbgpu.so),
# then the GPU tests named by $K with the product library
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06ab}
mkdir -p $O
cd $R
X="--no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering --no-file-read"
for rep in 1 2; do
for L in ${LIBS:-libgbgpu_base.so libgbgpu.so}; do
  n=${L%.so}
  GBGPU_LIB=$L timeout -k 10 200 python3 bench.py --steps 100 --warmup 4 --queries 8 --slots 1 $X > $O/one_$n.json 2> $O/one_$n.err || { echo "$L one failed"; tail -20 $O/one_$n.err; exit 1; }
  GBGPU_LIB=$L timeout -k 10 200 python3 bench.py --steps ${STEPS:-400} $X > $O/tp_$n.json 2> $O/tp_$n.err || { echo "$L tp failed"; tail -20 $O/tp_$n.err; exit 1; }
  python3 -c "import json;a=json.load(open('$O/one_$n.json'));b=json.load(open('$O/tp_$n.json'));print('$n', 'phases', a['phase_ms'], 'q/s', b['queries_per_sec'])"
done
done
if [ -n "$K$ALLT" ]; then
  timeout -k 10 900 python -u -m pytest $R/tests -m gpu -q -x --timeout 200 --timeout-method thread ${K:+-k "$K"} > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED" $O/tests.log | head -30; exit 1; }
  tail -1 $O/tests.log
fi
