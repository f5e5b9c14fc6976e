#!/bin/bash
# Round 6 A/B of the config-5 merge: ms per merge and phases for each library
# in $LIBS (lib/<name>), the config-2 part cut to a few steps
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06mab}
mkdir -p $O
cd $R
X="--steps 10 --warmup 1 --queries 2 --slots 1 --no-cpu-baseline --no-config3 --no-ceiling --no-clustering --no-file-read"
for rep in 1 2; do
for L in ${LIBS:-libgbgpu.so libgbgpu_t1024.so libgbgpu_t2048.so}; do
  n=${L%.so}
  GBGPU_LIB=$L timeout -k 10 300 python3 bench.py $X > $O/m_$n.json 2> $O/m_$n.err || { echo "$L failed"; tail -20 $O/m_$n.err; exit 1; }
  python3 -c "import json;b=json.load(open('$O/m_$n.json'))['config5_merge'];print('$n', b['ms_per_merge'], b['phase_ms'], b['tiles'])"
done
done
