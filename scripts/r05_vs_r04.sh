#!/bin/bash
# round-4 code (bis/r04: a7c54c1's bench + library) against HEAD on one box,
# alternating; config-2 rotation and config 3
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05vs}
mkdir -p $O
F="--steps 400 --no-cpu-baseline --no-merge --no-ceiling --no-clustering --no-file-read"
run() {  # name dir
  (cd $2 && timeout -k 10 300 python3 $2/bench.py $F > $O/$1.json 2> $O/$1.err) || { echo "bench $1 failed"; tail -20 $O/$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$1.json'));print('$1', 'q/s', d['queries_per_sec'], 'c3', d['config3']['queries_per_sec'], d['config3']['phase_ms_mean'])"
}
run r04_a $R/bis/r04 && run head_a $R && run r04_b $R/bis/r04 && run head_b $R && run r04_c $R/bis/r04 && run head_c $R
