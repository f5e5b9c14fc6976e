#!/bin/bash
# kernel + copy traces of the config-3 leg (12 slots) for round-4 code
# (bis/r04) and HEAD
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05c3t}
mkdir -p $O
F="--steps 40 --warmup 2 --queries 4 --no-cpu-baseline --no-merge --no-ceiling --no-clustering --no-file-read"
cd /tmp && export TMPDIR=/tmp
(cd $R/bis/r04 && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/r04 -o run --output-format csv -- python3 $R/bis/r04/bench.py $F > $O/r04.json 2> $O/r04.err) || { echo "r04 failed"; tail -20 $O/r04.err; exit 1; }
(cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/head -o run --output-format csv -- python3 $R/bench.py $F > $O/head.json 2> $O/head.err) || { echo "head failed"; tail -20 $O/head.err; exit 1; }
python3 -c "
import json
for n in ('r04','head'):
    d=json.load(open('$O/'+n+'.json')); print(n, d['queries_per_sec'], d['config3']['queries_per_sec'])"
