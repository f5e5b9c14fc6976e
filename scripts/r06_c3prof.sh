#!/bin/bash
# Round 6: kernel statistics of the config-3 leg, one query in flight (the
# config-2 part cut to a few queries), and its FETCH_SIZE pass
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06c3}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
F="--steps 100 --warmup 1 --queries 2 --slots 1 --no-cpu-baseline --no-merge --no-ceiling --no-clustering --no-file-read"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py $F > $O/c3.json 2> $O/c3.err || { echo "trace failed"; tail -20 $O/c3.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c3.json'));print('c3', d['config3']['queries_per_sec'], d['config3']['phase_ms_mean'])"
[ -n "$NOPMC" ] && exit 0
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $R/bench.py $F > $O/fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $O/fetch.log; exit 1; }
echo pmc ok
