#!/bin/bash
# Round-5 record: the default bench line, then kernel traces (stats) of the
# config-2 rotation (one query in flight) and of the clustered rotation, then
# the HBM traffic passes (FETCH_SIZE / WRITE_SIZE, separate runs, counters only)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05prof}
mkdir -p $O
cd $R
timeout -k 10 900 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('q/s', d['queries_per_sec'], 'file_read', d.get('file_read',{}).get('queries_per_sec'), 'GB/s', d['value'], 'frac', d['roofline']['frac'], 'clus', d['clustering']['queries_per_sec'], 'c3', d.get('config3',{}).get('queries_per_sec'), 'merge', d.get('config5_merge',{}).get('roofline',{}).get('frac'))"
cd /tmp && export TMPDIR=/tmp
[ -n "$NOTRACE" ] && exit 0
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c2 -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 5 --slots 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-clustering --no-file-read > $O/c2.log 2>&1 || { echo "c2 trace failed"; tail -20 $O/c2.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/clus -o run --output-format csv -- python3 $R/bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-config3 --no-merge --no-ceiling --no-file-read > $O/clus.log 2>&1 || { echo "clus trace failed"; tail -20 $O/clus.log; exit 1; }
echo "traces ok"
[ -n "$NOPMC" ] && exit 0
B="--steps 48 --warmup 1 --queries 16 --slots 1 --no-cpu-baseline --no-merge --no-config3 --no-ceiling --no-clustering --no-file-read"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $R/bench.py $B > $O/fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $O/fetch.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $R/bench.py $B > $O/write.log 2>&1 || { echo "write pass failed"; tail -20 $O/write.log; exit 1; }
echo "pmc ok"
