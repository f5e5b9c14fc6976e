#!/bin/bash
# resident-file read path: its tests, the golden suite (upload path refactor), a bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_file_read.py tests/test_golden.py > gpurun_out/fr_tests.log 2>&1 && tail -3 gpurun_out/fr_tests.log &&
timeout -k 10 400 python -u bench.py --no-config3 --no-merge --no-cpu-baseline > gpurun_out/fr_bench.json 2> gpurun_out/fr_bench.err &&
python -c "import json;r=json.load(open('gpurun_out/fr_bench.json'));print(r['value'],r['file_read'],r['pcie_inclusive'])"
