#!/bin/bash
# Release libraries of earlier commits (same ABI as HEAD's binding) built into
# open-source-search-engine_amd/lib/libgbgpu_bis_<commit>.so, for bench.py
# GBGPU_LIB=libgbgpu_bis_<commit>.so A/B runs.
#   scripts/bisect_libs.sh COMMIT...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
for c in "$@"; do
  W=/tmp/bis_$c
  [ -d $W ] || git -C $R worktree add --detach $W $c >/dev/null
  make -C $W/open-source-search-engine_amd -j8 lib/libgbgpu.so >/dev/null
  cp $W/open-source-search-engine_amd/lib/libgbgpu.so $R/open-source-search-engine_amd/lib/libgbgpu_bis_$c.so
  echo "built libgbgpu_bis_$c.so"
done
