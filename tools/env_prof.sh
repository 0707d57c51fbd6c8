#!/bin/bash
# Kernel stats of the default bench under environment settings: bash tools/env_prof.sh TAG "VAR=val ..." ...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
i=0
for e in "$@"; do
  d=gpurun_out/envprof/$TAG/$i
  mkdir -p $d
  env $e timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $d/bench.log 2>&1 || { echo "run $i failed"; exit 1; }
  echo "== $i: $e"; grep -o '"ms_per_step": [0-9.]*' $d/bench.log
  i=$((i+1))
done
