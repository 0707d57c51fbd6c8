#!/bin/bash
# C4-size kernel stats per experiment build: bash tools/exp_prof_c4.sh NAME... (base = in-tree build)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in "$@"; do
  if [ "$n" = base ]; then d=""; else d=exp/$n/lib; fi
  R3DG_LIB_DIR=$d timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/expc4/$n -o run --output-format csv -- python bench.py --P 2000000 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/expc4/$n.log 2>&1
  echo "== $n"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/expc4/$n.log
done
