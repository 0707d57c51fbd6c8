#!/bin/bash
# Time experiment builds: bash tools/exp_run.sh NAME... (default build = "base"); kernel_ms per build.
set -e
mkdir -p gpurun_out/exp
for n in "$@"; do
  if [ "$n" = base ]; then d=""; else d=exp/$n/lib; fi
  R3DG_LIB_DIR=$d timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/exp/$n.json 2> gpurun_out/exp/$n.err
  python -c "import json,sys; d=json.load(open('gpurun_out/exp/$n.json')); print('$n', d['ms_per_step'], d['kernel_ms'])"
done
