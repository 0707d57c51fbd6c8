#!/bin/bash
# Time BVH experiment builds: bash tools/exp_bvh.sh NAME... (base = default build), both scenes.
set -e
mkdir -p gpurun_out/expbvh
for n in "$@"; do
  if [ "$n" = base ]; then d=""; else d=exp/$n/lib; fi
  for sc in volume surface; do
    R3DG_LIB_DIR=$d timeout -k 10 200 python tools/bench_bvh.py --iters 5 --cpu-rays 200 --scene $sc --out gpurun_out/expbvh/$n.$sc.json > gpurun_out/expbvh/$n.$sc.log 2>&1
    python -c "import json; d=json.load(open('gpurun_out/expbvh/$n.$sc.json')); print('$n $sc', round(d['trace_ms'],2), round(d['trace_10k_ms'],2))"
  done
done
