#!/bin/bash
# Trace timing vs lanes per ray at 100k and 1M rays (shared-stack groups), both scenes.
set -e
OUT=gpurun_out/${1:-bvh_lanes2}
mkdir -p $OUT
for sc in volume surface; do
  for R in 100000 1000000; do
    for L in 16 32 64; do
      R3DG_BVH_LANES=$L timeout -k 10 200 python tools/bench_bvh.py --rays $R --iters 3 --cpu-rays 100 --scene $sc --out $OUT/$sc.r$R.l$L.json > $OUT/$sc.r$R.l$L.log 2>&1
      python -c "import json; d=json.load(open('$OUT/$sc.r$R.l$L.json')); print('$sc rays=$R lanes=$L', round(d['trace_ms'],2))"
    done
  done
done
