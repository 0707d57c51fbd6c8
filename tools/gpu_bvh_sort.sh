#!/bin/bash
# BVH parity tests, then trace timing with / without the Morton ray sort (R3DG_BVH_SORT), both scenes.
set -e
OUT=gpurun_out/${1:-bvh_sort}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_bvh.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest ok"
for sc in volume surface; do
  for S in 0 1; do
    R3DG_BVH_SORT=$S timeout -k 10 200 python tools/bench_bvh.py --iters 5 --cpu-rays 100 --scene $sc --out $OUT/$sc.s$S.json > $OUT/$sc.s$S.log 2>&1
    python -c "import json; d=json.load(open('$OUT/$sc.s$S.json')); print('$sc sort=$S', round(d['trace_ms'],2), round(d['trace_10k_ms'],3))"
  done
done
