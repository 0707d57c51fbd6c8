#!/bin/bash
# BVH parity tests, then the trace timing at several lanes-per-ray settings.
set -e
OUT=gpurun_out/${1:-bvh_lanes}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_bvh.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest ok"
timeout -k 10 200 python tools/bench_bvh.py --iters 5 --cpu-rays 2000 --out $OUT/auto.json > $OUT/auto.log 2>&1
for L in 1 4 16 64; do
  R3DG_BVH_LANES=$L timeout -k 10 200 python tools/bench_bvh.py --iters 5 --cpu-rays 500 --out $OUT/lanes$L.json > $OUT/lanes$L.log 2>&1
done
for f in $OUT/*.json; do echo $f; python -c "import json,sys; d=json.load(open('$f')); print({k:round(v,3) for k,v in d.items() if k.startswith('trace') and 'ms' in k})"; done
