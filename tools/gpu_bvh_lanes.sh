#!/bin/bash
# BVH parity tests, then the 10k-ray trace at several lanes-per-ray settings, both scenes,
# shared-stack groups (default) and the static subtree split (R3DG_BVH_SPLIT=1).
set -e
OUT=gpurun_out/${1:-bvh_lanes}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_bvh.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest ok"
for sc in volume surface; do
  for L in 8 32 64; do
    for SP in 0 1; do
      R3DG_BVH_SPLIT=$SP R3DG_BVH_LANES=$L timeout -k 10 200 python tools/bench_bvh.py --rays 10000 --iters 5 --cpu-rays 100 --scene $sc --out $OUT/$sc.l$L.s$SP.json > $OUT/$sc.l$L.s$SP.log 2>&1
      python -c "import json; d=json.load(open('$OUT/$sc.l$L.s$SP.json')); print('$sc lanes=$L split=$SP', round(d['trace_10k_ms'],2))"
    done
  done
done
