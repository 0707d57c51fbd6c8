#!/bin/bash
# One GPU call: A/B of backward variants (R3DG_BWD values) on the M1 bench, after the backward parity
# tests under each variant. Usage: bash tools/gpu_ab.sh TAG VARIANT...  ("-" = default variant)
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for v in "$@"; do
  if [ "$v" = "-" ]; then unset R3DG_BWD; else export R3DG_BWD=$v; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "backward" > $OUT/pytest_$v.log 2>&1
  echo "pytest $v ok: $(tail -1 $OUT/pytest_$v.log)"
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_$v.json 2> $OUT/bench_$v.err
  python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('$v', d['ms_per_step'], d['kernel_ms'])"
done
