#!/bin/bash
# One GPU call: bench A/B over (variant, lib dir) pairs: bash tools/gpu_ab2.sh TAG VARIANT:LIBDIR ...
# VARIANT "-" = default backward ("dpp" = the DPP cross-check), LIBDIR "-" = in-tree lib. Backward
# parity tests run per pair.
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for pair in "$@"; do
  v=${pair%%:*}; d=${pair#*:}; n=$(echo "$pair" | tr ':/' '__')
  if [ "$v" = "-" ]; then unset R3DG_BWD; else export R3DG_BWD=$v; fi
  if [ "$d" = "-" ]; then unset R3DG_LIB_DIR; else export R3DG_LIB_DIR=$d; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "backward" > $OUT/pytest_$n.log 2>&1
  echo "pytest $n ok: $(tail -1 $OUT/pytest_$n.log)"
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_$n.json 2> $OUT/bench_$n.err
  python -c "import json; d=json.load(open('$OUT/bench_$n.json')); print('$n', d['ms_per_step'], d['kernel_ms'])"
done
