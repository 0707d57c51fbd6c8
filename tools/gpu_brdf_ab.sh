#!/bin/bash
# One GPU call: BRDF parity tests, then bench_brdf's backward time per lib dir ("-" = in-tree).
# Usage: bash tools/gpu_brdf_ab.sh LIBDIR...
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "brdf" > gpurun_out/brdf_t.log 2>&1
tail -1 gpurun_out/brdf_t.log
for d in "$@"; do
  if [ "$d" = "-" ]; then unset R3DG_LIB_DIR; else export R3DG_LIB_DIR=$d; fi
  timeout -k 10 120 python tools/bench_brdf.py > gpurun_out/brdf_$(echo $d | tr '/' '_').json
  python -c "import json; d=json.load(open('gpurun_out/brdf_$(echo $d | tr '/' '_').json')); print('$d', {k: v['ms'] for k, v in d['results'].items()})"
done
