#!/bin/bash
# One GPU call: parity (forward/binning, full-size) of the in-tree depth sort, then M1 and C4 bench
# over lib dirs ("-" = in-tree). Usage: bash tools/gpu_sort_ab.sh TAG LIBDIR...
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest ok: $(tail -1 $OUT/pytest.log)"
for d in "$@"; do
  n=$(echo "$d" | tr '/' '_')
  if [ "$d" = "-" ]; then unset R3DG_LIB_DIR; else export R3DG_LIB_DIR=$d; fi
  if [ "$d" != "-" ]; then
    timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dense or forward_matches" > $OUT/pytest_$n.log 2>&1
    echo "pytest $n ok: $(tail -1 $OUT/pytest_$n.log)"
  fi
  for P in 1000000 2000000; do
    timeout -k 10 180 python bench.py --P $P --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_${n}_$P.json 2> $OUT/bench_${n}_$P.err
    python -c "import json; d=json.load(open('$OUT/bench_${n}_$P.json')); print('$n', $P, d['value'], d['ms_per_step'])"
  done
done
