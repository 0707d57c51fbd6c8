#!/bin/bash
# Round-4 checks, part 3: C4 (2M Gaussians, long tiles) sort A/B and a rocprof kernel split of the
# GUI shader path.
set -e
OUT=gpurun_out/r4f
mkdir -p $OUT
export TMPDIR=/tmp
BENCH_ARGS="--P 2000000" bash tools/gpu_ab_env.sh r4f_c4 base bitonic+R3DG_LIB_DIR=exp/BITONIC/lib base.2 bitonic.2+R3DG_LIB_DIR=exp/BITONIC/lib
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/guiprof -o run -- python tools/bench_gui.py --iters 3 > $OUT/guiprof.log 2>&1 \
  || { tail -20 $OUT/guiprof.log; exit 1; }
f=$(find $OUT/guiprof -name '*kernel_stats.csv' | head -1); cp "$f" $OUT/gui_kernel_stats.csv; head -25 $OUT/gui_kernel_stats.csv | cut -c1-150
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -s -k needles --timeout 250 --timeout-method thread > $OUT/needles.log 2>&1 || true; grep -h "needles\|passed\|failed" $OUT/needles.log | tail -8
