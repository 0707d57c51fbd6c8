#!/bin/bash
# Round-4 state check: full GPU suite, bench line, rocprof of the bench, GUI-path rocprof, configs.
set -e
OUT=gpurun_out/r4h
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_ab_env.sh r4h_ab base qsplit2+R3DG_LIB_DIR=exp/QSPLIT2/lib base.2 qsplit2.2+R3DG_LIB_DIR=exp/QSPLIT2/lib
bash tools/gpu_round.sh r4h tests bench prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/guiprof -o run -- python tools/bench_gui.py --iters 5 --out $OUT/gui.json > $OUT/guiprof.log 2>&1 \
  || { tail -20 $OUT/guiprof.log; exit 1; }
f=$(find $OUT/guiprof -name '*kernel_stats.csv' | head -1); cp "$f" $OUT/gui_kernel_stats.csv; head -14 $OUT/gui_kernel_stats.csv | cut -c1-150
timeout -k 10 400 python tools/bench_configs.py --iters 10 --out $OUT/configs.json > $OUT/configs.log 2>&1 || { tail -20 $OUT/configs.log; exit 1; }
tail -3 $OUT/configs.log | cut -c1-400
