#!/bin/bash
# Round-4 checks: parity subset (BRDF bit-exactness, both reductions, shader / post paths with the
# DMA shader blend and the DMA intermediate pass), the needle sensitivity bound, the M1 A/B of the
# backward reduction / flush splits / fused sort, and the GUI-path timing.
set -e
OUT=gpurun_out/r4g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_shaders.py tests/test_postprocess.py -m gpu -x -q -s \
  -k "brdf or reductions or shader or splat or post or texture or needles" --timeout 250 --timeout-method thread > $OUT/parity.log 2>&1 \
  || { grep -h "brdf \|needles\|passed\|failed\|Error\|assert" $OUT/parity.log | tail -40; exit 1; }
grep -h "needles\|passed\|failed" $OUT/parity.log | tail -12
bash tools/gpu_ab_env.sh r4g base base+R3DG_BWD_REDUCE=atomic base+R3DG_BWD_REDUCE=atomic,R3DG_BWD_SRS=24 rne+R3DG_LIB_DIR=exp/RNE/lib split2+R3DG_LIB_DIR=exp/SPLIT2/lib split2a+R3DG_LIB_DIR=exp/SPLIT2/lib,R3DG_BWD_REDUCE=atomic nosort+R3DG_LIB_DIR=exp/NOSORT/lib bitonic+R3DG_LIB_DIR=exp/BITONIC/lib base.2 base+R3DG_BWD_REDUCE=atomic.2
timeout -k 10 200 python tools/bench_gui.py --iters 10 --out $OUT/gui_dma.json
R3DG_INTER=reg timeout -k 10 200 python tools/bench_gui.py --iters 10 --out $OUT/gui_interreg.json
R3DG_FWD_SHADER=reg R3DG_INTER=reg timeout -k 10 200 python tools/bench_gui.py --iters 10 --out $OUT/gui_allreg.json
