#!/bin/bash
# Round-4 checks in one GPU call: BRDF / reduction / shader parity (printed diffs), reduction A/B,
# GUI-path timing (DMA vs register-staged shader blend), then the full suite.
set -e
OUT=gpurun_out/r4c
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_shaders.py tests/test_postprocess.py -m gpu -x -q -s \
  -k "brdf or reductions or shader or splat or post or texture" --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 \
  || { grep -h "brdf \|passed\|failed\|Error\|assert" $OUT/parity.log | tail -40; exit 1; }
grep -h "brdf \|passed\|failed" $OUT/parity.log | tail -40
bash tools/gpu_ab_env.sh r4c base base+R3DG_BWD_REDUCE=atomic rne+R3DG_LIB_DIR=exp/RNE/lib split2+R3DG_LIB_DIR=exp/SPLIT2/lib split2a+R3DG_LIB_DIR=exp/SPLIT2/lib,R3DG_BWD_REDUCE=atomic nosort+R3DG_LIB_DIR=exp/NOSORT/lib base.2 base+R3DG_BWD_REDUCE=atomic.2 rne.2+R3DG_LIB_DIR=exp/RNE/lib
timeout -k 10 200 python tools/bench_gui.py --iters 10 --out $OUT/gui_dma.json
R3DG_FWD_SHADER=reg timeout -k 10 200 python tools/bench_gui.py --iters 10 --out $OUT/gui_reg.json
bash tools/gpu_round.sh r4c tests
