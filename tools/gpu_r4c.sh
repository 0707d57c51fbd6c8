#!/bin/bash
# Round-4 checks, part 1: BRDF / reduction / shader parity (printed diffs), the bitonic fused sort's
# key parity, then the reduction / split / sort A/B.
set -e
OUT=gpurun_out/r4c
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_shaders.py tests/test_postprocess.py -m gpu -x -q -s \
  -k "brdf or reductions or shader or splat or post or texture" --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 \
  || { grep -h "brdf \|passed\|failed\|Error\|assert" $OUT/parity.log | tail -40; exit 1; }
grep -h "brdf \|passed\|failed" $OUT/parity.log | tail -40
R3DG_LIB_DIR=exp/BITONIC/lib timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  -k "keys or sort or dense or binning or forward" --timeout 200 --timeout-method thread > $OUT/bitonic.log 2>&1 \
  || { tail -30 $OUT/bitonic.log; exit 1; }
tail -1 $OUT/bitonic.log
bash tools/gpu_ab_env.sh r4c base base+R3DG_BWD_REDUCE=atomic,R3DG_BWD_SRS=24 base+R3DG_BWD_REDUCE=atomic rne+R3DG_LIB_DIR=exp/RNE/lib split2+R3DG_LIB_DIR=exp/SPLIT2/lib split2a+R3DG_LIB_DIR=exp/SPLIT2/lib,R3DG_BWD_REDUCE=atomic nosort+R3DG_LIB_DIR=exp/NOSORT/lib bitonic+R3DG_LIB_DIR=exp/BITONIC/lib base.2 base+R3DG_BWD_REDUCE=atomic.2 rne.2+R3DG_LIB_DIR=exp/RNE/lib bitonic.2+R3DG_LIB_DIR=exp/BITONIC/lib
