#!/bin/bash
# Round-4: LDS-DMA ids/bits + partial batch-end wait (exp/LDSIDS) -- backward parity with that build,
# then its A/B; shader / post parity of the coalesced shader records and the GUI timing.
set -e
OUT=gpurun_out/r4i
mkdir -p $OUT
export TMPDIR=/tmp
R3DG_LIB_DIR=exp/LDSIDS/lib timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  -k "(backward or reductions or needles or cull or chunked or ranks) and not brdf" --timeout 250 --timeout-method thread > $OUT/ldsids.log 2>&1 \
  || { tail -30 $OUT/ldsids.log; exit 1; }
tail -1 $OUT/ldsids.log
timeout -k 10 300 python -u -m pytest tests/test_shaders.py tests/test_postprocess.py tests/test_gpu_parity.py -k "shader or splat or post or texture or brdf" -s -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/shaders.log 2>&1 \
  || { tail -30 $OUT/shaders.log; exit 1; }
grep -h "brdf \|passed\|failed" $OUT/shaders.log | tail -30
bash tools/gpu_ab_env.sh r4i base ldsids+R3DG_LIB_DIR=exp/LDSIDS/lib base.2 ldsids.2+R3DG_LIB_DIR=exp/LDSIDS/lib ldsrows+R3DG_LIB_DIR=exp/LDSIDS/lib,R3DG_BWD_REDUCE=rows rows+R3DG_BWD_REDUCE=rows
timeout -k 10 200 python tools/bench_gui.py --iters 10 --out $OUT/gui.json
