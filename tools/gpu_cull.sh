#!/bin/bash
# One GPU call: cull exactness (cull on == off bitwise) and the full-size parity tests (the oracle
# has no cull: n_contrib / final_T bit-exact at M1 scale), then bench A/B against a lib dir.
set -e
mkdir -p gpurun_out/cull
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread -k "cull_is_exact or full" > gpurun_out/cull/pytest.log 2>&1
tail -2 gpurun_out/cull/pytest.log
bash tools/gpu_ab2.sh cullab "$@"
