#!/bin/bash
# Round-3 GPU check: the needle cull test against the constant-margin build (expected red), then the
# full GPU suite on the default build. Usage: bash tools/gpu_r3_tests.sh <tag>
TAG=${1:-r3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
R3DG_LIB_DIR=exp/CULL0/lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "needles" -x -v --timeout 400 --timeout-method thread > $OUT/cull0.log 2>&1
rc=$?; echo "cull0 rc=$rc"; tail -5 $OUT/cull0.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -15 $OUT/pytest.log; exit $rc
