#!/bin/bash
# One GPU call: the full GPU suite on the in-tree build, then kernel stats of experiment builds
# (tools/exp_prof.sh). Usage: bash tools/gpu_suite_ab.sh TAG NAME...
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest: $(tail -1 $OUT/pytest.log)"
bash tools/exp_prof.sh "$@"
