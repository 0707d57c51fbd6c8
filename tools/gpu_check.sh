#!/bin/bash
# One GPU call: parity tests, default bench, rocprofv3 kernel stats of the bench.
# Usage (from the repo root on the GPU box): bash tools/gpu_check.sh <tag>
set -e
TAG=${1:-latest}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest ok"
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1
echo "bench ok"; tail -1 $OUT/bench.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_prof.log 2>&1
echo "prof ok"
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs head -12
