#!/bin/bash
# One GPU call for the BVH tracer: parity tests, timing (both scenes), rocprofv3 kernel stats.
# Usage (repo root on the GPU box): bash tools/gpu_bvh.sh <tag>
set -e
TAG=${1:-bvh}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_bvh.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest ok"
timeout -k 10 300 python tools/bench_bvh.py --out $OUT/bench_bvh.json > $OUT/bench.log 2>&1
timeout -k 10 300 python tools/bench_bvh.py --scene surface --out $OUT/bench_bvh_surface.json > $OUT/bench_surface.log 2>&1
echo "bench ok"; cat $OUT/bench_bvh.json $OUT/bench_bvh_surface.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python tools/bench_bvh.py --iters 5 --cpu-rays 1000 > $OUT/prof.log 2>&1
echo "prof ok"
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs grep -i "bvh\|Name"
