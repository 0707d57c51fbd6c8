#!/bin/bash
# Binning work: the binning / sort parity tests, then the default bench and its kernel profile.
# Usage (GPU box, repo root): bash tools/gpu_bin_check.sh <tag>
set -e
TAG=${1:-bin}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "keys or binning or dense or cull or forward_matches or backward_matches" > $OUT/pytest.log 2>&1
echo "pytest ok"
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1
echo "bench ok"; tail -1 $OUT/bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_prof.log 2>&1
echo "prof ok"
