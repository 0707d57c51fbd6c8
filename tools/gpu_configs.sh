#!/bin/bash
# One GPU call: re-time BASELINE configs C2-C4 (tools/bench_configs.py) and a rocprofv3 kernel
# summary of the C4-size M1 step (bench.py --P 2000000). Usage: bash tools/gpu_configs.sh TAG
set -e
TAG=${1:-configs}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python tools/bench_configs.py --iters 10 --out $OUT/configs.json > $OUT/configs.log 2>&1
echo "configs ok"; tail -3 $OUT/configs.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4 -o run --output-format csv -- python bench.py --P 2000000 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c4.log 2>&1
echo "c4 prof ok"; tail -1 $OUT/bench_c4.log | cut -c1-300
