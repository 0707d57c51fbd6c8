#!/bin/bash
# One GPU call: the GPU suite, then a bench line (and optionally a rocprof kernel summary).
#   bash tools/gpu_round.sh TAG [tests|bench|prof]...   (default: tests bench)
# Output under gpurun_out/TAG/. Every GPU step has its own time limit; the first failure ends the call.
set -e
TAG=$1; shift
STEPS=${@:-tests bench}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 \
        || { tail -30 $OUT/pytest.log; exit 1; }
      tail -1 $OUT/pytest.log ;;
    bench)
      timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])" ;;
    benchq)
      timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/benchq.json 2> $OUT/benchq.err || { tail -20 $OUT/benchq.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/benchq.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])" ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1 \
        || { tail -20 $OUT/prof.log; exit 1; }
      f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); cp "$f" $OUT/kernel_stats.csv; head -12 $OUT/kernel_stats.csv | cut -c1-160 ;;
  esac
done
