#!/bin/bash
# Quick GPU iteration: a pytest selection (-k EXPR, may be empty = whole GPU suite) with the gradient
# report, then N bench lines. A test failure does not end the call; a timeout / abort / fault does.
#   bash tools/gpu_quick.sh TAG "K_EXPR" NBENCH
OUT=gpurun_out/$1; K=$2; NB=${3:-2}
mkdir -p $OUT
export TMPDIR=/tmp
ok() { local rc=$1; case $rc in 124|137|134|139) echo "fatal rc $rc"; exit $rc;; esac; return 0; }
if [ "$K" != "-" ]; then
  R3DG_GRAD_REPORT=$OUT/grad.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu ${K:+-k "$K"} -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; ok $?
  grep -E "^(FAILED|ERROR)|passed|failed" $OUT/pytest.log | tail -8
fi
for i in $(seq 1 $NB); do
  timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_$i.json 2> $OUT/bench_$i.err; ok $?
  python -c "import json; d=json.load(open('$OUT/bench_$i.json')); print(d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])" || tail -5 $OUT/bench_$i.err
done
