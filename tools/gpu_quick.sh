#!/bin/bash
# Quick GPU iteration: a pytest selection (-k EXPR; "" = the whole GPU suite, "-" = none) with the
# gradient report, then NBENCH rounds of bench lines: the in-tree build and every experiment build
# NAME:FLAGS (compiled here on the box into exp/NAME; exp/*/lib is not uploaded), alternating.
# A test failure does not end the call; a timeout / abort / fault does.
#   bash tools/gpu_quick.sh TAG "K_EXPR" NBENCH [NAME:FLAGS ...]
OUT=gpurun_out/$1; K=$2; NB=${3:-2}; shift 3
mkdir -p $OUT
export TMPDIR=/tmp
ok() { local rc=$1; case $rc in 124|137|134|139) echo "fatal rc $rc"; exit $rc;; esac; return 0; }
names=""
for spec in "$@"; do
  n=${spec%%:*}; f=${spec#*:}
  bash tools/exp_build.sh $n "$f" > $OUT/build_$n.log 2>&1 || { tail -5 $OUT/build_$n.log; exit 1; }
  names="$names $n"
done
if [ "$K" != "-" ]; then
  R3DG_GRAD_REPORT=$OUT/grad.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu ${K:+-k "$K"} -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; ok $?
  grep -E "^(FAILED|ERROR)|passed|failed" $OUT/pytest.log | tail -8
fi
for i in $(seq 1 $NB); do
  for n in base $names; do
    if [ $n = base ]; then lib=""; else lib="R3DG_LIB_DIR=exp/$n/lib"; fi
    env $lib timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/${n}_$i.json 2> $OUT/${n}_$i.err; ok $?
    python -c "import json; d=json.load(open('$OUT/${n}_$i.json')); print('$n', d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])" || tail -5 $OUT/${n}_$i.err
  done
done
