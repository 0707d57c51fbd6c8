#!/bin/bash
# Round 5, call b: gradient report (fullsize + negative / exact-split test), then a bench A/B of the
# default build against experiment builds compiled here on the box (exp/ libs are not uploaded).
#   bash tools/gpu_r5b.sh TAG "NAME:-DFLAG ..." ...
OUT=gpurun_out/${1:-r5b}; shift
mkdir -p $OUT
export TMPDIR=/tmp
ok() { local rc=$1; case $rc in 124|137|134|139) echo "fatal rc $rc"; exit $rc;; esac; return 0; }
names=""
for spec in "$@"; do
  n=${spec%%:*}; f=${spec#*:}
  bash tools/exp_build.sh $n "$f" > $OUT/build_$n.log 2>&1 || { tail -5 $OUT/build_$n.log; exit 1; }
  names="$names $n"
done
R3DG_GRAD_REPORT=$OUT/grad.jsonl timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py "tests/test_gpu_parity.py::test_one_term_reduction_fails_bar" "tests/test_gpu_parity.py::test_backward_matches_oracle" -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; ok $?
grep -E "passed|failed" $OUT/pytest.log | tail -3
for rep in 1 2; do
  for n in base $names; do
    if [ $n = base ]; then lib=""; else lib="R3DG_LIB_DIR=exp/$n/lib"; fi
    env $lib timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/${n}_$rep.json 2> $OUT/${n}_$rep.err; ok $?
    python -c "import json; d=json.load(open('$OUT/${n}_$rep.json')); print('$n', d['ms_per_step'], d['kernel_ms'])" || tail -5 $OUT/${n}_$rep.err
  done
done
