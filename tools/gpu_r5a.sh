#!/bin/bash
# Round 5, first call: v_exp_f32 correct-rounding probe, GPU suite with the gradient report, bench.
# A test failure does not end the call; a timeout / abort / fault does.
OUT=gpurun_out/${1:-r5a}
mkdir -p $OUT
export TMPDIR=/tmp
ok() { local rc=$1; case $rc in 124|137|134|139) echo "fatal rc $rc"; exit $rc;; esac; return 0; }
hipcc --offload-arch=gfx950 -O3 -o /tmp/vexp_cr tools/probe/vexp_cr.hip > /dev/null 2>&1 || exit 1
timeout -k 10 120 /tmp/vexp_cr > $OUT/vexp.json; ok $?
head -c 1500 $OUT/vexp.json
R3DG_GRAD_REPORT=$OUT/grad.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; ok $?
grep -E "passed|failed" $OUT/pytest.log | tail -3
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err; ok $?
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])"
