#!/bin/bash
# A/B of in-tree lib vs prebuilt variant libs: bash ab.sh TAG ROUNDS name=libdir ...
OUT=gpurun_out/$1; R=$2; shift 2
mkdir -p $OUT
export TMPDIR=/tmp
for i in $(seq 1 $R); do
  for spec in base "$@"; do
    n=${spec%%=*}; lib=${spec#*=}
    if [ "$n" = base ]; then e=""; else e="R3DG_LIB_DIR=$lib"; fi
    env $e timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > $OUT/${n}_$i.json 2> $OUT/${n}_$i.err || { tail -5 $OUT/${n}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/${n}_$i.json')); k=d['kernel_ms']; print('$n', d['ms_per_step'], k['render_fwd'], k['render_bwd'], k.get('gather_bwd'))"
  done
done
