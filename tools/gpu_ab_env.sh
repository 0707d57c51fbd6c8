#!/bin/bash
# Bench A/B over environment settings of the in-tree build, in one GPU call:
#   bash tools/gpu_ab_env.sh TAG SPEC...   SPEC = name or name+VAR=VAL[,VAR=VAL] ("base" = no extra env)
# ms/step and kernel_ms per SPEC, no profiler attached; outputs under gpurun_out/TAG/.
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for spec in "$@"; do
  envs=""
  if [[ "$spec" == *+* ]]; then envs=${spec#*+}; fi
  n=$(echo "$spec" | tr '+=,/' '__._')
  (for kv in ${envs//,/ }; do export "$kv"; done
   timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/$n.json 2> $OUT/$n.err) \
    || { tail -20 $OUT/$n.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$n.json')); print('$spec', d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])"
done
