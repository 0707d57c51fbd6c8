#!/bin/bash
# Time experiment builds: bash tools/exp_run.sh NAME... (base = the in-tree build; NAME.2 repeats
# NAME; NAME+VAR=VAL sets VAR=VAL): ms/step and kernel_ms per build, no profiler attached.
set -e
mkdir -p gpurun_out/exp
for n in "$@"; do
  lib=${n%%+*}; envs=""
  if [ "$lib" != "$n" ]; then envs=${n#*+}; fi
  b=${lib%%.*}
  if [ "$b" = base ]; then d=""; else d=exp/$b/lib; fi
  ([ -n "$envs" ] && export $envs; R3DG_LIB_DIR=$d timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/exp/$n.json 2> gpurun_out/exp/$n.err)
  python -c "import json,sys; d=json.load(open('gpurun_out/exp/$n.json')); print('$n', d['ms_per_step'], d['kernel_ms'])"
done
