#!/bin/bash
# Kernel stats per experiment build: bash tools/exp_prof.sh NAME... (base = the in-tree build).
# NAME.2 repeats NAME; NAME+VAR=VAL runs NAME with the environment variable VAR=VAL.
set -e
mkdir -p gpurun_out/expprof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in "$@"; do
  lib=${n%%+*}; envs=""
  if [ "$lib" != "$n" ]; then envs=${n#*+}; fi
  b=${lib%%.*}
  if [ "$b" = base ]; then d=""; else d=exp/$b/lib; fi
  ([ -n "$envs" ] && export $envs; R3DG_LIB_DIR=$d timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/expprof/$n -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/expprof/$n.log 2>&1)
  echo "== $n"; tail -1 gpurun_out/expprof/$n.log | cut -c1-200
done
