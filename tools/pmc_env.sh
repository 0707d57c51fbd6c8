#!/bin/bash
# HBM traffic / L2 counters of one step (tools/step_once.py) under environment settings, one
# rocprofv3 --pmc run per counter group:  bash tools/pmc_env.sh TAG "VAR=val ..." ...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
i=0
for e in "$@"; do
  OUT=gpurun_out/pmcenv/$TAG/$i
  mkdir -p $OUT
  for spec in "fetch FETCH_SIZE" "write WRITE_SIZE" "tcc TCC_HIT_sum TCC_MISS_sum"; do
    set -- $spec; name=$1; shift
    env $e timeout -k 10 -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "render_|gather_bwd|preprocess_kernel" \
       -d $OUT/$name -o run --output-format csv -- python tools/step_once.py > $OUT/$name.log 2>&1
  done
  echo "== $i: $e"
  python tools/pmc_summary.py $OUT > $OUT/summary.json
  python - $OUT/summary.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if "render_bwd" in k or "render_fwd" in k:
        print(k, "fetch GB %.3f write GB %.3f hit %.3g miss %.3g" % (v.get("FETCH_SIZE", 0) * 1024 / 1e9,
              v.get("WRITE_SIZE", 0) * 1024 / 1e9, v.get("TCC_HIT_sum", 0), v.get("TCC_MISS_sum", 0)))
PY
  i=$((i+1))
done
