#!/bin/bash
# Round evidence in one GPU call (every GPU step under its own time limit; the first failure ends
# the call). Output under gpurun_out/TAG/.
#   bash tools/gpu_evidence.sh TAG PART...
#   PART: tests | bench | prof | gui | configs | brdf | pmc | ab:SPEC,SPEC... (tools/gpu_ab_env.sh)
#   tests/bench/prof: tools/gpu_round.sh; gui: tools/bench_gui.py under rocprofv3 (kernel summary);
#   configs: tools/bench_configs.py (C1-C5); brdf: tools/bench_brdf.py; pmc: PMC passes ->
#   profiles/traffic_latest.json + profiles/valu_latest.json (copies under gpurun_out/TAG/).
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for part in "$@"; do
  case $part in
    tests|bench|benchq|prof) bash tools/gpu_round.sh $TAG $part ;;
    gui)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/guiprof -o run -- python tools/bench_gui.py --iters 5 --out $OUT/gui.json > $OUT/guiprof.log 2>&1 \
        || { tail -20 $OUT/guiprof.log; exit 1; }
      f=$(find $OUT/guiprof -name '*kernel_stats.csv' | head -1); cp "$f" $OUT/gui_kernel_stats.csv
      cat $OUT/gui.json; head -14 $OUT/gui_kernel_stats.csv | cut -c1-150 ;;
    configs)
      timeout -k 10 400 python tools/bench_configs.py --iters 10 --out $OUT/configs.json > $OUT/configs.log 2>&1 || { tail -20 $OUT/configs.log; exit 1; }
      tail -3 $OUT/configs.log | cut -c1-400 ;;
    brdf)
      timeout -k 10 300 python tools/bench_brdf.py > $OUT/brdf.log 2>&1 || { tail -20 $OUT/brdf.log; exit 1; }
      tail -5 $OUT/brdf.log | cut -c1-400 ;;
    pmc)
      bash tools/pmc_passes.sh
      python tools/pmc_summary.py gpurun_out/pmc > $OUT/pmc_summary.json
      python tools/make_traffic.py $OUT/pmc_summary.json profiles/traffic_latest.json "M1 P=1000000" > /dev/null
      python tools/make_valu.py $OUT/pmc_summary.json profiles/valu_count_latest.txt profiles/valu_latest.json > /dev/null
      cp profiles/traffic_latest.json profiles/valu_latest.json $OUT/ ;;
    ab:*)
      specs=${part#ab:}
      bash tools/gpu_ab_env.sh ${TAG}_ab ${specs//,/ } ;;
    *) echo "unknown part $part"; exit 2 ;;
  esac
done
