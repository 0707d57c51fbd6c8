#!/bin/bash
# Round-4 evidence in one GPU call: PMC passes (separate runs per counter group) -> per-kernel
# summary -> profiles/traffic_latest.json + profiles/valu_latest.json, then the full bench line (CPU
# baselines included) with those, and a rocprofv3 kernel-trace summary of a bench run.
set -e
OUT=gpurun_out/r4e
mkdir -p $OUT
bash tools/pmc_passes.sh
python tools/pmc_summary.py gpurun_out/pmc > $OUT/pmc_summary.json
python tools/make_traffic.py $OUT/pmc_summary.json profiles/traffic_latest.json "M1 P=1000000" > /dev/null
python tools/make_valu.py $OUT/pmc_summary.json profiles/r04/valu_count_from_r03.txt profiles/valu_latest.json > /dev/null
cp profiles/traffic_latest.json profiles/valu_latest.json $OUT/
bash tools/gpu_round.sh r4e bench prof
