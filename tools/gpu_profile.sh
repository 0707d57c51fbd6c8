#!/bin/bash
# One GPU call: the counter evidence behind bench.py's roofline (run from the repo root on the box).
#   1. PMC passes over tools/step_once.py (tools/pmc_passes.sh: SQ instruction / wait counters,
#      FETCH_SIZE, WRITE_SIZE, TCC hit/miss -- one rocprofv3 run per counter group);
#   2. the R3DG_EXP_COUNT build (exp/COUNT, built beforehand on the CPU with
#      `bash tools/exp_build.sh COUNT -DR3DG_EXP_COUNT`): live wave-steps of both blend kernels.
# Then: python tools/pmc_summary.py gpurun_out/pmc > profiles/rNN_pmc.json
#       python tools/make_traffic.py profiles/rNN_pmc.json profiles/traffic_latest.json "M1 P=1000000"
#       python tools/make_valu.py profiles/rNN_pmc.json gpurun_out/valu_count.txt profiles/valu_latest.json
set -e
bash tools/pmc_passes.sh
R3DG_LIB_DIR=exp/COUNT/lib timeout -k 10 180 python tools/exp_count.py > gpurun_out/valu_count.txt 2> gpurun_out/valu_count.err
tail -8 gpurun_out/valu_count.txt
python tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.json
echo profile done
