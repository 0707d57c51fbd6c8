#!/bin/bash
# Scalar-unit load of the blends (one scalar ALU per CU on MI300/MI355): SALUBusy =
# SQ_INST_CYCLES_SALU (quad-cycles) x 4 / CUs / GRBM_GUI_ACTIVE cycles. One rocprofv3 --pmc pass
# over tools/step_once.py. Output: gpurun_out/$1/salu/...counter_collection.csv
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --pmc SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_BRANCH GRBM_GUI_ACTIVE \
   --kernel-include-regex "render_|gather_bwd|preprocess_kernel|bin_" -d $OUT/salu -o run --output-format csv -- python tools/step_once.py > $OUT/salu.log 2>&1
echo salu pmc done
