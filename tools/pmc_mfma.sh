#!/bin/bash
# One PMC pass on the blend kernels: MFMA / VALU busy, instruction mix (no tracing domains).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_mfma
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex "render_" -d $OUT/a -o run --output-format csv -- python tools/step_once.py > $OUT/a.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU \
  --kernel-include-regex "render_" -d $OUT/b -o run --output-format csv -- python tools/step_once.py > $OUT/b.log 2>&1
echo done
