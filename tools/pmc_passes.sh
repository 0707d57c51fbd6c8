#!/bin/bash
# PMC counter passes over tools/step_once.py (one rocprofv3 run per counter group; no tracing
# domains combined with --pmc). Output: gpurun_out/pmc/<pass>/...counter_collection.csv
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc
mkdir -p $OUT
run() {
  name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-include-regex "render_|gather_bwd|row_sum|preprocess_kernel|bin_|tile_" \
     -d $OUT/$name -o run --output-format csv -- python tools/step_once.py > $OUT/$name.log 2>&1
}
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES
run sq2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
run fetch FETCH_SIZE
run write WRITE_SIZE
run tcc TCC_HIT_sum TCC_MISS_sum
echo pmc done
