#!/bin/bash
# PMC passes over one BVH build + 1M-ray trace (tools/bvh_once.py), one rocprofv3 run per group.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_bvh
mkdir -p $OUT
run() {
  name=$1; sc=$2; shift 2
  timeout -k 10 180 rocprofv3 --pmc "$@" --kernel-include-regex "bvh_" \
     -d $OUT/$name.$sc -o run --output-format csv -- python tools/bvh_once.py $sc > $OUT/$name.$sc.log 2>&1
}
for sc in volume surface; do
  run fetch $sc FETCH_SIZE
  run write $sc WRITE_SIZE
  run tcc $sc TCC_HIT_sum TCC_MISS_sum
  run sq $sc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES
done
echo pmc done
