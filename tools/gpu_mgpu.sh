#!/bin/bash
# One GPU call: the view-parallel exchange tests and a 2-rank gloo rehearsal of bench.py's N > 1
# path on the single GPU (the driver's 8-GPU run uses RCCL).
set -e
OUT=gpurun_out/${1:-mgpu}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "view_parallel or sh_rebuild or chunked" > $OUT/pytest.log 2>&1
echo pytest ok; tail -3 $OUT/pytest.log
R3DG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench2.log 2>&1
echo bench2 ok; tail -1 $OUT/bench2.log | cut -c1-400
