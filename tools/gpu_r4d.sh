#!/bin/bash
# Round-4 checks, part 2: GUI-path timing (DMA vs register-staged shader blend), the full GPU suite,
# a rocprof kernel summary of the bench.
set -e
OUT=gpurun_out/r4d
mkdir -p $OUT
timeout -k 10 200 python tools/bench_gui.py --iters 10 --out $OUT/gui_dma.json
R3DG_FWD_SHADER=reg timeout -k 10 200 python tools/bench_gui.py --iters 10 --out $OUT/gui_reg.json
bash tools/gpu_round.sh r4d tests prof
