mkdir -p gpurun_out/r3d
timeout -k 10 120 python tools/debug/sh_rebuild_bits.py > gpurun_out/r3d/shdbg.txt 2>&1; echo "dbg rc=$?"; cat gpurun_out/r3d/shdbg.txt | tail -8
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r3d/bench.json 2> gpurun_out/r3d/bench.err || exit 1
tail -c 1500 gpurun_out/r3d/bench.json
