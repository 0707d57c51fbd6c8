mkdir -p gpurun_out/r3k
R3DG_LIB_DIR=exp/COUNT/lib timeout -k 10 200 python tools/exp_count.py > gpurun_out/r3k/count.txt 2>&1 || exit 1
tail -16 gpurun_out/r3k/count.txt
bash tools/pmc_passes.sh && python tools/pmc_summary.py > gpurun_out/r3k/pmc.json && echo pmc ok
