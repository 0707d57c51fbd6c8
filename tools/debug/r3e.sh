mkdir -p gpurun_out/r3e
timeout -k 10 120 python tools/debug/sh_rebuild_bits.py > gpurun_out/r3e/shdbg.txt 2>&1; echo "dbg rc=$?"; tail -5 gpurun_out/r3e/shdbg.txt
for n in CW0 CW2 base; do
  if [ "$n" = base ]; then d=""; else d=exp/$n/lib; fi
  R3DG_LIB_DIR=$d timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3e/$n.json 2> gpurun_out/r3e/$n.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r3e/$n.json')); print('$n', d['ms_per_step'], d['kernel_ms'])"
done
