mkdir -p gpurun_out/r3q
for n in FL1 base FL1 base; do
  if [ "$n" = base ]; then d=""; else d=exp/$n/lib; fi
  R3DG_LIB_DIR=$d timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r3q/$n.json 2> gpurun_out/r3q/$n.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r3q/$n.json')); print('$n', d['ms_per_step'], d['kernel_ms'])"
done
