mkdir -p gpurun_out/r3o
for n in NOXMFMA NOYMFMA NOFLUSH base; do
  if [ "$n" = base ]; then d=""; else d=exp/$n/lib; fi
  R3DG_LIB_DIR=$d timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r3o/$n.json 2> gpurun_out/r3o/$n.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r3o/$n.json')); print('$n', d['ms_per_step'], d['kernel_ms'])"
done
