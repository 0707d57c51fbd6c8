mkdir -p gpurun_out/r3t
for n in ROWS0 base ROWS0 base; do
  if [ "$n" = base ]; then d=""; else d=exp/$n/lib; fi
  R3DG_LIB_DIR=$d timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r3t/$n.json 2> gpurun_out/r3t/$n.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r3t/$n.json')); print('$n', d['ms_per_step'], d['kernel_ms'])"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3t/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r3t/pytest.log; exit $rc
