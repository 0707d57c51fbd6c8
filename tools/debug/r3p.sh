mkdir -p gpurun_out/r3p
for n in SORT0 base SORT0 base; do
  if [ "$n" = base ]; then d=""; else d=exp/$n/lib; fi
  R3DG_LIB_DIR=$d timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r3p/$n.json 2> gpurun_out/r3p/$n.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r3p/$n.json')); print('$n', d['ms_per_step'], d['kernel_ms'])"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3p/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3p/prof.log 2>&1 || exit 1
grep -h "depth_sort" $(find gpurun_out/r3p/prof -name "*kernel_stats.csv") | cut -c1-200
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "forward or dense or m1 or c4 or sort" > gpurun_out/r3p/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r3p/pytest.log; exit $rc
