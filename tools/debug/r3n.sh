mkdir -p gpurun_out/r3n
timeout -k 10 300 python tools/bench_views.py --out gpurun_out/r3n/views.json > gpurun_out/r3n/views.log 2>&1 || { tail -20 gpurun_out/r3n/views.log; exit 1; }
tail -1 gpurun_out/r3n/views.log
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3n/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r3n/pytest.log; exit $rc
