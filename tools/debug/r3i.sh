mkdir -p gpurun_out/r3i
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r3i/bench.json 2> gpurun_out/r3i/bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r3i/bench.json')); print(d['ms_per_step'], d['value'], d['kernel_ms'])"
timeout -k 10 200 python -u -m pytest tests/test_gpu_fullsize.py -k "brdf" -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r3i/brdf.log 2>&1; grep -E "hip .* oracle|PASS|FAIL" gpurun_out/r3i/brdf.log | head -20
