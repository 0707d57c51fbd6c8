mkdir -p gpurun_out/r3m
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/bench_views.py --out gpurun_out/r3m/views.json > gpurun_out/r3m/views.log 2>&1 || { tail -20 gpurun_out/r3m/views.log; exit 1; }
tail -1 gpurun_out/r3m/views.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3m/prof -o run --output-format csv -- python tools/bench_views.py > gpurun_out/r3m/views_prof.log 2>&1 || exit 1
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r3m/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(r["Name"][:70], r["Calls"], r["AverageNs"])
PY
