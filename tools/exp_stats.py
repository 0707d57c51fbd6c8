"""Per-build kernel averages from tools/exp_prof.sh output: python tools/exp_stats.py NAME..."""
import csv
import glob
import json
import sys

KEYS = ["render_fwd_glds", "render_fwd_mfma", "render_bwd_glds", "row_sum", "gather_bwd", "preprocess_kernel", "bin_scatter",
        "tile_depth_sort"]
for n in sys.argv[1:]:
    f = glob.glob(f"gpurun_out/expprof/{n}/**/*kernel_stats.csv", recursive=True)
    out = {}
    for row in csv.DictReader(open(f[0])):
        for k in KEYS:
            if k in row["Name"]:
                out[k] = round(float(row["AverageNs"]) / 1e3, 1)
    try:
        ms = json.loads(open(f"gpurun_out/expprof/{n}.log").read().strip().splitlines()[-1])["ms_per_step"]
    except Exception:
        ms = None
    print(n, ms, out)
