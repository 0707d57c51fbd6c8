"""Per-build kernel times per step from tools/exp_prof.sh output: python tools/exp_stats.py NAME...
(us per step = total kernel time / number of render_bwd launches; ms/step from the bench line)."""
import csv
import glob
import json
import sys

KEYS = ["render_fwd_glds", "render_bwd_glds", "row_sum", "gather_bwd", "preprocess_kernel", "bin_scatter",
        "tile_depth_sort", "xyz_normal"]
for n in sys.argv[1:]:
    f = glob.glob(f"gpurun_out/expprof/{n}/**/*kernel_stats.csv", recursive=True)
    if not f:
        print(n, "missing")
        continue
    rows = list(csv.DictReader(open(f[0])))
    steps = max((int(r["Calls"]) for r in rows if "render_bwd_glds" in r["Name"]), default=1)
    out = {}
    for r in rows:
        for k in KEYS:
            if k in r["Name"]:
                out[k] = round(float(r["TotalDurationNs"]) / steps / 1e3, 1)
    ms = None
    for line in open(f"gpurun_out/expprof/{n}.log"):
        if line.startswith("{"):
            try:
                ms = json.loads(line)["ms_per_step"]
            except Exception:
                pass
    print(n, ms, out)
