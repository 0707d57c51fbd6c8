"""Per-kernel statistics from a rocprofv3 rocpd database (the default output format of ROCm 7's
rocprofv3): name, calls, total / average duration -- the same columns as its --stats CSV.

Usage: python tools/rocpd_stats.py RUN_results.db [OUT.csv]"""
import csv
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else cols[0])
rows = c.execute(f"select {name_col}, count(*), sum(end - start), avg(end - start), min(end - start), "
                 f"max(end - start) from kernels group by {name_col} order by sum(end - start) desc").fetchall()
total = sum(r[2] for r in rows) or 1
out = [["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"]]
for n, k, s, a, mn, mx in rows:
    out.append([n, k, int(s), round(a, 1), round(100.0 * s / total, 3), int(mn), int(mx)])
w = csv.writer(open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout)
w.writerows(out)
