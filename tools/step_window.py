"""Kernel timeline of one bench step from a rocprofv3 kernel trace (between two preprocess launches).
python tools/step_window.py gpurun_out/<tag>/prof/run_kernel_trace.csv [step index]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("r3dg::preprocess_kernel")]
i0, i1 = idx[k], idx[k + 1]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1 + 1]:
    s = int(r["Start_Timestamp"]) - t0
    e = int(r["End_Timestamp"]) - t0
    print(f"{s / 1e3:8.1f} {e / 1e3:8.1f} {(e - s) / 1e3:7.1f} {r['Kernel_Name'][:70]}")
