"""Print one step's kernel timeline (start offset, duration, gap) from a rocprofv3 kernel trace.
Usage: python tools/step_trace.py gpurun_out/<tag>/prof/run_kernel_trace.csv [step index from the end]"""
import csv
import sys

path = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("r3dg::preprocess_kernel")]
i0, i1 = idx[-k], idx[-k + 1]
t0 = int(rows[i0]["Start_Timestamp"])
prev = None
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
    if "rocprim" in name:
        name = "rocprim::" + ("lookback_init" if "init_lookback" in r["Kernel_Name"] else
                              "onesweep" if "onesweep_iteration" in r["Kernel_Name"] else
                              "histogram" if "histogram" in r["Kernel_Name"] else "scan/other")
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:8.1f} gap {gap:6.1f}  {name}")
    prev = e
print("step span", (int(rows[i1]["Start_Timestamp"]) - t0) / 1e3)
