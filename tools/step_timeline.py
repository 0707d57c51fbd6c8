"""Per-step kernel timeline from a rocprofv3 kernel trace: start offset, gap to the previous
kernel, duration. Usage: python tools/step_timeline.py gpurun_out/TAG/prof/run_kernel_trace.csv [step]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
idx = [i for i, r in enumerate(rows) if "preprocess_kernel" in r["Kernel_Name"]]
a, b = idx[k], idx[k + 1]
t0 = int(rows[a]["Start_Timestamp"])
prev = None
busy = 0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    busy += e - s
    print(f"{(s - t0) / 1e3:8.1f} +{gap:6.1f} {(e - s) / 1e3:8.1f}us {r['Kernel_Name'][:70].replace('void ', '')}")
    prev = e
print(f"step {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us")
