"""Counting experiment (R3DG_EXP_COUNT build): one M1 step, then the device counters.
R3DG_LIB_DIR=exp/COUNT/lib python tools/exp_count.py"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import relightable3dgaussian_amd as r3  # noqa: E402

sys.argv = ["bench.py", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"]
bench.main()
lib = ctypes.CDLL(os.path.join(r3.LIB_DIR, "libr3dg_hip.so"))
buf, fb = (ctypes.c_ulonglong * 8)(), (ctypes.c_ulonglong * 8)()
lib.r3dg_exp_counters_bwd(buf)
lib.r3dg_exp_counters_fwd(fb)
names = ["bwd live pairs", "bwd mfma groups", "bwd staging wall ticks (sum over waves)",
         "bwd batch-loop wall ticks (sum over waves)"]
for i, n in enumerate(names):
    print(f"{n}: {buf[i]}")
print(f"bwd staging fraction: {buf[2] / max(buf[3], 1):.3f}")
print(f"bwd mask/issue ticks: {buf[4]} ({buf[4] / max(buf[3], 1):.3f})")
print(f"bwd in-loop flush ticks: {buf[7]} ({buf[7] / max(buf[3], 1):.3f})")
# bench.main runs the warm-up steps, the timed steps and as many profiled steps: 2 at --steps 1
print("m1 steps run: 2")
print(f"fwd steps done: {fb[2]}\nfwd live pairs (pre-exit): {fb[3]}")
print(f"fwd accumulated lane-steps: {fb[4]}\nfwd instances with any accumulating pixel: {fb[5]}")
print(f"bwd visited instances with any ok pixel: {buf[5]} of {buf[0]}\nbwd ok lane-steps: {buf[6]}")
