"""Run a few M1 fwd+bwd steps (no timing) -- the target of rocprofv3 runs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("R3DG_STEPS", "3")
import bench  # noqa: E402

sys.argv = ["bench.py", "--steps", os.environ["R3DG_STEPS"], "--warmup", "1", "--no-cpu-baseline"]
bench.main()
