"""Times bench.bench_esim_train (the cfg3-shape ESIM training step) on its own; run under rocprofv3 for the
per-kernel split of the step."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = ["bench.py", "--steps", sys.argv[1] if len(sys.argv) > 1 else "20"]
import bench  # noqa: E402

print(json.dumps(bench.bench_esim_train(bench.parse())))
