"""cfg3 forward timing probe: runs bench.bench_esim several times in one process at the driver's step count and at a
long one, so the whole-forward graph's wall time can be compared with its stage times without the other legs around
it. Usage: REPS=2 python tools/cfg3_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.argv = [sys.argv[0], "--cpu-seconds", "0"]

import torch  # noqa: E402

import bench  # noqa: E402

args = bench.parse()
args.probes = None
reps = int(os.environ.get("REPS", "2"))
for steps in (20, 400, 20):
    for r in range(reps):
        args.steps = steps
        out = bench.bench_esim(args)
        print(json.dumps({"steps": steps, "rep": r, "ms": out["ms_per_step"], "eager_ms": out["eager_ms_per_step"],
                          "stage_ms": out["stage_ms"], "unfused": out["unfused_stage_ms"]}), flush=True)
        torch.cuda.empty_cache()
