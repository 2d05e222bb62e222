"""The cfg3 ESIM and cfg2 DSSM bench legs under different untimed warm-up lengths (diagnostics: clock ramp after
idle vs sustained-load clock). Calls bench.py's own leg functions."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    args = bench.parse() if hasattr(bench, "parse") else None
    args.steps, args.warmup = 20, 5
    for w in (0.0, 0.05, 0.25, 1.0, 0.0):
        bench._time_stages.__defaults__ = (w,)
        r = bench.bench_esim(args)
        print(json.dumps({"leg": "cfg3", "warm_s": w, "ms": r["ms_per_step"], "eager_ms": r["eager_ms_per_step"],
                          "stages": r["stage_ms"]}), flush=True)


if __name__ == "__main__":
    sys.argv = [sys.argv[0]]
    main()
