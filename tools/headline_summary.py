"""Timed-window summary of the headline kernel from a rocprofv3 kernel trace.

usage: python tools/headline_summary.py <rocprofv3 output dir> <bench line json> [--warmup W] [--steps K]
(W and K default to the bench line's own "warmup" / "steps": the driver's protocol is --warmup 5 --steps 20)

Picks the launches of the headline kernel (fused_hash_embed_kernel) with the headline grid (the grid of the
first such launch: the bench's headline leg runs first), takes them in dispatch order, and reports the
average duration over the bench's timed window (launches warmup .. warmup + steps - 1), over the warm-up,
and over every launch of that shape; then the roofline fraction recomputed from the bench line's algorithmic
bytes per launch. Output: plain text on stdout (committed under profiles/rNN/).
"""
import argparse
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("bench_json")
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--kernel", default="fused_hash_embed_kernel")
    ap.add_argument("--peak", type=float, default=8000.0)
    ap.add_argument("--write-trace", default=None, help="write the headline-shape launches' trace rows here (CSV)")
    a = ap.parse_args()
    files = sorted(glob.glob(os.path.join(a.prof_dir, "**", "*kernel_trace.csv"), recursive=True))
    if not files:
        raise SystemExit(f"no *kernel_trace.csv under {a.prof_dir}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if a.kernel in r["Kernel_Name"]:
                    rows.append(r)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if not rows:
        raise SystemExit(f"no {a.kernel} launches")
    grid = rows[0]["Grid_Size_X"] if "Grid_Size_X" in rows[0] else rows[0].get("Grid_Size")
    gkey = "Grid_Size_X" if "Grid_Size_X" in rows[0] else "Grid_Size"
    head = [r for r in rows if r[gkey] == grid]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in head]
    line = None
    with open(a.bench_json) as fh:
        for ln in fh:
            ln = ln.strip()
            if ln.startswith("{") and '"metric"' in ln:
                line = json.loads(ln)
    if a.warmup is None:
        a.warmup = int(line["warmup"]) if line else 5
    if a.steps is None:
        a.steps = int(line["steps"]) if line else 20
    win = dur[a.warmup:a.warmup + a.steps]
    # the settled rate beside it: launches past the bench's window (the uniform leg runs another grid, so these are
    # the headline shape's later launches if any; else the window's second half)
    later = dur[a.warmup + a.steps:]
    if a.write_trace:
        keep = [k for k in ("Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp", gkey, "Workgroup_Size_X",
                            "LDS_Block_Size", "VGPR_Count", "SGPR_Count") if k in head[0]]
        with open(a.write_trace, "w", newline="") as fh:
            wr = csv.writer(fh)
            wr.writerow(keep + ["duration_us"])
            for r, d in zip(head[:a.warmup + a.steps], dur):
                wr.writerow([r[k] for k in keep] + [f"{d:.3f}"])
    print(f"headline kernel {head[0]['Kernel_Name'][:120]}")
    print(f"grid {grid}; trace files: {len(files)}; launches of this shape: {len(head)}")
    print(f"timed window (launches {a.warmup}..{a.warmup + len(win) - 1}): average {statistics.mean(win):.2f} us, "
          f"median {statistics.median(win):.2f} us, min {min(win):.2f}, max {max(win):.2f}")
    if a.warmup:
        print(f"warm-up launches 0..{a.warmup - 1}: average {statistics.mean(dur[:a.warmup]):.2f} us")
    print(f"all {len(dur)} launches of this shape: average {statistics.mean(dur):.2f} us")
    if later:
        print(f"launches after the window ({a.warmup + a.steps}..{len(dur) - 1}): average {statistics.mean(later):.2f} us")
    if line is not None:
        rl = line.get("roofline", {})
        by = rl.get("algorithmic_bytes_per_launch")
        if by:
            ach = by / (statistics.mean(win) * 1e-6) / 1e9
            print(f"bench line (same command, un-profiled run): kernel_ms {rl.get('kernel_ms')}, achieved {rl.get('achieved')} "
                  f"GB/s, frac {rl.get('frac')}")
            print(f"recomputed from the trace: {by} B / {statistics.mean(win):.2f} us = {ach:.1f} GB/s = "
                  f"{ach / a.peak:.4f} of {a.peak:.0f} GB/s"
                  + (f" = {ach / rl['peak_measured']:.4f} of the measured STREAM-copy peak {rl['peak_measured']} GB/s"
                     if rl.get("peak_measured") else ""))


if __name__ == "__main__":
    main()
