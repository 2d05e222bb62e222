"""Split a rocprofv3 kernel trace into busy time and idle gaps (diagnostics).
    python tools/trace_gaps.py <run_kernel_trace.csv> [--last N]
Prints, over the last N kernels (default all): the span, the sum of kernel durations (overlaps merged), the
idle time between them, and per kernel name its count, average duration and the average gap before it."""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 0
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    if last:
        rows = rows[-last:]
    span = rows[-1][1] - rows[0][0]
    busy, cur_s, cur_e = 0, rows[0][0], rows[0][1]
    gap_before = defaultdict(list)
    dur = defaultdict(list)
    for k, (s, e, n) in enumerate(rows):
        dur[n].append(e - s)
        if k:
            gap_before[n].append(max(0, s - max(x[1] for x in rows[max(0, k - 4):k])))
        if s > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"kernels {len(rows)}  span {span / 1e3:.1f} us  busy {busy / 1e3:.1f} us  idle {(span - busy) / 1e3:.1f} us")
    for n in sorted(dur, key=lambda n: -sum(dur[n])):
        g = gap_before.get(n, [0])
        print(f"  {len(dur[n]):5d}  avg {sum(dur[n]) / len(dur[n]) / 1e3:8.2f} us  gap-before {sum(g) / len(g) / 1e3:7.2f} us  {n[:110]}")


if __name__ == "__main__":
    main()
