"""Print the per-search kernel times of tools/flatprof_ab.sh's two profiles (25 searches each)."""
import csv
import glob
import sys

for d in sys.argv[1:] or ["gpurun_out/fp_new", "gpurun_out/fp_old"]:
    f = sorted(glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True))
    if not f:
        continue
    print("==", d)
    for x in list(csv.DictReader(open(f[0])))[:8]:
        print(f"{float(x['TotalDurationNs']) / 25 / 1e3:9.1f} us/search  avg {float(x['AverageNs']) / 1e3:8.1f} us  "
              f"n={x['Calls']}  {x['Name'][:90]}")
