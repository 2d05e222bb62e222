"""Turn rocprofv3 PMC passes (tools/pmc.sh: FETCH_SIZE, WRITE_SIZE) into per-launch HBM bytes for the fused
kernel, with the gfx950 corrections of MI355X_MICROARCH.md §HBM: FETCH_SIZE counts 64 B per 128-B request
for wide (16 B/lane) reads -> x2; WRITE_SIZE is exact for 16-B-per-lane stores. Units: KiB.
usage: python tools/traffic.py gpurun_out/<tag> profiles/traffic_cfg2.json [batch] [table_rows] [dim]
"""
import collections
import csv
import glob
import json
import sys


def per_launch(d, counter, kernel="fused_hash_embed_kernel"):
    vals = collections.defaultdict(float)
    for f in glob.glob(f"{d}/pmc_*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return sum(vals.values()) / len(vals) if vals else None, len(vals)


def main():
    d, out = sys.argv[1], sys.argv[2]
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    rows = int(sys.argv[4]) if len(sys.argv) > 4 else 10_000_000
    dim = int(sys.argv[5]) if len(sys.argv) > 5 else 64
    fetch, nf = per_launch(d, "FETCH_SIZE")
    write, nw = per_launch(d, "WRITE_SIZE")
    rd = fetch * 1024 * 2
    wr = write * 1024
    res = {"kernel": "fused_hash_embed_kernel", "batch": batch, "table_rows": rows, "dim": dim,
           "fetch_size_kib_raw": fetch, "write_size_kib_raw": write, "dispatches": [nf, nw],
           "hbm_read_bytes_per_launch": int(rd), "hbm_write_bytes_per_launch": int(wr),
           "hbm_bytes_per_launch": int(rd + wr),
           "correction": "read = FETCH_SIZE*1024*2 (gfx950 counts 64 B per 128-B wide-read request), write = WRITE_SIZE*1024",
           "source": d}
    # every other counter of the passes, averaged per launch (occupancy / stall / request counters)
    names = set()
    for f in glob.glob(f"{d}/pmc_*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "fused_hash_embed_kernel" in r["Kernel_Name"]:
                names.add(r["Counter_Name"])
    res["counters_per_launch"] = {n: per_launch(d, n)[0] for n in sorted(names - {"FETCH_SIZE", "WRITE_SIZE"})}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
