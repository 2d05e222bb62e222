"""Random-row gather ceiling (diagnostics): rf_gather_rows of N uniformly random rows of W bytes from a
table far larger than the caches, HIP-event timed. Tells whether an embedding kernel reading rows of the
same width is at the gather ceiling. Usage: python tools/gather_probe.py [--rows 200000000] [--dim 64]
[--dtype bf16|f32] [--n 819200]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch

from recommendflow_amd.runtime import lib as L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=200_000_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--n", type=int, default=819_200)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    table = torch.empty((a.rows, a.dim), dtype=dt, device="cuda")
    L.call("rf_table_init_uniform", L.ptr(table), L.torch_dtype_code(dt), a.rows, a.dim, 0, 1, 7, -0.05, 0.05,
           L.stream_ptr(None))
    g = torch.Generator(device="cuda").manual_seed(1)
    res = {}
    for name, ids in (("uniform", torch.randint(0, a.rows, (a.n,), generator=g, device="cuda")),
                      ("sorted", torch.sort(torch.randint(0, a.rows, (a.n,), generator=g, device="cuda")).values)):
        out = torch.empty((a.n, a.dim), dtype=dt, device="cuda")

        def run():
            L.call("rf_gather_rows", L.ptr(ids), a.n, L.ptr(table), L.torch_dtype_code(dt), a.rows, a.dim, L.ptr(out),
                   L.stream_ptr(None))

        for _ in range(5):
            run()
        s = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps)]
        e = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps)]
        for i in range(a.reps):
            s[i].record()
            run()
            e[i].record()
        torch.cuda.synchronize()
        t = sorted(x.elapsed_time(y) for x, y in zip(s, e))[a.reps // 2]
        row_b = a.dim * table.element_size()
        res[name] = {"ms": round(t, 4), "GBs_read_plus_write": round(a.n * (2 * row_b + 8) / t / 1e6, 1),
                     "row_bytes": row_b}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
