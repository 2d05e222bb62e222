"""rf_gemm_f32 probe (diagnostics, not product): every DSSM tower GEMM shape of the cfg2 training step (forward
y = x W^T, weight gradient G = dpre^T h, input gradient dz = dpre W) plus ragged shapes, checked against a float64
torch GEMM on the GPU and timed with HIP events next to torch.mm (hipBLASLt) on the same operands.

usage: python tools/gemm32_probe.py [--lib path/to/lib.so] [--reps 20] [--only fwd,dw,dz,edge]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 157.3e12

CASES = [
    # name, M, N, K, a_kc, b_kc, act
    ("fwd_user", 4096, 1024, 8704, 1, 1, 3), ("fwd_ad", 4096, 1024, 20480, 1, 1, 3),
    ("fwd_l2", 4096, 512, 1024, 1, 1, 3), ("fwd_l3", 4096, 256, 512, 1, 1, 3),
    ("dw_user", 1024, 8704, 4096, 0, 0, 0), ("dw_ad", 1024, 20480, 4096, 0, 0, 0),
    ("dw_l2", 512, 1024, 4096, 0, 0, 0), ("dw_l3", 256, 512, 4096, 0, 0, 0),
    ("dz_user", 4096, 8704, 1024, 1, 0, 0), ("dz_ad", 4096, 20480, 1024, 1, 0, 0),
    ("dz_l2", 4096, 1024, 512, 1, 0, 0), ("dz_l3", 4096, 512, 256, 1, 0, 0),
    ("edge_kk", 300, 200, 100, 1, 1, 3), ("edge_mm", 132, 260, 36, 0, 0, 0), ("edge_km", 257, 132, 1028, 1, 0, 1),
    ("edge_mk", 132, 127, 68, 0, 1, 2), ("edge_k0", 64, 64, 0, 1, 1, 3), ("edge_tail", 1000, 700, 4100, 0, 0, 0),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "recommendflow_amd", "lib", "librf.so"))
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--cases", default="", help="extra cases name:M:N:K:akc:bkc:act,...")
    args = ap.parse_args()
    lib = ctypes.CDLL(args.lib)
    lib.rf_gemm_f32_ws_bytes.restype = ctypes.c_size_t
    lib.rf_gemm_f32_ws_bytes.argtypes = [ctypes.c_int64] * 3
    lib.rf_gemm_f32.restype = ctypes.c_int
    lib.rf_gemm_f32.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64,
                                ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t,
                                ctypes.c_void_p]
    lib.rf_last_error.restype = ctypes.c_char_p
    dev = torch.device("cuda:0")
    ws_n = max(int(lib.rf_gemm_f32_ws_bytes(M, N, K)) for _, M, N, K, *_ in CASES) * 2
    ws = torch.zeros(ws_n, dtype=torch.uint8, device=dev)
    only = set(args.only.split(",")) if args.only else None
    cases = list(CASES)
    if args.cases:
        cases = [(c.split(":")[0], *map(int, c.split(":")[1:])) for c in args.cases.split(",")]
    out = []
    for name, M, N, K, akc, bkc, act in cases:
        if only and name.split("_")[0] not in only:
            continue
        g = torch.Generator(device=dev).manual_seed(M * 7 + N * 3 + K)
        a = torch.randn((M, K) if akc else (K, M), device=dev, generator=g)
        b = torch.randn((N, K) if bkc else (K, N), device=dev, generator=g)
        bias = torch.randn(N, device=dev, generator=g) if act else None
        opA = a if akc else a.t()
        opB = b.t() if bkc else b
        c = torch.full((M, N), float("nan"), device=dev)
        st = torch.cuda.current_stream().cuda_stream

        def run():
            rc = lib.rf_gemm_f32(a.data_ptr(), a.stride(0), akc, b.data_ptr(), b.stride(0), bkc, M, N, K,
                                 bias.data_ptr() if bias is not None else None, act, c.data_ptr(), c.stride(0),
                                 ws.data_ptr(), ws.numel(), st)
            if rc != 0:
                raise RuntimeError(lib.rf_last_error().decode())

        run()
        torch.cuda.synchronize()
        ref = opA.double() @ opB.double()
        if bias is not None:
            ref += bias.double()
        if act == 3:
            ref = torch.selu(ref)
        elif act == 2:
            ref = torch.relu(ref)
        elif act == 1:
            ref = torch.nn.functional.gelu(ref)
        scale = (opA.double().abs() @ opB.double().abs()) + (bias.double().abs() if bias is not None else 0) + 1e-30
        err = float(((c.double() - ref).abs() / scale).max()) if M * N else 0.0
        bad = int(torch.isnan(c).sum())
        # repeat determinism: the same bits every launch (fixed combine order)
        c1 = c.clone()
        run()
        torch.cuda.synchronize()
        same = bool(torch.equal(c1, c))
        t_ms = bl_ms = None
        if K >= 256 and M * N >= 1 << 20:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            for _ in range(3):
                run()
            ev[0].record()
            for _ in range(args.reps):
                run()
            ev[1].record()
            for _ in range(3):
                torch.mm(opA, opB)
            ev[2].record()
            for _ in range(args.reps):
                torch.mm(opA, opB)
            ev[3].record()
            torch.cuda.synchronize()
            t_ms = ev[0].elapsed_time(ev[1]) / args.reps
            bl_ms = ev[2].elapsed_time(ev[3]) / args.reps
        fl = 2.0 * M * N * K
        rec = {"case": name, "M": M, "N": N, "K": K, "rel_err": err, "nan": bad, "deterministic": same,
               "ms": t_ms, "tflops": fl / t_ms / 1e9 if t_ms else None,
               "frac": fl / t_ms / 1e9 / (PEAK / 1e12) if t_ms else None,
               "blaslt_ms": bl_ms, "blaslt_frac": fl / bl_ms / 1e9 / (PEAK / 1e12) if bl_ms else None}
        out.append(rec)
        print(json.dumps(rec), flush=True)
    ok = all((r["rel_err"] < 2e-6 or (r["K"] == 0 and r["rel_err"] < 1e-4)) and r["nan"] == 0 and r["deterministic"] for r in out)
    print("ALL_OK" if ok else "FAILED", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
