"""Benchmark: BASELINE.json metric "examples/sec at 1/2/4/8 GPU + achieved HBM GB/s on embedding gather".

Workload (BASELINE.json configs[1]): the sparse hot path of base_recall_sdpa.yaml —
229 hashing slots (68+1 user incl. slot 0 by deviation D-ellipsis, 160 ad; 30 ArrayType multi-valued),
double hashing (seeds 2022/2023) -> gather -> sum pool -> concat, over ONE fused 10,000,000 x 64 fp32
table (458 segments x 21,834 rows), B = 4096 examples per GPU, synthetic Zipf(1.1) tokens
f"s{slot:03d}:{id}" (runtime/batch.synthetic_batch). A step = one rf_fused_hash_embed_fwd over one
resident CSR batch (inputs in HBM when the timed region starts).

Multi-GPU: one process per GPU; each rank holds a replica of the 2.56 GB table and its own batches (the
reference mirrors tables per GPU, gpu_utils.py:13-14): no data-path collective, weak scaling; value =
examples of all ranks / max-over-ranks time. `--gpus N` without a torchrun environment starts the N
ranks itself (a torch.distributed.run child, launched before this process touches the GPU), like
MirroredStrategy using every visible GPU without a launcher (gpu_utils.py:13-14). Under torchrun the
world size must equal --gpus. `--device cpu --backend gloo` is a dry run of that launcher and of the
barrier / max-over-ranks timing with a no-op step (no GPU, no kernels; the line says "dry_run").

Also reported: roofline of the fused kernel (algorithmic bytes / HIP-event kernel time vs 8 TB/s),
PMC-measured HBM traffic when profiles/ holds it for this workload, and the CPU baseline (the C
oracle — the "port" of the reference semantics — on a bounded sample, rank 0, N=1 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "examples/sec at 1/2/4/8 GPU + achieved HBM GB/s on embedding gather"
HBM_PEAK_GBS = 8000.0
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic_cfg2.json")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); started here unless torchrun set WORLD_SIZE")
    p.add_argument("--device", choices=("cuda", "cpu"), default="cuda", help="cpu = launcher dry run (no kernels)")
    p.add_argument("--backend", choices=("nccl", "gloo"), default=None, help="process-group backend (default: nccl on cuda)")
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=50, help="untimed launches: the clocks and the hot-row cache settle over ~50")
    p.add_argument("--batch", type=int, default=4096)
    p.add_argument("--batches", type=int, default=4, help="distinct resident batches cycled through")
    p.add_argument("--table-rows", type=int, default=10_000_000)
    p.add_argument("--dim", type=int, default=64)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline budget (0 = skip)")
    p.add_argument("--uniform", action="store_true", help="uniform ids instead of Zipf(1.1)")
    p.add_argument("--no-extras", action="store_true", help="skip the cfg3 ESIM / cfg2 DSSM full-forward lines")
    p.add_argument("--no-sharded", action="store_true", help="skip the cfg4 row-sharded extra")
    p.add_argument("--shard-rows", type=int, default=125_000_000, help="cfg4 weak scaling: fused-table rows per GPU")
    p.add_argument("--shard-dim", type=int, default=128)
    p.add_argument("--shard-batch", type=int, default=8192, help="cfg4: examples per GPU (65536 at P=8)")
    p.add_argument("--sim-ranks", type=int, default=8, help="cfg4 at N=1: also time rank 0 of this many ranks "
                                                              "(LoopbackComm; 0 = skip)")
    p.add_argument("--no-train", action="store_true", help="skip the cfg2 DSSM training-step extra")
    p.add_argument("--no-shard-train", action="store_true", help="skip the cfg4 sharded training-step extra")
    p.add_argument("--no-cascade", action="store_true", help="skip the cfg5 recall->prerank->rank extra")
    p.add_argument("--catalog", type=int, default=1_000_000, help="cfg5: items in the catalog")
    p.add_argument("--cascade-sharded", action="store_true", help="cfg5 sharded-recall leg at N=1 too (always at N>1)")
    p.add_argument("--no-pipe", action="store_true", help="skip the TFRecord(GZIP) -> HBM feature-pipe extra")
    p.add_argument("--pipe-examples", type=int, default=65536, help="feature pipe: examples written and read back")
    p.add_argument("--pipe-threads", type=int, default=16, help="feature pipe: reader threads (the box's CPU share)")
    p.add_argument("--no-probes", action="store_true", help="skip the STREAM-copy peak and random-row gather ceilings")
    p.add_argument("--probe-table-gb", type=float, default=32.0, help="gather-ceiling table size (>> 256 MiB Infinity Cache)")
    p.add_argument("--no-uniform-leg", action="store_true", help="skip the uniform-id (no locality) headline leg")
    p.add_argument("--dist-timeout", type=int, default=300, help="seconds before a stuck collective raises (N > 1)")
    return p.parse_args()


def launch(args) -> int:
    """Start args.gpus ranks as a torch.distributed.run CHILD (never exec: this process has not touched
    the GPU, and it only relays the child's exit code). Rank 0 of the child prints the JSON line."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "1"))
    return subprocess.call(cmd, env=env)


def dry_run(args, world, rank):
    """--device cpu: the launcher and timing protocol with a no-op step (gloo). Proves every rank ran
    (all_gather of the ranks) and that value / n_gpus aggregate over the world."""
    import torch
    import torch.distributed as dist

    for _ in range(args.warmup):
        pass
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.001)
    if world > 1:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    ranks = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_gather(ranks, torch.tensor([rank], dtype=torch.int64))
    elapsed = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(args.batch * world * args.steps / elapsed, 1),
                          "unit": "examples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed / args.steps * 1e3, 4), "dry_run": True,
                          "ranks_reported": [int(r.item()) for r in ranks] if world > 1 else [0],
                          "dist_world_size": dist.get_world_size() if world > 1 else 1}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a "
                         f"{world}-rank number as an {args.gpus}-GPU point")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch
    import torch.distributed as dist

    backend = args.backend or ("nccl" if args.device == "cuda" else "gloo")
    if args.device == "cpu":
        if world > 1:
            dist.init_process_group(backend)
        return dry_run(args, world, rank)
    torch.cuda.set_device(local)
    if world > 1:
        # a collective that never completes (an extra leg failing on one rank only) raises after the
        # timeout instead of hanging the run, so the headline line still prints
        os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")
        import datetime

        dist.init_process_group(backend, device_id=torch.device("cuda", local),
                                timeout=datetime.timedelta(seconds=args.dist_timeout))
        assert dist.get_world_size() == world == args.gpus
        # host-side group for the legs' failure flags: a leg that failed on one rank may have aborted the RCCL
        # communicator, so the decision to run the next collective leg goes over gloo
        args.flag_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=args.dist_timeout))

    from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec
    from recommendflow_amd.config_parser.configuration import Configuration
    from recommendflow_amd.runtime.batch import synthetic_batch

    conf = Configuration(os.path.join(ROOT, "tests", "golden", "conf", "base_recall_sdpa.yaml"))
    feats = conf.features.hashing_features
    S = len(feats)
    n_bins = args.table_rows // (2 * S)
    specs = [SlotSpec(f.name, n_bins, tuple(f.hash_seeds), f.pooling.value) for f in feats]
    enc = FusedSparseEncoder(specs, args.dim, table_dtype=torch.float32, seed=2023)
    multi = [bool(f.multivalued) for f in feats]
    host = [synthetic_batch(args.batch, multi, seed=1234 + rank * 1000 + i, uniform=args.uniform)
            for i in range(args.batches)]
    dev = [h.to("cuda") for h in host]
    out = torch.empty((args.batch, enc.out_width), dtype=torch.float32, device="cuda")
    algo_bytes = [enc.algorithmic_bytes(h) for h in host]                 # SURVEY §8d (the roofline's bytes)
    algo_bytes_pad = [enc.algorithmic_bytes(h, pad_rows=True) for h in host]  # round-5 form, for comparison
    torch.cuda.synchronize()

    def step(i):
        enc(dev[i % len(dev)], out=out)

    # The peak the roofline divides by is measured first (STREAM copy, random-row gather ceilings): it also leaves
    # the GPU at its loaded clock. Measured cause of the headline's first-launch slope (tools/settle_probe.py,
    # profiles/r05/settle_probe.txt): launches 5-24 after 2 s idle take 271 us, after any 0.3 s of unrelated GPU
    # work 256 us (the settled value); a full pass over the table's pages does not remove the slope: it is the
    # clock ramp, not cache or TLB warm-up.
    probes = None
    if not args.no_probes:
        try:
            probes = bench_probes(args)
        except Exception as e:  # noqa: BLE001
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            probes = {"error": f"{type(e).__name__}: {e}"[:300]}
    args.probes = probes
    torch.cuda.synchronize()

    for i in range(args.warmup):
        step(i)
    # HIP events around the whole timed region on the launch stream (none between launches: a timing marker between
    # two launches adds ~10 us of gap under rocprof and 3-5 us to a per-launch event pair here); the average launch
    # duration = window / steps, back-to-back launches, gaps included (profiles/r05: the trace's window agrees)
    win0 = torch.cuda.Event(enable_timing=True)
    win1 = torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    win0.record()
    for i in range(args.steps):
        step(i)
    win1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    avg_kern_s = win0.elapsed_time(win1) / args.steps / 1e3
    bytes_per_launch = sum(algo_bytes[i % len(algo_bytes)] for i in range(args.steps)) / args.steps
    bytes_per_launch_pad = sum(algo_bytes_pad[i % len(algo_bytes_pad)] for i in range(args.steps)) / args.steps
    achieved = bytes_per_launch / avg_kern_s / 1e9
    n_tok = sum(h.n_tokens for h in host) / len(host)

    uniform_leg = None
    if not args.no_uniform_leg and not args.uniform:
        try:
            uniform_leg = bench_uniform(args, enc, multi, rank, out)
        except Exception as e:  # noqa: BLE001 — the headline line must still print
            uniform_leg = {"error": f"{type(e).__name__}: {e}"[:300]}

    sharded = None
    if not args.no_sharded:
        del dev, out
        torch.cuda.empty_cache()
        try:
            sharded = bench_sharded(args, specs, multi, rank, world)
        except Exception as e:  # noqa: BLE001 — the headline line must still print
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            sharded = {"error": f"{type(e).__name__}: {e}"[:300]}

    cascade_sh = None
    sharded_failed = isinstance(sharded, dict) and "error" in sharded
    if world > 1:  # every rank skips the next collective leg together if the sharded leg failed on ANY rank
        flag = torch.tensor([1 if sharded_failed else 0], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=args.flag_group)
        sharded_failed = bool(flag.item())
    if not args.no_cascade and (world > 1 or args.cascade_sharded) and not (sharded_failed and world > 1):
        torch.cuda.empty_cache()
        try:
            cascade_sh = bench_cascade_sharded(args, specs, rank, world)
        except Exception as e:  # noqa: BLE001 — reported in place of the numbers; the headline line still prints
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            cascade_sh = {"error": f"{type(e).__name__}: {e}"[:300]}
    if rank != 0:
        if world > 1:
            try:
                dist.destroy_process_group()
            except Exception:  # noqa: BLE001 — a communicator aborted by a failed leg
                pass
        return

    traffic = None
    if os.path.exists(TRAFFIC_FILE):
        tr = json.load(open(TRAFFIC_FILE))
        if tr.get("batch") == args.batch and tr.get("table_rows") == args.table_rows and tr.get("dim") == args.dim:
            traffic = tr.get("hbm_bytes_per_launch")

    cpu = None
    if world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(enc, host[0], args.cpu_seconds)

    def guarded(fn, *a):
        # an extra line must never cost the headline: report its failure in place of its numbers
        try:
            return fn(*a)
        except Exception as e:  # noqa: BLE001
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            return {"error": f"{type(e).__name__}: {e}"[:300]}

    extras = None
    if world == 1 and not args.no_extras:
        if args.no_sharded:
            del dev, out
        torch.cuda.empty_cache()
        extras = {"cfg2_h2d_inclusive": guarded(bench_h2d, args, enc, host),
                  "cfg3_esim_forward": guarded(bench_esim, args), "cfg2_dssm_forward": guarded(bench_dssm, args, enc, host)}
    if world == 1 and not args.no_cascade:
        extras = dict(extras or {}, cfg5_cascade=guarded(bench_cascade, args, enc))
    if world == 1 and not args.no_train:
        extras = dict(extras or {}, cfg2_dssm_train_step=guarded(bench_train, args, specs, multi))
    if world == 1 and not args.no_train:
        extras = dict(extras or {}, cfg3_esim_train_step=guarded(bench_esim_train, args))
    if world == 1 and not args.no_pipe:
        extras = dict(extras or {}, feature_pipe=guarded(bench_pipe, args, enc, specs, multi))
    if world == 1 and not args.no_extras:
        extras = dict(extras or {}, cfg1_demo_two_tower=guarded(bench_cfg1, args))

    value = args.batch * world * args.steps / elapsed
    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "examples/s",
        "n_gpus": world,
        "dist_world_size": dist.get_world_size() if world > 1 else 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": "cfg2 base_recall_sdpa.yaml sparse encoder: hash x2 -> gather -> sum pool -> concat",
            "global_batch": args.batch * world,
            "batch_per_gpu": args.batch,
            "slots": S,
            "table": f"{enc.table_rows}x{args.dim} fp32 fused ({2 * S} segments x {n_bins})",
            "tokens_per_example": round(n_tok / args.batch, 2),
            "ids": "uniform" if args.uniform else "zipf1.1",
            "parallelism": f"replicas{world}",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "fused_hash_embed_kernel",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "algorithmic_bytes_per_launch": int(bytes_per_launch),
            "algorithmic_bytes_form": "SURVEY 8d: rows 2*L*D*4 + pooled out + token bytes + 4 B per token (frac uses this)",
            "algorithmic_bytes_per_launch_with_pad_rows": int(bytes_per_launch_pad),
            "frac_with_pad_rows": round(bytes_per_launch_pad / avg_kern_s / 1e9 / HBM_PEAK_GBS, 4),
            "kernel_ms": round(avg_kern_s * 1e3, 4),
            "kernel_ms_timing": "HIP events around the timed window on the launch stream / steps (launches back to back)",
            "peak_measured": (probes or {}).get("stream_copy_GBs"),
            "frac_of_peak_measured": (round(achieved / probes["stream_copy_GBs"], 4)
                                      if probes and probes.get("stream_copy_GBs") else None),
            "gather_ceiling_256B_GBs": (probes or {}).get("gather_copy_256B_GBs"),
            "frac_of_gather_ceiling": (round(achieved / probes["gather_copy_256B_GBs"], 4)
                                       if probes and probes.get("gather_copy_256B_GBs") else None),
            "uniform": uniform_leg,
        },
        "probes": probes,
        "cpu_baseline": cpu,
        "extras": extras,
        "cfg4_sharded": sharded,
        "cfg5_cascade_sharded": cascade_sh,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        try:
            dist.destroy_process_group()
        except Exception:  # noqa: BLE001 — a communicator aborted by a failed leg
            pass


def _warm(fn, warm_s: float = 0.25, min_iters: int = 2):
    """Untimed repetitions of fn until about warm_s seconds of GPU work have run (see _time_stages)."""
    import torch

    for _ in range(min_iters):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < warm_s and n < 10000:
        fn()
        n += 1
        if n % 8 == 0:  # bounded queue: thousands of unsynchronised graph launches slow later ones on the host
            torch.cuda.synchronize()
    torch.cuda.synchronize()


def _time_stages(stages, steps, warmup, warm_s: float = 0.25):
    """stages: list of (name, fn). HIP events around every stage on the current stream; returns
    (ms per step, {stage: ms}). The untimed warm-up runs `warmup` steps and then more until about warm_s seconds of
    the same work have run: a leg starts after host-side setup (graph capture, allocation) with the GPU idle, and the
    clock takes tens of ms of load to come back (tools/gemm32_insitu_probe.py: the towers' 20480-wide GEMM 1.19 ms
    back to back, 1.24 after 1 ms idle, 1.40 after 50 ms idle; tools/settle_probe.py for the encoder)."""
    import torch

    for _ in range(warmup):
        for _, fn in stages:
            fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < warm_s and n < 10000:
        for _, fn in stages:
            fn()
        n += 1
        if n % 8 == 0:  # bounded queue: thousands of unsynchronised graph launches slow later ones on the host
            torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(len(stages) + 1)] for _ in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        ev[i][0].record()
        for k, (_, fn) in enumerate(stages):
            fn()
            ev[i][k + 1].record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e3
    per = {name: sum(ev[i][k].elapsed_time(ev[i][k + 1]) for i in range(steps)) / steps for k, (name, _) in enumerate(stages)}
    return wall, per


def bench_esim(args):
    """cfg3: ESIM ranking, 200 slots (100 user = q, 100 ad = a) x 1M bins per hash table, D = 64 bf16
    (token dim 128; fused tables 2 x 200M x 64 bf16 = 51.2 GB), 16 dense features, B = 4096."""
    import torch

    from recommendflow_amd.backend.encoder.sparse_encoder import SlotSpec
    from recommendflow_amd.models.ranking.esim import Esim
    from recommendflow_amd.runtime.batch import synthetic_batch

    B, Ls = args.batch, 100
    user = [SlotSpec(f"u{i:03d}", 1_000_000, (2022, 2023)) for i in range(Ls)]
    ad = [SlotSpec(f"a{i:03d}", 1_000_000, (2022, 2023)) for i in range(Ls)]
    model = Esim(user, ad, n_dense=16, dim=64, table_dtype=torch.bfloat16, seed=3)
    hu = [synthetic_batch(B, [False] * Ls, seed=77 + i, slot_ids=range(Ls)).to("cuda") for i in range(2)]
    ha = [synthetic_batch(B, [False] * Ls, seed=99 + i, slot_ids=range(Ls, 2 * Ls)).to("cuda") for i in range(2)]
    dense = torch.randn(B, 16, device="cuda")
    q = torch.empty((B, Ls * 128), dtype=torch.bfloat16, device="cuda")
    a = torch.empty_like(q)
    pooled = torch.empty((B, model.pooled_width), device="cuda")
    from recommendflow_amd.backend.layers.attention_layers import esim_soft_attention_pool

    par = {"s": 0, "f": 0, "e": 0, "i": 0}

    def nxt(k):
        par[k] ^= 1
        return par[k]

    def att():
        esim_soft_attention_pool(q.view(B, Ls, 128), a.view(B, Ls, 128), out=pooled, out_col=model.d_emb)

    def in_mlp():  # the forward's first launch (Esim.concurrent_input_mlp = False: measured faster than a side stream)
        model.input_mlp(dense, out=pooled[:, : model.d_emb])

    def mlp():  # the output MLP + Dense(2, softmax): the critical path after the attention
        model.dense_output(model.output_mlp(pooled))

    steps = max(10, args.steps // 2)

    def fwd(p):  # the model's own forward
        return model(hu[p], ha[p], dense)

    eager_wall, _ = _time_stages([("forward", lambda: fwd(nxt("e")))], steps, 3)
    # hipGraphs (runtime.graphs): one per stage for the stage times, one per whole forward for the wall
    # number; the two resident input batches alternate, as in the eager loop
    from recommendflow_amd.runtime.graphs import CapturedGraph

    def enc_p(p):
        model.enc_q(hu[p], out=q)
        model.enc_a(ha[p], out=a)

    # the fused scorer (Esim.fused_scorer, gather path): the input MLP and the attention write the pooled row as bf16
    # + slice partials, the output MLP folds both LayerNorms and carries the head (no LayerNorm pass, no fp32 pooled)
    fused = model._gather_ok(hu[0], ha[0]) and model._fused_scorer_ok(dense)
    if fused:
        import recommendflow_amd.runtime.lib as RL

        W = model.pooled_width
        pb = torch.empty((B, W), dtype=torch.bfloat16, device="cuda")
        pst = torch.empty((B, W // 32, 2), device="cuda")

        def in_mlp():  # noqa: F811 — the fused forward's first launch
            model.input_mlp.forward_stats(dense, pb[:, : model.d_emb], pst, 0)

        def mlp():  # noqa: F811
            model.output_mlp.forward_prenormed_head(pb, pst, model.dense_output)

        def gat(qi, ai):
            eq, ea = model.enc_q, model.enc_a
            RL.call("rf_esim_gather_stats_fwd", RL.ptr(qi), RL.ptr(ai), RL.ptr(eq.table), eq.table.shape[0],
                    RL.ptr(ea.table), ea.table.shape[0], RL.DT_BF16, B, Ls, model.d, RL.ptr(pb), pb.stride(0),
                    model.d_emb, RL.ptr(pst), W // 32, model.d_emb // 32, RL.stream_ptr(None))
    else:
        def gat(qi, ai):
            model.attention_gather(qi, ai, pooled)
    in_mlp()
    mlp()
    g_enc = [CapturedGraph(lambda p=p: enc_p(p)) for p in (0, 1)]
    g_att, g_in, g_mlp = CapturedGraph(att), CapturedGraph(in_mlp), CapturedGraph(mlp)
    g_full = [CapturedGraph(lambda p=p: fwd(p)) for p in (0, 1)]

    # the forward's stages: with Esim.gather (single-valued slots, bf16 tables) the attention gathers the token
    # rows by id and the encoders' q / a are never written: input_mlp -> token_ids -> esim_gather_attention ->
    # mlp_scorer; the unfused stages (encoders writing q / a, then the attention) are timed beside them
    gather = model._gather_ok(hu[0], ha[0])
    stages = [("input_mlp", g_in.replay)]
    if gather:
        ids_p = [model.token_ids(hu[p], ha[p]) for p in (0, 1)]
        g_ids = [CapturedGraph(lambda p=p: model.token_ids(hu[p], ha[p])) for p in (0, 1)]
        g_gat = CapturedGraph(lambda: gat(ids_p[0][0], ids_p[0][1]))
        stages += [("token_ids", lambda: g_ids[nxt("i")].replay()), ("esim_gather_attention", g_gat.replay)]
    else:
        stages += [("sparse_encoders", lambda: g_enc[nxt("s")].replay()), ("esim_attention", g_att.replay)]
    stages += [("mlp_scorer", g_mlp.replay)]
    _, per = _time_stages(stages, steps, 3)
    _, per_u = _time_stages([("sparse_encoders", lambda: g_enc[nxt("s")].replay()), ("esim_attention", g_att.replay)],
                            steps, 3)
    wall, _ = _time_stages([("forward", lambda: g_full[nxt("f")].replay())], steps, 3)
    att_flops = 2 * Ls * Ls * 128 * 3 * B
    mlp_flops = sum(2 * dn.in_features * dn.units for dn in model.output_mlp.denses) * B + 2 * model.dense_output.in_features * 2 * B
    tok_bytes = sum(int(h.tok_bytes.numel()) + 4 * h.n_tokens for h in (hu[0], ha[0]))
    enc_bytes = 2 * (2 * B * Ls * 128 + B * Ls * 2 * 64 * 2) + tok_bytes
    cpu = None
    if args.cpu_seconds > 0:
        cpu = cpu_baseline_cfg3(model, q.view(B, Ls, 128), a.view(B, Ls, 128), dense, args.cpu_seconds)
    return {"examples_per_s": round(B / wall * 1e3, 1), "ms_per_step": round(wall, 4), "launch": "hipGraph",
            "eager_ms_per_step": round(eager_wall, 4), "cpu_baseline": cpu,
            "stage_ms": {k: round(v, 4) for k, v in per.items()},
            "gather_path": gather,
            "fused_scorer": fused,
            "unfused_stage_ms": {k: round(v, 4) for k, v in per_u.items()},
            "encoder_GBs": round(enc_bytes / per_u["sparse_encoders"] / 1e6, 1),
            "encoder_frac_of_measured_gather_ceiling": (
                round(enc_bytes / per_u["sparse_encoders"] / 1e6 / args.probes["gather_copy_128B_GBs"], 4)
                if isinstance(getattr(args, "probes", None), dict) and args.probes.get("gather_copy_128B_GBs") else None),
            "esim_TFLOPs": round(att_flops / per_u["esim_attention"] / 1e9, 1),
            "esim_mfma_frac_of_2500TF": round(att_flops / per_u["esim_attention"] / 1e9 / 2500, 4),
            "esim_gather_TFLOPs": round(att_flops / per["esim_gather_attention"] / 1e9, 1) if gather else None,
            "mlp_TFLOPs": round(mlp_flops / per["mlp_scorer"] / 1e9, 1),
            "stages_note": "each stage is its own replayed hipGraph (graph launch included); the forward runs "
                           "input_mlp -> token_ids -> esim_gather_attention (rows gathered by id inside the "
                           "attention kernel) -> mlp_scorer on one stream; unfused_stage_ms = the encoders writing "
                           "q / a and the attention reading them (encoder_GBs, esim_TFLOPs); mlp_scorer = output MLP "
                           "+ Dense(2, softmax); mlp_TFLOPs over those GEMMs; fused_scorer: the pooled row leaves the "
                           "input MLP and the attention as bf16 + 32-column slice partials and both output-MLP "
                           "LayerNorms and the head are folded into its two GEMMs (no norm pass, no fp32 pooled)",
            "config": "200 slots (100 q + 100 a) x 1M bins/hash, D=64 bf16 (tables 51.2 GB), L=100, d=128, "
                      "input_mlp 16->256->512, output_mlp 1280->1024->512, Dense(2, softmax), bf16 MFMA"}


def cpu_baseline_cfg3(model, q, a, dense, budget_s, sample=512):
    """cfg3's dense stages a.5-a.7 in float32 numpy / BLAS on the host (oracle.esim_scorer_f32) over the
    first `sample` examples of the GPU's own encoder outputs; all host threads (BLAS)."""
    from oracle import oracle as O

    def params(m):
        return [{"W": dn.weight.float().cpu().numpy().T.copy(), "b": dn.bias.cpu().numpy(), "gamma": nm.gamma.cpu().numpy(),
                 "beta": nm.beta.cpu().numpy()} for nm, dn in zip(m.norms, m.denses)]

    qs, as_, ds = (t[:sample].float().cpu().numpy() for t in (q, a, dense))
    pin, pout = params(model.input_mlp), params(model.output_mlp)
    Wo = model.dense_output.weight.float().cpu().numpy().T.copy()
    bo = model.dense_output.bias.cpu().numpy()
    cpu_model, ncpu = host_cpu()
    r = timed_runs(lambda: O.esim_scorer_f32(qs, as_, ds, pin, pout, Wo, bo), sample, budget_s / 2, warmup=2)
    usable, src = usable_cpus()
    omp = os.environ.get("OMP_NUM_THREADS")
    cores = min(int(omp), usable) if omp else usable
    return dict(r, unit="examples/s", cores=cores, cores_source=f"numpy BLAS threads: {'OMP_NUM_THREADS' if omp else 'all usable CPUs'}; {src}",
                kind="port", cpu=cpu_model,
                host_cpus=ncpu, sample=f"{r['runs']} x {sample} cfg3 examples through oracle.esim_scorer_f32 (SoftAttention, "
                                       f"ESIM combine/pool, input/output MLPs, Dense(2, softmax); float32 numpy/BLAS) "
                                       f"in {r['seconds']} s; the sparse encoders are not included")


def bench_dssm(args, enc, host):
    """cfg2 full forward: the same 229-slot fused table split into user (69) / ad (160) encoders + fp32
    towers [1024, 512, 256] selu/BatchNorm (exact-fp32 MFMA) + l2norm + dot."""
    import numpy as np
    import torch

    from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder
    from recommendflow_amd.config_parser.configuration import Configuration
    from recommendflow_amd.models.matching.dssm import Dssm
    from recommendflow_amd.runtime.batch import synthetic_batch

    conf = Configuration(os.path.join(ROOT, "tests", "golden", "conf", "base_recall_sdpa.yaml"))
    B = args.batch
    specs = enc.slots
    users = [i for i, f in enumerate(conf.features.hashing_features) if f.tower.value == "user"]
    ads = [i for i, f in enumerate(conf.features.hashing_features) if f.tower.value == "ad"]
    eu = FusedSparseEncoder([specs[i] for i in users], enc.dim, table=enc.table, row_base0=0)
    ea = FusedSparseEncoder([specs[i] for i in ads], enc.dim, table=enc.table,
                            row_base0=int(enc.host_desc[ads[0]]["row_base"][0]))
    model = Dssm(eu, ea, seed=5)
    mv = [bool(f.multivalued) for f in conf.features.hashing_features]
    hu = synthetic_batch(B, [mv[i] for i in users], seed=11, slot_ids=users).to("cuda")
    ha = synthetic_batch(B, [mv[i] for i in ads], seed=12, slot_ids=ads).to("cuda")
    xu = torch.empty((B, eu.out_width), device="cuda")
    xa = torch.empty((B, ea.out_width), device="cuda")

    def sparse():
        eu(hu, out=xu)
        ea(ha, out=xa)

    def towers():
        u, v = model.towers(xu, xa)
        (u * v).sum(-1)

    steps = max(5, args.steps // 5)
    eager_wall, _ = _time_stages([("forward", lambda: (sparse(), towers()))], steps, 2)
    from recommendflow_amd.runtime.graphs import CapturedGraph

    g_sp, g_tw, g_full = CapturedGraph(sparse), CapturedGraph(towers), CapturedGraph(lambda: (sparse(), towers()))
    _, per = _time_stages([("sparse_encoders", g_sp.replay), ("fp32_towers", g_tw.replay)], steps, 2)
    wall, _ = _time_stages([("forward", g_full.replay)], steps, 2)
    flops = model.flops_per_example() * B
    return {"examples_per_s": round(B / wall * 1e3, 1), "ms_per_step": round(wall, 4), "launch": "hipGraph",
            "eager_ms_per_step": round(eager_wall, 4),
            "stage_ms": {k: round(v, 4) for k, v in per.items()},
            "towers_TFLOPs_fp32": round(flops / per["fp32_towers"] / 1e9, 1),
            "towers_frac_of_157TF_fp32": round(flops / per["fp32_towers"] / 1e9 / 157.3, 4),
            "config": "base_recall_sdpa.yaml: 69 user + 160 ad slots, 10M x 64 fp32 table, towers [1024,512,256] "
                      "selu + BatchNorm fp32"}


def bench_sharded(args, specs, multi, rank, world):
    """cfg4, weak scaling: the cfg2 slot layout over a row-sharded fused fp32 table of
    shard_rows x P rows x shard_dim (owner = row mod P), shard_batch examples per GPU. One step =
    route (hash rows; hash-table dedup of the rows other ranks own; the counts' all-to-all and ONE host read)
    -> all-to-all ids -> owners gather -> all-to-all vectors -> pool (this rank's own rows read in place from
    its shard, the others from the receive buffer through the row map). Bit-identical to the unsharded kernel
    (tests/test_sharded_gpu.py). All ranks run; value = examples of all ranks / max-over-ranks time. Also
    the pipelined forward (2 micro-batches, async all-to-alls overlapping the other micro-batch's stages)."""
    import torch
    import torch.distributed as dist

    from recommendflow_amd.backend.encoder.sharded_encoder import LocalComm, ShardedFusedEncoder, TorchDistComm
    from recommendflow_amd.backend.encoder.sparse_encoder import SlotSpec
    from recommendflow_amd.runtime.batch import synthetic_batch

    P, B, D = world, args.shard_batch, args.shard_dim
    S = len(specs)
    n_bins = args.shard_rows * P // (2 * S)
    sp = [SlotSpec(s.name, n_bins, s.seeds, s.combiner, s.mask_empty) for s in specs]
    comm = TorchDistComm() if world > 1 else LocalComm()
    enc = ShardedFusedEncoder(sp, D, rank, P, comm=comm, seed=2024)
    host_b = [synthetic_batch(B, multi, seed=4321 + 1000 * rank + i) for i in range(2)]
    batches = [h.to("cuda") for h in host_b]
    out = torch.empty((B, enc.out_width), dtype=torch.float32, device="cuda")
    ev_names = ["route", "a2a_ids", "gather", "a2a_rows", "pool"]
    st = {}

    def step(i, ev=None):
        b = batches[i % 2]
        r, recv = enc.route_exchange(b, local_fast=enc.local_fast)  # hash route + counts exchange, one host sync
        if ev: ev[1].record()
        wanted = comm.exchange(r.local, r.counts, recv)
        if ev: ev[2].record()
        vec = enc.serve(wanted)
        if ev: ev[3].record()
        back = comm.exchange(vec, recv, r.counts)
        if ev: ev[4].record()
        enc.combine(b, r, back, out, local_fast=enc.local_fast)
        if ev: ev[5].record()
        st["req"], st["served"], st["logical"] = r.n_requests, int(wanted.shape[0]), r.n_logical
        st["row_map"] = r.row_map

    steps = max(5, args.steps // 5)
    for i in range(3):
        step(i)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(6)] for _ in range(steps)]

    def timed(fn):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            fn(i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def staged(i):
        evs[i][0].record()
        step(i, evs[i])

    el = timed(staged)
    stage = {n: round(sum(e[k].elapsed_time(e[k + 1]) for e in evs) / steps, 4) for k, n in enumerate(ev_names)}
    # the pipelined forward: 2 micro-batches, all-to-alls on RCCL's stream beside the other micro-batch's stages
    from recommendflow_amd.runtime.batch import split_examples

    micro = [[m.to("cuda") for m in split_examples(h, 2)] for h in host_b]
    mouts = [torch.empty((m.batch, enc.out_width), dtype=torch.float32, device="cuda") for m in micro[0]]
    for i in range(2):
        enc.forward_pipelined(micro[i % 2], mouts)
    el_pipe = timed(lambda i: enc.forward_pipelined(micro[i % 2], mouts))
    # the owner-side partial-pooling exchange (SURVEY §8e alternative): partial vectors per (unit, owner) return
    try:
        for i in range(2):
            enc.forward_partial(batches[i % 2], out)
        el_pp = timed(lambda i: enc.forward_partial(batches[i % 2], out))
    except Exception as e:  # noqa: BLE001 — the variant's failure must not cost the leg
        el_pp = None
        pp_err = f"{type(e).__name__}: {e}"[:200]
    row_b = D * 4
    xgmi = (st["req"] * (8 + row_b)) * (P - 1) / P if P > 1 else 0
    res = {"examples_per_s": round(B * P * steps / el, 1), "ms_per_step": round(el / steps * 1e3, 4),
           "pipelined_examples_per_s": round(B * P * steps / el_pipe, 1),
           "pipelined_ms_per_step": round(el_pipe / steps * 1e3, 4),
           "partial_pool_ms_per_step": round(el_pp / steps * 1e3, 4) if el_pp else pp_err,
           "stage_ms_rank0": stage, "gather_GBs": round(st["served"] * (2 * row_b + 8) / max(stage["gather"], 1e-6) / 1e6, 1),
           "a2a_bytes_per_rank_each_way": int(xgmi),
           "rows_read_by_pool": st["logical"], "rows_requested_after_dedup": st["req"],
           "rows_pooled_in_place": st["logical"] - st["req"] if P == 1 else None,
           "route": enc.route_mode + (" + local rows pooled in place" if enc.local_fast else ""),
           "config": f"cfg2 slots ({S}) over a {enc.table_rows}x{D} fp32 fused table row-sharded over {P} GPU(s) "
                     f"({enc.local_rows} rows/GPU), {B} examples/GPU (global {B * P}), owner = row mod P, "
                     f"hash-table dedup of the remote rows, this rank's rows pooled in place, RCCL all_to_all_single "
                     f"for ids and rows; pipelined = 2 micro-batches with async all-to-alls"}
    if not args.no_shard_train:
        res["train_step"] = bench_sharded_train(args, enc, batches, out, world)
    del enc, batches, out, micro, mouts
    torch.cuda.empty_cache()
    if world == 1 and args.sim_ranks > 1:
        try:
            res["simulated_p8" if args.sim_ranks == 8 else f"simulated_p{args.sim_ranks}"] = \
                bench_sharded_sim(args, specs, multi, args.sim_ranks)
        except Exception as e:  # noqa: BLE001 — a failed diagnostic leg must not cost the line
            res["simulated_p8"] = f"{type(e).__name__}: {e}"[:300]
        torch.cuda.empty_cache()
    return res


def bench_sharded_sim(args, specs, multi, P):
    """cfg4's remote-row path at P ranks, timed on ONE GPU: this GPU plays rank 0 of P with a
    LoopbackComm, so (P-1)/P of every batch's rows are remote and go route (hash-table dedup) -> id exchange ->
    owner gather -> row exchange -> pool through the row map; the all-to-alls are device copies of the same bytes
    (what xGMI would carry is reported beside them, not timed). Rank 0's shard is shard_rows x shard_dim fp32, the
    logical table P times that; shard_batch examples. Pooled values of remote rows come from the wrong shard (the
    loopback serves its own rows): timing only; the parity of this path is tests/test_sharded_gpu.py."""
    import torch

    from recommendflow_amd.backend.encoder.sharded_encoder import LoopbackComm, ShardedFusedEncoder
    from recommendflow_amd.backend.encoder.sparse_encoder import SlotSpec
    from recommendflow_amd.runtime.batch import synthetic_batch

    B, D = args.shard_batch, args.shard_dim
    S = len(specs)
    n_bins = args.shard_rows * P // (2 * S)
    sp = [SlotSpec(s.name, n_bins, s.seeds, s.combiner, s.mask_empty) for s in specs]

    class CountingLoopback(LoopbackComm):
        """LoopbackComm that also counts the bytes each exchange sends and times its device copy."""

        def __init__(self, world):
            super().__init__(world)
            self.reset()

        def reset(self):
            self.bytes, self.events = [], []

        def exchange(self, x, send_splits, recv_splits):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            y = x.clone()
            e1.record()
            self.bytes.append(x.numel() * x.element_size())
            self.events.append((e0, e1))
            return y

        def copy_ms(self):
            torch.cuda.synchronize()
            return sum(a.elapsed_time(b) for a, b in self.events)

    comm = CountingLoopback(P)
    enc = ShardedFusedEncoder(sp, D, 0, P, comm=comm, seed=2024)
    batches = [synthetic_batch(B, multi, seed=4321 + i).to("cuda") for i in range(2)]
    out = torch.empty((B, enc.out_width), dtype=torch.float32, device="cuda")
    names = ["route", "a2a_ids", "gather", "a2a_rows", "pool"]
    st = {}

    def step(i, ev=None):
        b = batches[i % 2]
        r, recv = enc.route_exchange(b, local_fast=enc.local_fast)
        if ev: ev[1].record()
        wanted = comm.exchange(r.local, r.counts, recv)
        if ev: ev[2].record()
        vec = enc.serve(wanted)
        if ev: ev[3].record()
        back = comm.exchange(vec, recv, r.counts)
        if ev: ev[4].record()
        enc.combine(b, r, back, out, local_fast=enc.local_fast)
        if ev: ev[5].record()
        st["req"], st["served"], st["logical"] = r.n_requests, int(wanted.shape[0]), r.n_logical
        st["row_map"] = r.row_map

    steps = max(5, args.steps // 5)
    for i in range(3):
        step(i)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(6)] for _ in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        evs[i][0].record()
        step(i, evs[i])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    stage = {n: round(sum(e[k].elapsed_time(e[k + 1]) for e in evs) / steps, 4) for k, n in enumerate(names)}
    row_b = D * 4
    # per-step bytes each way of the row-return exchange (ids out, rows back; the own-rank share never leaves
    # the GPU) and the owner-side partial-pooling exchange (entries out, one partial per (unit, owner) back), and
    # each mode's predicted step at P with the all-to-alls at xGMI's 7 x 153 GB/s per GPU in place of
    # the loopback copies (no overlap assumed: the plain forward runs them in line)
    xgmi = 7 * 153e9
    remote = (P - 1) / P
    comm.reset()
    step(0)
    torch.cuda.synchronize()
    row_bytes = [b * remote for b in comm.bytes]
    row_copy_ms = comm.copy_ms()
    el_ms = el / steps * 1e3
    row_pred = el_ms - row_copy_ms + sum(row_bytes) / xgmi * 1e3
    partial = {}
    try:
        for i in range(3):
            enc.forward_partial(batches[i % 2], out)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            enc.forward_partial(batches[i % 2], out)
        torch.cuda.synchronize()
        pp_ms = (time.perf_counter() - t0) / steps * 1e3
        comm.reset()
        enc.forward_partial(batches[0], out)
        torch.cuda.synchronize()
        pp_bytes = [b * remote for b in comm.bytes]
        pp_copy_ms = comm.copy_ms()
        pp_pred = pp_ms - pp_copy_ms + sum(pp_bytes) / xgmi * 1e3
        partial = {"ms_per_step": round(pp_ms, 4), "loopback_copy_ms": round(pp_copy_ms, 4),
                   "xgmi_bytes_each_way": {"entries_out": int(pp_bytes[0]), "partials_back": int(pp_bytes[1])},
                   "predicted_ms_at_xgmi": round(pp_pred, 4)}
    except Exception as e:  # noqa: BLE001
        partial = {"error": f"{type(e).__name__}: {e}"[:200]}
    pp_pred = partial.get("predicted_ms_at_xgmi")
    res_modes = {"row_return": {"ms_per_step": round(el_ms, 4), "loopback_copy_ms": round(row_copy_ms, 4),
                                "xgmi_bytes_each_way": {"ids_out": int(row_bytes[0]), "rows_back": int(row_bytes[1])},
                                "predicted_ms_at_xgmi": round(row_pred, 4)},
                 "partial_pool": partial,
                 "default_by_prediction": ("partial_pool" if pp_pred is not None and pp_pred < row_pred else "row_return"),
                 "xgmi_GBs_per_gpu": xgmi / 1e9}
    res = {"ms_per_step": round(el / steps * 1e3, 4), "examples_per_s_this_rank": round(B * steps / el, 1),
           "modes": res_modes,
           "stage_ms": stage, "rows_read_by_pool": st["logical"], "rows_requested_after_dedup": st["req"],
           "requests_local_in_place": int((st["row_map"] < 0).sum()),  # row_map bit 31: read from the own shard
           "requests_remote": int((st["row_map"] >= 0).sum()),
           "dedup_ratio": round(st["req"] / max(1, st["logical"]), 4),
           "gather_GBs": round(st["served"] * (2 * row_b + 8) / max(stage["gather"], 1e-6) / 1e6, 1),
           "xgmi_bytes_each_way_not_timed": int(st["req"] * (8 + row_b)),
           "config": f"rank 0 of P = {P} on one GPU (LoopbackComm: each all-to-all is a device copy of the same bytes), "
                     f"{enc.local_rows} x {D} fp32 shard of a {enc.table_rows}-row logical table, {B} examples, cfg2 slots"}
    del enc, batches, out
    return res


def bench_sharded_train(args, enc, batches, out, world):
    """cfg4 training step: forward_train (route, ids/rows all-to-all, pool) ->
    backward (rf_pool_rows_bwd on the requester, reverse all-to-all of (local id, grad) pairs,
    rf_segment_sum_rows on the owner) -> Keras Adam on the shard (dense semantics, deferred per row).
    Bit-exact vs the oracle (tests/test_sharded_gpu.py::test_simulated_backward_and_adam)."""
    import torch
    import torch.distributed as dist

    from recommendflow_amd.backend.optim import SparseAdam

    B = batches[0].batch
    # Keras' dense Adam on the shard, deferred per row: the rows this shard serves are replayed current before the
    # forward reads them (serve_hook), the gradient's rows before their update
    opt = SparseAdam(enc.shard, learning_rate=1e-4, deferred=True)
    enc.serve_hook = opt.prepare_ids
    g = torch.Generator(device="cuda").manual_seed(5 + enc.rank)
    dout = torch.randn((B, enc.out_width), generator=g, device="cuda") * 1e-3
    names = ["forward", "backward", "adam"]
    st = {}

    def step(i, ev=None):
        ctx = enc.forward_train(batches[i % 2], out=out)
        if ev: ev[1].record()
        sg = enc.backward(ctx, dout)
        if ev: ev[2].record()
        opt.apply(sg, rows_current=True)  # every gradient row was served, so replayed, this step
        if ev: ev[3].record()
        st["rows"] = sg.cap

    steps = max(5, args.steps // 5)
    for i in range(2):
        step(i)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        evs[i][0].record()
        step(i, evs[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    stage = {n: round(sum(e[k].elapsed_time(e[k + 1]) for e in evs) / steps, 4) for k, n in enumerate(names)}
    n_rows = int(opt.m.shape[0])
    enc.serve_hook = None
    del opt
    torch.cuda.empty_cache()
    return {"examples_per_s": round(B * enc.nranks * steps / el, 1), "ms_per_step": round(el / steps * 1e3, 4),
            "stage_ms_rank0": stage, "shard_rows": n_rows,
            "optimizer": "Keras Adam, dense semantics deferred per row (SparseAdam(deferred=True) + serve_hook; "
                         "tests/test_sharded_gpu.py::test_sharded_deferred_adam_equals_dense)"}


def bench_cascade(args, enc):
    """cfg5 on one GPU: recall (cfg2 towers: 69 user + 160 ad slots over the 10M x 64
    fp32 table, [1024, 512, 256]) over a catalog of `--catalog` items (Flat inner-product top-200,
    MFMA score blocks + rf_topk_merge) -> prerank (light interaction MLP, top-50) -> rank (cfg3 ESIM,
    100 + 100 slots x 1M bins, bf16 tables, fp16 MFMA attention) -> top-10, for 1024 users per step."""
    import numpy as np
    import torch

    from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec
    from recommendflow_amd.config_parser.configuration import Configuration
    from recommendflow_amd.models.cascade import Cascade
    from recommendflow_amd.models.matching.dssm import Dssm
    from recommendflow_amd.models.ranking.esim import Esim
    from recommendflow_amd.runtime.batch import synthetic_batch

    conf = Configuration(os.path.join(ROOT, "tests", "golden", "conf", "base_recall_sdpa.yaml"))
    feats = conf.features.hashing_features
    users = [i for i, f in enumerate(feats) if f.tower.value == "user"]
    ads = [i for i, f in enumerate(feats) if f.tower.value == "ad"]
    mv = [bool(f.multivalued) for f in feats]
    eu = FusedSparseEncoder([enc.slots[i] for i in users], enc.dim, table=enc.table, row_base0=0)
    ea = FusedSparseEncoder([enc.slots[i] for i in ads], enc.dim, table=enc.table,
                            row_base0=int(enc.host_desc[ads[0]]["row_base"][0]))
    dssm = Dssm(eu, ea, seed=5)
    Ls = 100
    esim = Esim([SlotSpec(f"u{i:03d}", 1_000_000, (2022, 2023)) for i in range(Ls)],
                [SlotSpec(f"a{i:03d}", 1_000_000, (2022, 2023)) for i in range(Ls)], n_dense=16, dim=64,
                table_dtype=torch.bfloat16, seed=3)
    cas = Cascade(dssm, esim, k_recall=200, k_prerank=50, k_final=10, seed=9)
    N, CB = args.catalog, 8192
    t0 = time.perf_counter()
    rb = [synthetic_batch(CB, [mv[i] for i in ads], seed=600 + j, slot_ids=ads).to("cuda") for j in range(2)]
    kb = [synthetic_batch(CB, [False] * Ls, seed=700 + j, slot_ids=range(Ls, 2 * Ls)).to("cuda") for j in range(2)]
    nb = (N + CB - 1) // CB
    cas.index_catalog([rb[j % 2] for j in range(nb)], [kb[j % 2] for j in range(nb)])
    cas.searcher.index = cas.searcher.index[:N].contiguous()
    cas.a_item = cas.a_item[:N].contiguous()
    torch.cuda.synchronize()
    index_s = time.perf_counter() - t0
    B = 1024
    ur = [synthetic_batch(B, [mv[i] for i in users], seed=800 + j, slot_ids=users).to("cuda") for j in range(2)]
    uk = [synthetic_batch(B, [False] * Ls, seed=900 + j, slot_ids=range(Ls)).to("cuda") for j in range(2)]
    dense = torch.randn(B, 16, device="cuda")
    for j in range(2):
        cas(ur[j % 2], uk[j % 2], dense)
    steps = max(3, args.steps // 10)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(steps):
        res = cas(ur[j % 2], uk[j % 2], dense)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    out = {"users_per_s": round(B / ms * 1e3, 1), "ms_per_step": round(ms, 3), "catalog_items": N,
           "catalog_index_s": round(index_s, 2), "pairs_ranked_per_s": round(B * 50 / ms * 1e3, 1),
           "config": f"1024 users/step; recall: cfg2 towers, Flat IP top-200 over {N} items (exact: fp32 lead blocks + rf_topk_merge, the rest screened in bf16 within its error bound and rescored in fp32; bit-identical to the block loop); "
                     "prerank: u*v -> Dense(64, relu) -> Dense(1), top-50; rank: cfg3 ESIM (fp16 attention) top-10"}
    del cas, esim, dssm, rb, kb, ur, uk
    torch.cuda.empty_cache()
    return out


def bench_cascade_sharded(args, specs, rank, world):
    """cfg5 as configured (BASELINE.json configs[4]): recall -> prerank -> rank with DATA-PARALLEL request
    batches (1024 users per rank per step) and the recall towers' sparse lookups on ROW-SHARDED tables (the
    cfg2 user / ad slot layouts, 10M x 64 fp32 rows in all, owner = row mod P, one RCCL all-to-all pair per
    lookup); the catalog index is encoded collectively (rank r: its 1/P slice) and all-gathered; prerank and
    the cfg3 ESIM ranker (fp16 attention, replicated tables) run on each rank's own candidates. Timed: a
    barrier, K steps, a barrier; users/s = users of all ranks / the max-over-ranks time."""
    import torch
    import torch.distributed as dist

    from recommendflow_amd.backend.encoder.sharded_encoder import LocalComm, ShardedFusedEncoder, TorchDistComm
    from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec
    from recommendflow_amd.config_parser.configuration import Configuration
    from recommendflow_amd.models.cascade import ShardedCascade
    from recommendflow_amd.models.matching.dssm import Dssm
    from recommendflow_amd.models.ranking.esim import Esim
    from recommendflow_amd.runtime.batch import synthetic_batch

    conf = Configuration(os.path.join(ROOT, "tests", "golden", "conf", "base_recall_sdpa.yaml"))
    feats = conf.features.hashing_features
    users = [i for i, f in enumerate(feats) if f.tower.value == "user"]
    ads = [i for i, f in enumerate(feats) if f.tower.value == "ad"]
    mv = [bool(f.multivalued) for f in feats]
    comm = TorchDistComm() if world > 1 else LocalComm()
    eu = ShardedFusedEncoder([specs[i] for i in users], args.dim, rank, world, comm=comm, seed=31)
    ea = ShardedFusedEncoder([specs[i] for i in ads], args.dim, rank, world, comm=comm, seed=32)
    # the towers' weights: a Dssm over two tiny stand-in encoders of the same output widths (never called)
    tiny = lambda sl: FusedSparseEncoder([SlotSpec(s.name, 2, (1, 2)) for s in sl], args.dim)
    dssm = Dssm(tiny([specs[i] for i in users]), tiny([specs[i] for i in ads]), seed=5)
    Ls = 100
    esim = Esim([SlotSpec(f"u{i:03d}", 1_000_000, (2022, 2023)) for i in range(Ls)],
                [SlotSpec(f"a{i:03d}", 1_000_000, (2022, 2023)) for i in range(Ls)], n_dense=16, dim=64,
                table_dtype=torch.bfloat16, seed=3)
    cas = ShardedCascade(dssm, esim, eu, ea, comm, k_recall=200, k_prerank=50, k_final=10, seed=9)
    N, CB = args.catalog, 8192
    nb = max(1, (N + CB - 1) // CB)
    per = (nb + world - 1) // world  # catalog batches per rank (every rank encodes the same count)
    t0 = time.perf_counter()
    rb = [synthetic_batch(CB, [mv[i] for i in ads], seed=600 + j, slot_ids=ads).to("cuda") for j in range(2)]
    kb = [synthetic_batch(CB, [False] * Ls, seed=700 + j, slot_ids=range(Ls, 2 * Ls)).to("cuda") for j in range(2)]
    cas.index_catalog([rb[(rank * per + j) % 2] for j in range(per)], [kb[j % 2] for j in range(per * world)])
    torch.cuda.synchronize()
    index_s = time.perf_counter() - t0
    B = 1024
    ur = [synthetic_batch(B, [mv[i] for i in users], seed=800 + 10 * rank + j, slot_ids=users).to("cuda") for j in range(2)]
    uk = [synthetic_batch(B, [False] * Ls, seed=900 + 10 * rank + j, slot_ids=range(Ls)).to("cuda") for j in range(2)]
    dense = torch.randn(B, 16, device="cuda")
    for j in range(2):
        cas(ur[j % 2], uk[j % 2], dense)
    steps = max(3, args.steps // 10)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(steps):
        cas(ur[j % 2], uk[j % 2], dense)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms = float(t.item()) / steps * 1e3
    out = {"users_per_s": round(B * world / ms * 1e3, 1), "ms_per_step": round(ms, 3), "ranks": world,
           "users_per_rank_per_step": B, "catalog_items": int(cas.searcher.index.shape[0]),
           "catalog_index_s": round(index_s, 2), "recall_table_rows": eu.table_rows + ea.table_rows,
           "recall_shard_rows_rank0": eu.local_rows + ea.local_rows,
           "config": f"DP {B} users/rank/step; recall towers over row-sharded cfg2 user/ad tables (P={world}, "
                     "RCCL all-to-all per lookup), catalog encoded per rank + all-gathered, Flat IP top-200; prerank "
                     "top-50; rank cfg3 ESIM (fp16 attention, replicated 1M-bin tables) top-10"}
    del cas, esim, dssm, eu, ea, rb, kb, ur, uk
    torch.cuda.empty_cache()
    return out


def bench_train(args, specs, multi):
    """one DSSM training step on cfg2 (base_recall_sdpa.yaml: 229 slots, 10M x 64 fp32 fused
    table, B = 4096, towers [1024, 512, 256], cosent_loss): fused encoder forward -> torch towers + our
    cosent kernel -> backward -> rf_fused_hash_embed_bwd (dedup sort-reduce) -> rf_adam_apply (Keras
    dense Adam over the whole table + m + v) and torch Adam on the towers. Also times the sparse stages
    alone, the towers' forward + backward alone, and the lazy-Adam variant of the table update."""
    import numpy as np
    import torch

    from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder
    from recommendflow_amd.config_parser.configuration import Configuration
    from recommendflow_amd.models.matching.dssm import TrainableDssm
    from recommendflow_amd.runtime import gemm as GM
    from recommendflow_amd.runtime.batch import synthetic_batch

    conf = Configuration(os.path.join(ROOT, "tests", "golden", "conf", "base_recall_sdpa.yaml"))
    n_user = sum(1 for f in conf.features.hashing_features if f.tower.value == "user")
    B = args.batch
    enc = FusedSparseEncoder(specs, args.dim, seed=2023)
    model = TrainableDssm(enc, n_user, learning_rate=1e-3, seed=7)
    batches = [synthetic_batch(B, multi, seed=555 + i).to("cuda") for i in range(2)]
    y = (torch.rand(B, generator=torch.Generator().manual_seed(0)) < 0.3).float().cuda()
    steps = max(5, args.steps // 5)
    wi = [0]

    def warm_step():
        model.step(batches[wi[0] % 2], y)
        wi[0] += 1

    _warm(warm_step)  # the clock back at load after the previous leg's host-side setup (_time_stages)
    t0 = time.perf_counter()
    for i in range(steps):
        loss = model.step(batches[i % 2], y)
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) / steps * 1e3
    # sparse stages alone (HIP events on the launch stream)
    dout = torch.randn((B, enc.out_width), device="cuda")
    out = torch.empty((B, enc.out_width), device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    from recommendflow_amd.backend.optim import SparseAdam

    dense_opt = SparseAdam(enc.table, learning_rate=1e-3)  # the one-launch dense step, timed as a stage
    acc = np.zeros(4)
    for i in range(steps):
        ev[0].record()
        enc(batches[i % 2], out=out)
        ev[1].record()
        g = enc.backward(batches[i % 2], dout, out=out)
        ev[2].record()
        dense_opt.apply(g)
        ev[3].record()
        model.sparse_opt.apply(g)  # deferred: replay of the gradient's rows + their update
        ev[4].record()
        torch.cuda.synchronize()
        acc += [ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]), ev[2].elapsed_time(ev[3]), ev[3].elapsed_time(ev[4])]
    acc /= steps
    n_uniq = g.count()
    del dense_opt
    # the r04 schedule for A/B: the whole-table untouched update on a side stream beside the towers
    split = TrainableDssm(enc, n_user, learning_rate=1e-3, seed=7, deferred_adam=False)
    wi[0] = 0
    _warm(lambda: (split.step(batches[wi[0] % 2], y), wi.__setitem__(0, wi[0] + 1)))
    t0 = time.perf_counter()
    for i in range(steps):
        split.step(batches[i % 2], y)
    torch.cuda.synchronize()
    split_ms = (time.perf_counter() - t0) / steps * 1e3
    del split

    lazy = SparseAdam(enc.table, lazy=True)
    for i in range(2):
        lazy.apply(g)
    torch.cuda.synchronize()
    ev[0].record()
    for i in range(steps):
        lazy.apply(g)
    ev[1].record()
    torch.cuda.synchronize()
    lazy_ms = ev[0].elapsed_time(ev[1]) / steps
    # the towers alone: forward + l2norm + loss + backward to the embedding gradient, then the towers' Adam
    xin = torch.randn((B, enc.out_width), generator=torch.Generator().manual_seed(3)).cuda() * 0.05
    model.train()
    tw = np.zeros(2)
    from recommendflow_amd.backend.blocks.train_mlp import towers_forward

    def tower_fb(xg):
        # the step's tower path: both towers layer by layer over column blocks of one input (towers_forward)
        tu, ta = towers_forward(xg, [(model.user_tower, 0, model.wu), (model.ad_tower, model.wu, model.wa)])
        uu = torch.nn.functional.normalize(tu, dim=-1, eps=1e-6)
        vv = torch.nn.functional.normalize(ta, dim=-1, eps=1e-6)
        model.loss_fn(y, uu, vv).backward()

    _warm(lambda: tower_fb(xin.detach().requires_grad_(True)), min_iters=1)
    model.dense_opt.zero_grad(set_to_none=True)
    for i in range(steps + 2):
        xg = xin.detach().requires_grad_(True)
        ev[0].record()
        tower_fb(xg)
        ev[1].record()
        model.dense_opt.step()
        ev[2].record()
        model.dense_opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        if i >= 2:
            tw += [ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])]
    tw /= steps
    # the same step with the table gradient's long rows summed as a fixed-order tree (RF_FLAG_TREE_REDUCE: within
    # SURVEY §8d's L 2^-23 sum|x| of the reference's CPU order instead of bit-exact with it)
    enc.tree_reduce = True
    try:
        for i in range(2):
            model.step(batches[i % 2], y)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            model.step(batches[i % 2], y)
        torch.cuda.synchronize()
        tree_ms = (time.perf_counter() - t0) / steps * 1e3
        ev[0].record()
        for i in range(steps):
            g = enc.backward(batches[i % 2], dout, out=out)
        ev[1].record()
        torch.cuda.synchronize()
        tree_bwd_ms = ev[0].elapsed_time(ev[1]) / steps
    finally:
        enc.tree_reduce = False
    tower_flops = 3 * 2 * B * sum(t.W[l].numel() for t in (model.user_tower, model.ad_tower) for l in range(len(t.units)))
    adam_bytes = enc.table.numel() * 4 * 6 + enc.table.shape[0] * 4 + n_uniq * (args.dim * 4 + 8)
    res = {"examples_per_s": round(B / step_ms * 1e3, 1), "ms_per_step": round(step_ms, 4), "loss": round(float(loss), 4),
           "sparse_stage_ms": {"fwd": round(acc[0], 4), "bwd_dedup": round(acc[1], 4), "adam_dense": round(acc[2], 4),
                               "adam_deferred": round(acc[3], 4), "adam_lazy": round(lazy_ms, 4)},
           "table_adam": "deferred (SparseAdam(deferred=True): exact dense Keras Adam, a row's missed untouched steps "
                         "replayed when it is next read; tests/test_train_step_gpu.py::test_deferred_table_adam_equals_dense)",
           "split_dense_adam": {"examples_per_s": round(B / split_ms * 1e3, 1), "ms_per_step": round(split_ms, 4),
                                "note": "the same exact step with the whole-table untouched update on a side stream "
                                        "beside the towers (rf_adam_untouched, the r04 schedule)"},
           "tower_stage_ms": {"fwd_bwd": round(tw[0], 4), "adam": round(tw[1], 4)},
           "tower_fwd_bwd_TFLOPs": round(tower_flops / tw[0] / 1e9, 1),
           "distinct_rows_per_step": n_uniq,
           "adam_dense_GBs": round(adam_bytes / acc[2] / 1e6, 1),
           "tree_reduce": {"examples_per_s": round(B / tree_ms * 1e3, 1), "ms_per_step": round(tree_ms, 4),
                           "bwd_dedup_ms": round(tree_bwd_ms, 4),
                           "note": "FusedSparseEncoder.tree_reduce = True (RF_FLAG_TREE_REDUCE): rows with > 256 positions "
                                   "summed as fixed-order partials + a pairwise tree, within |d| <= L 2^-23 sum|x| of the "
                                   "reference's CPU order (tests/test_train_gpu.py::test_bwd_tree_reduce_within_bound); the "
                                   "line's examples_per_s keeps the bit-exact CPU order"},
           "config": "cfg2 DSSM train step: 229 slots, 9999972x64 fp32 table (+ m, v), B=4096, towers [1024,512,256] "
                     "BatchNormalization(batch stats)/selu/dropout 0.3 on librf (train_mlp.TrainTower: BN folded into "
                     "the exact-fp32 MFMA GEMM rf_gemm_f32 for forward, dW and dx, SELU/dropout/BN backward kernels; "
                     f"torch GEMM fallbacks this run: {GM.torch_fallbacks}), "
                     "cosent_loss (HIP), Keras Adam (dense semantics, exact; deferred per row) on the table, Adam on the towers"}
    del model, enc, batches
    torch.cuda.empty_cache()
    return res


def bench_esim_train(args):
    """SURVEY §8f.1 for the ranker: one ESIM training step (models/ranking/esim_train.TrainableEsim; esim.py:45-53,69-89
    under model.fit, example/ranking_search/train.py:96-104) at the cfg3 shape: 100 user + 100 ad single-valued
    slots, token dim 128 (D = 64 per hash), 16 dense features, input_mlp [256, 512], output_mlp [1024, 512],
    Dropout 0.3, Dense(2, softmax) + sparse categorical CE, Keras Adam on the fused fp32 table (deferred, exact dense
    semantics) and on every dense parameter, B = 4096. The table has 100K bins per hash (not cfg3's 1M): Keras
    trains float32 tables, and 2 x 200 x 1M x 64 fp32 with Adam's m and v would be 307 GB, over one GPU's 288 GB."""
    import numpy as np
    import torch

    from recommendflow_amd.backend.encoder.sparse_encoder import SlotSpec
    from recommendflow_amd.models.ranking.esim_train import TrainableEsim
    from recommendflow_amd.runtime import lib as RL
    from recommendflow_amd.runtime.batch import synthetic_batch

    B, Ls, bins = args.batch, 100, 100_000
    user = [SlotSpec(f"u{i:03d}", bins, (2022, 2023)) for i in range(Ls)]
    ad = [SlotSpec(f"a{i:03d}", bins, (2022, 2023)) for i in range(Ls)]
    m = TrainableEsim(user, ad, 16, dim=64, seed=5)
    batches = [synthetic_batch(B, [False] * (2 * Ls), seed=311 + i, slot_ids=range(2 * Ls)).to("cuda") for i in range(2)]
    g = torch.Generator().manual_seed(4)
    dense = [torch.randn((B, 16), generator=g).cuda() for _ in range(2)]
    labels = [(torch.rand(B, generator=g) < 0.3).to(torch.int32).cuda() for _ in range(2)]
    steps = max(5, args.steps // 4)
    wi = [0]

    def one():
        i = wi[0] % 2
        wi[0] += 1
        return m.step(batches[i], dense[i], labels[i])

    _warm(one)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = one()
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) / steps * 1e3
    # the attention block's kernels alone (HIP events on the launch stream)
    x = m.enc(batches[0])
    Ld = Ls * 128
    pooled = torch.empty((B, m.pooled_width), device="cuda")
    aux = torch.empty((B, 256), device="cuda")
    dp = torch.randn((B, m.pooled_width), device="cuda")
    dx = torch.empty_like(x)
    ws = torch.empty(int(RL.load().rf_esim_train_ws_bytes(B, Ls, 128)), dtype=torch.uint8, device="cuda")
    st = RL.stream_ptr()

    def fwd():
        RL.call("rf_esim_train_fwd_f32", RL.ptr(x), RL.ptr(x) + 4 * Ld, B, Ls, 128, x.stride(0), 128, RL.ptr(pooled),
                pooled.stride(0), m.d_emb, RL.ptr(aux), st)

    def bwd():
        RL.call("rf_esim_train_bwd_f32", RL.ptr(x), RL.ptr(x) + 4 * Ld, B, Ls, 128, x.stride(0), 128, RL.ptr(pooled),
                pooled.stride(0), m.d_emb, RL.ptr(dp), dp.stride(0), m.d_emb, RL.ptr(aux), RL.ptr(dx), RL.ptr(dx) + 4 * Ld,
                dx.stride(0), 128, RL.ptr(ws), ws.numel(), st)

    _, per = _time_stages([("attention_fwd", fwd), ("attention_bwd", bwd)], max(10, args.steps // 2), 3)
    fl_f = 6.0 * Ls * Ls * 128 * B  # E, S q, S a
    fl_b = 18.0 * Ls * Ls * 128 * B  # E, S q, S a again; dS (2); dE q; S^T G_q, S^T G_a, dE^T a
    res = {"examples_per_s": round(B / step_ms * 1e3, 1), "ms_per_step": round(step_ms, 4), "loss": round(float(loss.item()), 4),
           "stage_ms": {k: round(v, 4) for k, v in per.items()},
           "attention_fwd_TFLOPs_fp32": round(fl_f / per["attention_fwd"] / 1e9, 1),
           "attention_bwd_TFLOPs_fp32": round(fl_b / per["attention_bwd"] / 1e9, 1),
           "attention_frac_of_157TF_fp32": round((fl_f + fl_b) / (per["attention_fwd"] + per["attention_bwd"]) / 1e9 / 157.3, 4),
           "config": "cfg3 shape: 100 + 100 single-valued slots, 100K bins per hash (fp32 fused table 40M x 64 + Adam m, v), "
                     "d = 128, dense 16 -> [256, 512], pooled 1280 -> [1024, 512] -> Dense(2, softmax), Dropout 0.3, "
                     "B = 4096; exact fp32 on librf (rf_esim_train_{fwd,bwd}_f32 on v_mfma_f32_16x16x4_f32, rf_gemm_f32, "
                     "LayerNorm / gelu+dropout / CE kernels, Keras Adam)"}
    del m, batches, x, dx, ws
    torch.cuda.empty_cache()
    return res


def bench_pipe(args, enc, specs, multi):
    """cfg2 examples as TFRecord files (the reference's on-disk format, make_tfrecord.py:142,
    read by TFRecordDataset(compression_type), dataloader.py:567) -> the fused encoder, three ways:
      gzip_host    GZIP files, C++ inflate + framing + tf.train.Example parse into pinned buffers,
                   side-stream H2D (the host decode rate alone is reported too);
      gzip_device  GZIP files, C++ inflate + framing on the host, Example parse on the GPU;
      none_device  uncompressed files (compression_type=""), host framing + CRC only, records streamed
                   to HBM as they are and parsed there (rf_tfr_parse_device).
    Each end-to-end rate has the encoder consuming every batch (decode, copy and kernels overlap).
    Files are written first (zlib level 1 for GZIP; not timed) and read from the page cache."""
    import shutil
    import tempfile
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np
    import torch

    from recommendflow_amd.runtime import tfrecord as T
    from recommendflow_amd.runtime.batch import synthetic_batch

    n_files = max(1, min(16, args.pipe_threads))  # one part file per reader thread (tf.data interleave)
    passes = 4  # end-to-end legs read the file list 4 times (epochs): the startup fill, when every slot inflates its
    # first file before the interleave's first batch, is paid once, as in a training job
    per = max(1, args.pipe_examples // n_files)
    fspecs = [T.FeatureSpec(s.name, T.BYTES, T.SEQ, "") for s in specs] + [T.FeatureSpec("label", T.FLOAT, T.SCALAR, 0.0)]
    tmp = tempfile.mkdtemp(prefix="rf_pipe_", dir="/tmp")
    paths = {c: [os.path.join(tmp, f"part-{f:02d}.tfrecord{'.gz' if c == 'GZIP' else ''}") for f in range(n_files)]
             for c in ("GZIP", None)}

    def write(f):
        hb = synthetic_batch(per, multi, seed=777 + f)
        fb = T.FeatureBatch(per, hb, [s.name for s in specs], None, None, np.zeros((per, 0), np.int64), [],
                            np.ones((per, 1), np.float32), ["label"])
        data, off = T.encode_examples(fspecs, fb)
        for c in ("GZIP", None):
            with T.TFRecordWriter(paths[c][f], c, level=1) as w:
                w.write_many(data, off)
        return int(off[-1])

    steady = {}

    def e2e(comp, parse, leg=None):
        out = torch.empty((B, enc.out_width), dtype=torch.float32, device="cuda")
        pipe = T.FeaturePipe(paths[comp] * passes, fspecs, B, thread_num=thr, prefetch=3, compression_type=comp,
                             parse=parse)
        torch.cuda.synchronize()
        t0, m, t1, m1 = time.perf_counter(), 0, None, 0
        for fb in pipe:
            enc(fb.sparse, out=out[: fb.batch])
            m += fb.batch
            if t1 is None:  # the pipeline is full once the first batch is out
                t1, m1 = time.perf_counter(), m
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        pipe.close()
        if leg is not None and t1 is not None and t2 > t1:
            steady[leg] = round((m - m1) / (t2 - t1), 1)
        return round(m / (t2 - t0), 1)

    try:
        with ThreadPoolExecutor(n_files) as ex:
            raw = sum(ex.map(write, range(n_files)))
        gz = sum(os.path.getsize(p) for p in paths["GZIP"])
        B, thr = args.batch, args.pipe_threads
        rd = T.TFRecordReader(paths["GZIP"], fspecs, B, thread_num=thr, pinned=True)
        cols, n = rd.new_columns(), 0
        t0 = time.perf_counter()
        while True:
            r = rd.read_into(cols)
            if r is None:
                break
            cols, c = r
            n += c.batch
        dec = time.perf_counter() - t0
        rd.close()
        e2e("GZIP", "host")  # warm the pinned pools and the allocator
        legs = {"gzip_host": e2e("GZIP", "host", "gzip_host"), "gzip_device": e2e("GZIP", "device", "gzip_device")}
        e2e(None, "device")
        legs["none_device"] = e2e(None, "device", "none_device")
        return {"pipe_to_encoder_examples_per_s": max(legs.values()), "legs_examples_per_s": legs,
                "legs_after_first_batch_examples_per_s": steady,
                "decode_examples_per_s": round(n / dec, 1), "decode_raw_GBs": round(raw / dec / 1e9, 3),
                "none_device_raw_GBs": round(legs["none_device"] * raw / n / 1e9, 3),
                "examples": n, "examples_e2e": passes * n, "threads": thr,
                "bytes_per_example_raw": round(raw / n, 1), "bytes_per_example_gzip": round(gz / n, 1),
                "config": f"{n_files} TFRecord files x {per} cfg2 examples (229 bytes features + label), batch {B}, "
                          f"{thr} reader threads, pinned ring of 3, side-stream H2D, fused encoder consumes; end-to-end legs read "
                          f"the file list {passes} times; single-member GZIP inflated by libdeflate (whole file, next files "
                          f"opened ahead); "
                          f"decode_* = host C++ parse alone on the GZIP files; legs_after_first_batch_* = the same runs timed from "
                          f"the first batch out (pipeline full: every slot has inflated its first file) to the last"}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def _event_ms(fn, reps, warmup=3):
    """Mean ms per call of fn(i) over `reps` calls, HIP events on the current stream."""
    import torch

    for i in range(warmup):
        fn(i)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for i in range(reps):
        fn(warmup + i)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def bench_probes(args):
    """The ceilings the roofline is stated against, both from librf.so:
      stream_copy_GBs       rf_stream_copy, float4 STREAM copy of 4 GiB (read + write bytes / time; the best of its four
                            variants): the box's
                            achievable streaming HBM rate, reported beside the 8 TB/s spec as roofline.peak_measured;
      gather_copy_{R}B_GBs  rf_gather_probe: uniformly random R-byte rows of a `--probe-table-gb` table (far past the
                            256 MiB Infinity Cache; a new row set every call) copied to a contiguous output, as many
                            rows as one batch of the encoder reads (R = 128: cfg3's bf16 D=64 rows, 2 x 200 x 4096;
                            R = 256: cfg2's fp32 D=64 rows, 2 x 439 x 4096), best of 4 / 8 / 16 rows in flight per
                            team; bytes = read + write. gather_read_*: the same reads without the copy."""
    import torch

    from recommendflow_amd.runtime import lib as L

    res = {}
    n = 4 << 30
    src = torch.empty(n, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    best = {}
    for var in range(4):  # the best of four copy kernels is the measured peak
        ms = _event_ms(lambda i, var=var: L.call("rf_stream_copy", L.ptr(src), L.ptr(dst), n, var, L.stream_ptr()), 10)
        best[var] = round(2 * n / ms / 1e6, 1)
    res["stream_copy_GBs"] = max(best.values())
    res["stream_copy_variants_GBs"] = best
    res["stream_copy_bytes"] = n
    del src, dst
    torch.cuda.empty_cache()
    tb = int(args.probe_table_gb * (1 << 30)) // 512 * 512
    table = torch.empty(tb, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    res["table_bytes"] = tb
    for rb, nread in ((128, 2 * 200 * args.batch), (256, 2 * 439 * args.batch)):
        out = torch.empty(nread * rb, dtype=torch.uint8, device="cuda")
        for mode, o in (("copy", out), ("read", None)):
            best, best_g = 0.0, None
            for g in (4, 8, 16):
                ms = _event_ms(lambda i, g=g, o=o: L.call("rf_gather_probe", L.ptr(table), tb // rb, rb, nread, g,
                                                        0x5eed0000 + 977 * i + g, L.ptr(o), L.ptr(sink), L.stream_ptr()), 10)
                gbs = nread * rb * (2 if o is not None else 1) / ms / 1e6
                if gbs > best:
                    best, best_g = gbs, g
            res[f"gather_{mode}_{rb}B_GBs"] = round(best, 1)
            res[f"gather_{mode}_{rb}B_in_flight"] = best_g
        res[f"gather_{rb}B_rows_per_call"] = nread
        del out
    del table, sink
    torch.cuda.empty_cache()
    return res


def bench_uniform(args, enc, multi, rank, out):
    """The headline kernel on uniformly random ids over [1, 1e6] instead of Zipf(1.1) (the
    no-locality worst case): same slots, table, batch and timing protocol (50 warm-up launches, HIP events)."""
    import torch

    from recommendflow_amd.runtime.batch import synthetic_batch

    host = [synthetic_batch(args.batch, multi, seed=91234 + rank * 1000 + i, uniform=True) for i in range(args.batches)]
    dev = [h.to("cuda") for h in host]
    algo = [enc.algorithmic_bytes(h) for h in host]
    for i in range(args.warmup):
        enc(dev[i % len(dev)], out=out)
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    torch.cuda.synchronize()
    ev[0].record()
    for i in range(args.steps):
        enc(dev[i % len(dev)], out=out)
    ev[1].record()
    torch.cuda.synchronize()
    k = ev[0].elapsed_time(ev[1]) / args.steps / 1e3  # the headline's window timing
    by = sum(algo[i % len(algo)] for i in range(args.steps)) / args.steps
    ach = by / k / 1e9
    res = {"ids": "uniform [1, 1e6]", "kernel_ms": round(k * 1e3, 4), "examples_per_s_kernel": round(args.batch / k, 1),
           "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
           "algorithmic_bytes_per_launch": int(by)}
    del dev
    return res


def bench_cfg1(args):
    """cfg1 (BASELINE.json configs[0]): demo_conf.yaml two-tower matching end to end — 4096 synthetic examples
    of its working features written as GZIP TFRecord by the build's writer (make_tfrecord.py:142), read back by
    FeaturePipe (device parse), scored by ConfTwoTower (get_preprocess_layers operators + BN/selu towers).
    Plumbing: the rate is dominated by the tiny batches and the per-batch host work; parity is tested in
    tests/test_cfg1_gpu.py."""
    import shutil
    import tempfile

    import torch

    from recommendflow_amd.config_parser.configuration import Configuration
    from recommendflow_amd.models.matching.two_tower import ConfTwoTower
    from recommendflow_amd.runtime import tfrecord as T
    from recommendflow_amd.runtime.batch import synthetic_demo_rows

    conf = Configuration(os.path.join(ROOT, "tests", "golden", "conf", "demo_conf.yaml"))
    specs = T.build_feature_description(conf)
    n, B = 4096, 1024
    tmp = tempfile.mkdtemp(prefix="rf_cfg1_", dir="/tmp")
    try:
        path = os.path.join(tmp, "demo-part-0.tfrecord.gz")
        data, off = T.encode_examples(specs, T.columns_from_rows(specs, synthetic_demo_rows(n, 2024)))
        with T.TFRecordWriter(path, "GZIP") as w:
            w.write_many(data, off)
        model = ConfTwoTower(conf, seed=1)

        def run():
            pipe = T.FeaturePipe([path], specs, B, thread_num=1, compression_type="GZIP", parse="device")
            m = 0
            for fb in pipe:
                model(fb)
                m += fb.batch
            torch.cuda.synchronize()
            pipe.close()
            return m

        run()
        t0 = time.perf_counter()
        m = run()
        dt = time.perf_counter() - t0
        return {"examples_per_s": round(m / dt, 1), "examples": m, "batch": B, "file_bytes": os.path.getsize(path),
                "config": "demo_conf.yaml working features (2 user + 3 ad incl. app_id hashing 3000x16 sum), GZIP "
                          "TFRecord -> FeaturePipe(device parse) -> ConfTwoTower towers [64, 32] selu/BN fp32, l2norm, dot"}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def host_cpu():
    """CPU model name and logical CPU count of this host (the 'lscpu' model line, from /proc/cpuinfo)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model, os.cpu_count() or 1


def usable_cpus():
    """The CPUs this process may use: its scheduler affinity (os.sched_getaffinity), capped by a cgroup CPU quota
    when one is set (cgroup v2 cpu.max, v1 cfs_quota / cfs_period). Returns (count, how it was derived)."""
    import math

    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    n = aff if quota is None else max(1, min(aff, math.ceil(quota)))
    src = f"os.sched_getaffinity(0) = {aff} CPUs" + ("" if quota is None else f", cgroup CPU quota {quota:g}")
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp:
        src += f" (OMP_NUM_THREADS={omp} in the environment, not used)"
    return n, src


def timed_runs(fn, examples, budget_s, warmup=5, min_runs=5):
    """SURVEY §8d CPU protocol: `warmup` untimed runs, then runs until budget_s has passed (at least
    min_runs); examples/s as the total rate, the median and the p90 of the per-run rates."""
    import numpy as np

    for _ in range(warmup):
        fn()
    ts = []
    t0 = time.perf_counter()
    while len(ts) < min_runs or time.perf_counter() - t0 < budget_s:
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    rates = examples / np.asarray(ts)
    return {"value": round(examples * len(ts) / sum(ts), 1), "median": round(float(np.median(rates)), 1),
            "p90": round(float(np.percentile(rates, 90)), 1), "runs": len(ts), "seconds": round(sum(ts), 2)}


def cpu_baseline(enc, hb, budget_s):
    """The C oracle (OpenMP) on the same batch: examples/s, median and p90 per batch."""
    from oracle import oracle as O

    threads, cores_src = usable_cpus()
    model, ncpu = host_cpu()
    table = enc.table.cpu().numpy()
    r = timed_runs(lambda: O.fused_hash_embed(enc.host_desc, hb.tok_bytes, hb.tok_off, hb.bag_off, hb.lmax, hb.batch,
                                              table, enc.dim, enc.out_width, n_threads=threads), hb.batch, budget_s)
    return dict(r, unit="examples/s", cores=threads, cores_source=cores_src, kind="port", cpu=model, host_cpus=ncpu,
                sample=f"{r['runs']} x one {hb.batch}-example cfg2 batch through oracle/rf_oracle.c "
                       f"(orf_fused_hash_embed_fwd, OpenMP {threads} threads, gcc -O3) after 5 warm-up runs, "
                       f"{r['seconds']} s; median / p90 are per-batch rates")


def bench_h2d(args, enc, host):
    """cfg2 with the CSR batches starting in PINNED HOST memory (BASELINE.md §2's second number): batch
    i+1 is copied H2D on a side stream into the other of two static device buffers while the fused kernel
    runs on batch i (double buffering, stream-ordered by events). Not the headline (inputs resident)."""
    import torch

    from recommendflow_amd.runtime.graphs import StaticSparseBatch

    pinned = [[torch.from_numpy(a).pin_memory() for a in (h.tok_bytes, h.tok_off, h.bag_off, h.lmax)] for h in host]
    cap_b = max(len(h.tok_bytes) for h in host)
    cap_t = max(h.n_tokens for h in host)
    bufs = [StaticSparseBatch(host[0], cap_b, cap_t) for _ in range(2)]
    out = torch.empty((args.batch, enc.out_width), dtype=torch.float32, device="cuda")
    cs, comp = torch.cuda.Stream(), torch.cuda.current_stream()
    copied = [torch.cuda.Event() for _ in range(2)]
    consumed = [torch.cuda.Event() for _ in range(2)]
    nbytes = sum(int(t.numel() * t.element_size()) for t in pinned[0])

    def issue_copy(i):
        k, (tb, to, bo, lm) = i & 1, pinned[i % len(pinned)]
        with torch.cuda.stream(cs):
            cs.wait_event(consumed[k])
            b = bufs[k]
            b.tok_bytes[: tb.numel()].copy_(tb, non_blocking=True)
            b.tok_off[: to.numel()].copy_(to, non_blocking=True)
            b.bag_off.copy_(bo, non_blocking=True)
            b.lmax.copy_(lm, non_blocking=True)
            copied[k].record(cs)

    def run(n):
        issue_copy(0)
        for i in range(n):
            if i + 1 < n:
                issue_copy(i + 1)
            comp.wait_event(copied[i & 1])
            enc(bufs[i & 1], out=out)
            consumed[i & 1].record(comp)

    run(8)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"examples_per_s": round(args.batch * args.steps / el, 1), "ms_per_step": round(el / args.steps * 1e3, 4),
            "h2d_bytes_per_batch": nbytes, "h2d_GBs": round(nbytes * args.steps / el / 1e9, 2),
            "config": "cfg2 encoder, CSR batches in pinned host memory, H2D on a side stream double-buffered "
                      "against the fused kernel (PCIe-inclusive; the headline value keeps inputs in HBM)"}


if __name__ == "__main__":
    main()
