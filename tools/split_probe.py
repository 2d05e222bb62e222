"""Headline encoder split probe (diagnostics): cfg2's 229 slots timed as one fused launch against the 198 single-valued
slots and the 31 multi-valued slots launched separately (single-token kernel / fused kernel), one after the other and
concurrently on two streams. HIP events on the main stream; the side stream joins it before the end event.
    python tools/split_probe.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec  # noqa: E402
from recommendflow_amd.config_parser.configuration import Configuration  # noqa: E402
from recommendflow_amd.runtime.batch import synthetic_batch  # noqa: E402


def timeit(fn, reps=100, warm_s=0.3):
    import time
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < warm_s:
        fn()
        n += 1
        if n % 8 == 0:
            torch.cuda.synchronize()
    s = [torch.cuda.Event(enable_timing=True) for _ in range(reps)]
    e = [torch.cuda.Event(enable_timing=True) for _ in range(reps)]
    torch.cuda.synchronize()
    for i in range(reps):
        s[i].record()
        fn()
        e[i].record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in zip(s, e))
    return round(sum(t) / len(t), 4), round(t[len(t) // 2], 4)


def main():
    conf = Configuration(os.path.join(ROOT, "tests", "golden", "conf", "base_recall_sdpa.yaml"))
    feats = conf.features.hashing_features
    S = len(feats)
    nb = 10_000_000 // (2 * S)
    specs = [SlotSpec(f.name, nb, tuple(f.hash_seeds), "sum") for f in feats]
    multi = [bool(f.multivalued) for f in feats]
    enc = FusedSparseEncoder(specs, 64, seed=1)
    si = [i for i in range(S) if not multi[i]]
    mi = [i for i in range(S) if multi[i]]
    enc_s = FusedSparseEncoder([specs[i] for i in si], 64, table=enc.table)
    enc_m = FusedSparseEncoder([specs[i] for i in mi], 64, table=enc.table)
    res = {"slots": S, "single": len(si), "multi": len(mi)}
    for name, kw in [("zipf", {}), ("uniform", {"uniform": True})]:
        hb = synthetic_batch(4096, multi, seed=1234, **kw)
        db = hb.to("cuda")
        hs = synthetic_batch(4096, [False] * len(si), seed=1234, slot_ids=si, **kw)
        hm = synthetic_batch(4096, [True] * len(mi), seed=1235, slot_ids=mi, **kw)
        ds, dm = hs.to("cuda"), hm.to("cuda")
        out = torch.empty((4096, enc.out_width), device="cuda")
        os_ = torch.empty((4096, enc_s.out_width), device="cuda")
        om = torch.empty((4096, enc_m.out_width), device="cuda")
        side = torch.cuda.Stream()

        def both_seq():
            enc_s(ds, out=os_)
            enc_m(dm, out=om)

        def both_conc():
            ev = torch.cuda.Event()
            ev.record()
            side.wait_event(ev)
            with torch.cuda.stream(side):
                enc_s(ds, out=os_)
            enc_m(dm, out=om)
            ev2 = torch.cuda.Event()
            ev2.record(side)
            torch.cuda.current_stream().wait_event(ev2)

        def single_fused():
            enc_s.single_token = False
            enc_s(ds, out=os_)
            enc_s.single_token = True

        r = {"all_fused": timeit(lambda: enc(db, out=out)),
             "single_slots_single_kernel": timeit(lambda: enc_s(ds, out=os_)),
             "single_slots_fused_kernel": timeit(single_fused),
             "multi_slots_fused_kernel": timeit(lambda: enc_m(dm, out=om)),
             "split_sequential": timeit(both_seq),
             "split_concurrent": timeit(both_conc)}
        r["bytes_all"] = enc.algorithmic_bytes(hb)
        r["bytes_single"] = enc_s.algorithmic_bytes(hs)
        r["bytes_multi"] = enc_m.algorithmic_bytes(hm)
        res[name] = r
        print(json.dumps({name: r}), flush=True)


if __name__ == "__main__":
    main()
