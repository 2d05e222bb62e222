"""Feature-pipe probe (host only): writes cfg2-shaped TFRecord files (GZIP and plain), then times
(1) zlib inflate alone per file, (2) the C++ reader's decode into columns, for both compressions.
Usage: python tools/pipe_probe.py [--files 8] [--per 2048] [--threads 8]"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from recommendflow_amd.config_parser.configuration import Configuration  # noqa: E402
from recommendflow_amd.runtime import tfrecord as T  # noqa: E402
from recommendflow_amd.runtime.batch import synthetic_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=8)
    ap.add_argument("--per", type=int, default=2048)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--modes", default="GZIP,NONE")
    a = ap.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    feats = Configuration(os.path.join(root, "tests", "golden", "conf", "base_recall_sdpa.yaml")).features.hashing_features
    specs, multi = feats, [bool(f.multivalued) for f in feats]
    fspecs = [T.FeatureSpec(s.name, T.BYTES, T.SEQ, "") for s in specs] + [T.FeatureSpec("label", T.FLOAT, T.SCALAR, 0.0)]
    tmp = tempfile.mkdtemp(prefix="rf_pprobe_", dir="/tmp")
    res = {}
    try:
        encs = []
        for f in range(a.files):
            hb = synthetic_batch(a.per, multi, seed=777 + f)
            fb = T.FeatureBatch(a.per, hb, [s.name for s in specs], None, None, np.zeros((a.per, 0), np.int64), [],
                                np.ones((a.per, 1), np.float32), ["label"])
            encs.append(T.encode_examples(fspecs, fb))
        raw = sum(int(off[-1]) for _, off in encs)
        n = a.files * a.per
        for mode in a.modes.split(","):
            ext = ".gz" if mode == "GZIP" else ""
            paths = [os.path.join(tmp, f"part-{f:02d}.tfrecord{ext}") for f in range(a.files)]
            for p, (data, off) in zip(paths, encs):
                with T.TFRecordWriter(p, mode, level=1) as w:
                    w.write_many(data, off)
            r = {"file_bytes_per_example": round(sum(os.path.getsize(p) for p in paths) / n, 1)}
            if mode == "GZIP":
                def inf(p):
                    with open(p, "rb") as fh:
                        d = fh.read()
                    t0 = time.perf_counter()
                    out = zlib.decompress(d, 16 + zlib.MAX_WBITS)
                    return len(out), time.perf_counter() - t0
                one = [inf(p) for p in paths[:2]]
                r["zlib_inflate_1thread_GBs"] = round(sum(x for x, _ in one) / sum(t for _, t in one) / 1e9, 3)
            for thr in sorted({1, a.threads}):
                rd = T.TFRecordReader(paths, fspecs, a.batch, thread_num=thr, compression_type=mode, pinned=False)
                cols, m = rd.new_columns(), 0
                t0 = time.perf_counter()
                while True:
                    x = rd.read_into(cols)
                    if x is None:
                        break
                    cols, c = x
                    m += c.batch
                dt = time.perf_counter() - t0
                rd.close()
                r[f"decode_t{thr}_ex_per_s"] = round(m / dt, 1)
                r[f"decode_t{thr}_raw_GBs"] = round(raw / dt / 1e9, 3)
            res[mode] = r
        res["raw_bytes_per_example"] = round(raw / n, 1)
        print(json.dumps(res, indent=1))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
