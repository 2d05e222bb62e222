"""Static instruction mix of one kernel in a hipcc -S listing (diagnostics).
    python tools/isa_stats.py <file.s> <symbol-substring> [--dump]
Counts by class (MFMA, VALU, transcendental, LDS, VMEM, SALU, waits, barriers) over the whole body, plus the
kernel's VGPR / AGPR / LDS figures from its metadata.
"""
import re
import sys
from collections import Counter


def body(lines, key):
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\S*:", l) and key in l.split(":")[0]:
            start = i
        elif start is not None and l.startswith(".Lfunc_end"):
            return lines[start:i + 1]
    raise SystemExit(f"{key}: not found")


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")):
        return "trans"
    if op.startswith("v_permlane"):
        return "permlane"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return None


def main():
    path, key = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    b = body(lines, key)
    c, ops = Counter(), Counter()
    for l in b:
        t = l.strip()
        if not t or t.startswith((";", ".", "_")) or t.endswith(":"):
            continue
        op = t.split()[0]
        k = classify(op)
        if k:
            c[k] += 1
            ops[op] += 1
    print(b[0].split(":")[0][:160])
    print(dict(c))
    for op, n in ops.most_common(40):
        print(f"  {n:6d} {op}")
    meta = "\n".join(lines)
    name = b[0].split(":")[0]
    m = re.search(r"\.name:\s+" + re.escape(name) + r".*?(?=\n\s+- \.|\Z)", meta, re.S)
    if m:
        for f in ("vgpr_count", "agpr_count", "sgpr_count", "group_segment_fixed_size", "private_segment_fixed_size"):
            mm = re.search(r"\." + f + r":\s+(\d+)", meta[m.start() - 4000:m.end()])
    for l in lines:
        if name in l and ("NumVgprs" in l or "Occupancy" in l):
            print(l)
    if "--dump" in sys.argv:
        print("\n".join(b))


if __name__ == "__main__":
    main()
