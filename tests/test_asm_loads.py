"""Build-time guard for the register-staged GEMM (rf_dense.hip gemm_kernel): its next-stage tile loads are
inline asm the compiler does not track, so no instruction may read their destination registers before the
explicit `s_waitcnt vmcnt(0)` that precedes the LDS stores. Compiles the device code to assembly (hipcc -S,
no GPU needed) and checks every instantiation's main loop."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_gemm_kernel_asm_loads_are_not_read_before_their_wait(tmp_path):
    src = os.path.join(ROOT, "recommendflow_amd", "csrc", "rf_dense.hip")
    asm = tmp_path / "dense.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                    "--cuda-device-only", "-S", src, "-o", str(asm)], check=True, capture_output=True, timeout=600)
    text = asm.read_text()
    kernels = re.findall(r"^(_ZN12_GLOBAL__N_1\d+gemm_kernelI\w+):", text, flags=re.M)
    assert len(kernels) >= 8, kernels
    for k in kernels:
        body = text[text.index(k + ":"):]
        body = body[:body.index("s_endpgm")]
        lines = body.split("\n")
        loop = [i for i, l in enumerate(lines) if "Inner Loop Header" in l]
        assert loop, k
        regs, reads = set(), []
        for line in lines[loop[0]:]:
            m = re.search(r"global_load_dwordx4 v\[(\d+):(\d+)\]", line)
            if m:
                regs.update(range(int(m.group(1)), int(m.group(2)) + 1))
                continue
            if "s_waitcnt vmcnt(0)" in line:
                break
            parts = line.split(None, 1)
            if len(parts) < 2 or parts[0].startswith(";"):
                continue
            for mm in re.finditer(r"v\[(\d+):(\d+)\]|\bv(\d+)\b", parts[1]):
                rs = range(int(mm.group(1)), int(mm.group(2)) + 1) if mm.group(1) else [int(mm.group(3))]
                if regs.intersection(rs):
                    reads.append(line.strip())
                    break
        assert regs, f"{k}: no tile loads found in the main loop"
        assert not reads, f"{k}: in-flight load registers read before the wait: {reads[:3]}"
