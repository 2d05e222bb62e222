"""Which library kernel torch (hipBLASLt / rocBLAS) runs for the DSSM fp32 tower GEMMs (diagnostics: run under
rocprofv3 --kernel-trace --stats; the kernel name encodes its macro tile / matrix instruction / split)."""
import torch

for M, K, N in ((4096, 8704, 1024), (4096, 20480, 1024)):
    x = torch.randn((M, K), device="cuda")
    w = torch.randn((N, K), device="cuda")
    for _ in range(5):
        torch.nn.functional.linear(x, w)
torch.cuda.synchronize()
print("ok")
