// probe: semantics of gfx950 v_permlane16_swap / v_permlane32_swap and DPP row ops (prints per lane)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out) {
    int l = threadIdx.x;
    int a = 100 + l, b = 200 + l;
    auto p32 = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    auto p16 = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    out[l * 8 + 0] = p32[0];
    out[l * 8 + 1] = p32[1];
    out[l * 8 + 2] = p16[0];
    out[l * 8 + 3] = p16[1];
    out[l * 8 + 4] = __builtin_amdgcn_update_dpp(0, l, 0x141, 0xf, 0xf, false);  // row_half_mirror
    out[l * 8 + 5] = __builtin_amdgcn_update_dpp(0, l, 0x140, 0xf, 0xf, false);  // row_mirror
    out[l * 8 + 6] = __builtin_amdgcn_update_dpp(0, l, 0xB1, 0xf, 0xf, false);   // quad_perm 1,0,3,2
    out[l * 8 + 7] = __builtin_amdgcn_update_dpp(0, l, 0x4E, 0xf, 0xf, false);   // quad_perm 2,3,0,1
}
int main() {
    int* d; hipMalloc(&d, 64 * 8 * 4); hipLaunchKernelGGL(k, 1, 64, 0, 0, d);
    int h[512]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; ++l) { printf("%2d:", l); for (int j = 0; j < 8; ++j) printf(" %3d", h[l*8+j]); printf("\n"); }
    return 0;
}
