// Semantics probe of the cross-lane moves used by the tile solve (DPP row_newbcast, v_permlane16/32_swap,
// DPP row_shr with bound_ctrl). Prints OK or the first mismatching lane.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(int* o) {
    const int l = threadIdx.x;
    const int x = 1000 + l;
    o[l] = __builtin_amdgcn_mov_dpp(x, 0x153, 0xf, 0xf, false);               // lane 3 of the row
    auto s16 = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    o[64 + l] = s16[0];
    o[128 + l] = s16[1];
    auto s32 = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    o[192 + l] = s32[0];
    o[256 + l] = s32[1];
    o[320 + l] = __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);      // row_shr:2, zero fill
}

int main() {
    int* d;
    hipMalloc(&d, 384 * sizeof(int));
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    int h[384];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        const int row = l >> 4, c = l & 15;
        const int exp[6] = {1000 + 16 * row + 3,
                            1000 + 16 * (row & ~1) + c,          // even row of each pair
                            1000 + 16 * (row | 1) + c,           // odd row of each pair
                            1000 + 16 * (row & 1) + c,           // low pair
                            1000 + 16 * (2 + (row & 1)) + c,     // high pair
                            c >= 2 ? 1000 + l - 2 : 0};
        for (int t = 0; t < 6; ++t)
            if (h[64 * t + l] != exp[t]) {
                if (bad++ < 12) printf("probe %d lane %d: got %d expected %d\n", t, l, h[64 * t + l], exp[t]);
            }
    }
    printf(bad ? "XLANE MISMATCH %d\n" : "XLANE OK\n", bad);
    return bad != 0;
}
