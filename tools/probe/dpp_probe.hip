// Probe: which DPP wavefront-shift control moves lane i+1 -> lane i (shfl_down 1) on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int *out) {
    int l = threadIdx.x;
    out[l] = __builtin_amdgcn_update_dpp(-1, l * 10, 0x130, 0xF, 0xF, false);
    out[64 + l] = __builtin_amdgcn_update_dpp(-1, l * 10, 0x138, 0xF, 0xF, false);
    out[128 + l] = __builtin_amdgcn_update_dpp(-1, l * 10, 0x134, 0xF, 0xF, false);
    out[192 + l] = __builtin_amdgcn_update_dpp(-1, l * 10, 0x13C, 0xF, 0xF, false);
}
int main() {
    int *d, h[256];
    hipMalloc(&d, sizeof(h));
    k<<<1, 64>>>(d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char *nm[4] = {"0x130 wave_shl1", "0x138 wave_shr1", "0x134 wave_rol1", "0x13C wave_ror1"};
    for (int j = 0; j < 4; ++j) {
        printf("%s:", nm[j]);
        for (int l : {0, 1, 2, 15, 16, 31, 32, 62, 63}) printf(" [%d]=%d", l, h[64 * j + l]);
        printf("\n");
    }
    return 0;
}
