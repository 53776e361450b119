// Probe: does a 160 KiB dynamic-LDS workgroup see 40960 distinct words?  Each thread writes a
// word id pattern, then after a barrier every word is read back and compared.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void __launch_bounds__(1024) probe(uint32_t *bad, int words) {
    extern __shared__ uint32_t lds[];
    for (int i = threadIdx.x; i < words; i += 1024) lds[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < words; i += 1024) atomicAdd(&lds[i], (uint32_t)i + 1);
    __syncthreads();
    for (int i = threadIdx.x; i < words; i += 1024)
        if (lds[i] != (uint32_t)i + 1) atomicAdd(&bad[0], 1u), atomicMin(&bad[1], (uint32_t)i);
}

int main() {
    uint32_t *bad;
    hipMalloc(&bad, 8);
    for (int kib : {128, 144, 152, 160}) {
        int words = kib * 256;
        uint32_t h[2] = {0, 0xFFFFFFFFu};
        hipMemcpy(bad, h, 8, hipMemcpyHostToDevice);
        hipError_t e = hipFuncSetAttribute((const void *)probe, hipFuncAttributeMaxDynamicSharedMemorySize, words * 4);
        probe<<<256, 1024, words * 4>>>(bad, words);
        hipError_t e2 = hipDeviceSynchronize();
        hipMemcpy(h, bad, 8, hipMemcpyDeviceToHost);
        printf("%d KiB: attr=%d launch=%d bad=%u first_bad_word=%d\n", kib, (int)e, (int)e2, h[0], (int)h[1]);
    }
    return 0;
}
