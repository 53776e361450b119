// LDS atomic throughput probe: 256 workgroups x 1024 threads, each lane adds 1 << (16 * half) to
// pseudo-random dwords of a 160 KiB LDS table, with and without the returned value, and with the
// address spread restricted (conflict-free pattern) for comparison.  (tools/probe; not the product)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int RTN, int PATTERN>
__global__ void __launch_bounds__(1024) k(uint32_t *out, int iters, uint32_t seed) {
    __shared__ uint32_t t[40960];
    for (int i = threadIdx.x; i < 40960; i += 1024) t[i] = 0;
    __syncthreads();
    uint32_t x = seed ^ (blockIdx.x * 1024 + threadIdx.x) * 0x9E3779B1u;
    uint32_t a[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        a[e] = PATTERN == 0 ? (x & 0x7FFFu) * 4 : ((threadIdx.x & 63) + 64 * ((x >> 8) & 511u)) * 4;
    }
    uint32_t acc = 0;
    for (int i = 0; i < iters; ++i) {
        const uint32_t off = PATTERN == 0 ? (uint32_t)i * 4 * 641 : (uint32_t)i * 4 * 64 * 7;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            // (address and half from registers: one add and one compare-free wrap per atomic)
            const uint32_t b = (a[(e + (i & 1) * 4)] + off) & 0x1FFFCu;   // 128 KiB of the table
            const uint32_t inc = 1u << ((b << 2) & 16u);
            uint32_t *p = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(t) + (b & ~3u));
            if (RTN) acc |= atomicAdd(p, inc);
            else __hip_atomic_fetch_add(p, inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    __syncthreads();
    if (RTN) out[blockIdx.x * 1024 + threadIdx.x] = acc;
    else out[blockIdx.x * 1024 + threadIdx.x] = t[threadIdx.x];
}

template <int RTN, int P>
float run(uint32_t *d, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    k<RTN, P><<<256, 1024>>>(d, iters, 1);
    hipEventRecord(a);
    k<RTN, P><<<256, 1024>>>(d, iters, 2);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    uint32_t *d;
    hipMalloc(&d, 256 * 1024 * 4);
    const int iters = 1024;
    const double ops = 256.0 * 16 * 4 * iters;   // wave-instructions
    float m;
    m = run<1, 0>(d, iters); printf("rtn random     %.3f ms  %.1f cyc/instr/CU\n", m, m * 1e-3 * 2.4e9 / (ops / 256));
    m = run<0, 0>(d, iters); printf("noret random   %.3f ms  %.1f cyc/instr/CU\n", m, m * 1e-3 * 2.4e9 / (ops / 256));
    m = run<1, 1>(d, iters); printf("rtn spread     %.3f ms  %.1f cyc/instr/CU\n", m, m * 1e-3 * 2.4e9 / (ops / 256));
    m = run<0, 1>(d, iters); printf("noret spread   %.3f ms  %.1f cyc/instr/CU\n", m, m * 1e-3 * 2.4e9 / (ops / 256));
    return 0;
}
