// Streaming-read ceiling of k_step_loop's access pattern by loads in flight per wave (D) and by
// VALU work per chunk: 256 workgroups x 16 waves (one workgroup per CU, as the product), one
// contiguous region per wave, 1 KiB non-temporal buffer loads (16 B/lane), a register ring of D
// chunks.  WORK = dependent VALU ops per chunk (about 3 VALU each; the product spends ~86 VALU + ~51 SALU per chunk).
// With LDS_KB the workgroup also reserves that much LDS (the product holds all 160 KiB).
// Prints one line per (D, WORK): ms per 4 GiB pass and GB/s.  (tools/probe; not the product)
#include <hip/hip_runtime.h>
#include <cstdio>

template <int D, int WORK>
__global__ void __launch_bounds__(1024) k_stream(const int *ids, long cpr, int R, int *out) {
    extern __shared__ int lds[];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int r = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 16 + w));
    if (r >= R) return;
    const long c0 = (long)r * cpr;
    const int nc = (int)cpr;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(ids + c0 * 256), 0,
                                                                       (int)((long)nc * 1024), 0x00020000);
    int acc = 0;
    int4 q[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
        auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, i * 1024, 2);
        q[i] = make_int4(x[0], x[1], x[2], x[3]);
    }
    for (int c = 0; c < nc; c += D) {
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const int4 v = q[i];
            auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, (c + i + D) * 1024, 2);
            q[i] = make_int4(x[0], x[1], x[2], x[3]);
            int t = v.x ^ v.y ^ v.z ^ v.w;
#pragma unroll
            for (int k = 0; k < WORK; ++k) t = (t * 0x9E37) ^ (t >> 3) ^ k;   // dependent VALU chain
            acc += t;
        }
    }
    if (acc == 0x12345678) { lds[threadIdx.x] = acc; out[0] = lds[(threadIdx.x + 1) & 1023]; }
}

template <int D, int WORK>
void run(const int *d, long n_chunks, int *dout, int lds_kb) {
    const int G = 256, R = G * 16;
    const long cpr = n_chunks / R;
    const size_t sh = (size_t)lds_kb * 1024;
    hipFuncSetAttribute((const void *)k_stream<D, WORK>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int it = 0; it < 3; ++it) k_stream<D, WORK><<<G, 1024, sh>>>(d, cpr, R, dout);
    hipEventRecord(a);
    const int N = 20;
    for (int it = 0; it < N; ++it) k_stream<D, WORK><<<G, 1024, sh>>>(d, cpr, R, dout);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("{\"D\": %d, \"work\": %d, \"lds_kb\": %d, \"ms_per_pass\": %.4f, \"GBps\": %.0f}\n", D, WORK, lds_kb,
           ms / N, R * cpr * 1024.0 / (ms / N * 1e-3) / 1e9);
    fflush(stdout);
}

template <int WORK>
void sweep(const int *d, long n, int *o, int lds) {
    run<1, WORK>(d, n, o, lds);
    run<2, WORK>(d, n, o, lds);
    run<3, WORK>(d, n, o, lds);
    run<4, WORK>(d, n, o, lds);
    run<5, WORK>(d, n, o, lds);
    run<6, WORK>(d, n, o, lds);
    run<8, WORK>(d, n, o, lds);
}

int main() {
    const long n_chunks = 1L << 22;   // 4 GiB: C3's 2^30 slots
    int *d, *dout;
    hipMalloc(&d, n_chunks * 1024 + 1024 * 64 * 16);
    hipMalloc(&dout, 4);
    hipMemset(d, 1, n_chunks * 1024 + 1024 * 64 * 16);
    sweep<0>(d, n_chunks, dout, 160);
    sweep<16>(d, n_chunks, dout, 160);
    sweep<32>(d, n_chunks, dout, 160);
    sweep<48>(d, n_chunks, dout, 160);
    return 0;
}
