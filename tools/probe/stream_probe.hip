// Streaming-read ceiling of the k_step access pattern: 256 workgroups x 16 waves, one contiguous
// region per wave, 1 KiB buffer loads (16 B/lane) through a register ring of depth D, trivial
// compute.  Prints GB/s per ring depth and per workgroup count.  (tools/probe; not the product)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int D>
__global__ void __launch_bounds__(1024) k_stream(const int *ids, long n_chunks, long cpr, int R, int *out) {
    const int lane = threadIdx.x & 63;
    const int r = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 16 + (threadIdx.x >> 6)));
    if (r >= R) return;
    const long c0 = (long)r * cpr;
    const long c1 = c0 + cpr < n_chunks ? c0 + cpr : n_chunks;
    const int nc = (int)(c1 - c0);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(ids + c0 * 256), 0, nc * 1024, 0x00020000);
    int acc = 0;
    int4 q[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
        auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, i * 1024, 0);
        q[i] = make_int4(x[0], x[1], x[2], x[3]);
    }
    for (int c = 0; c < nc; c += D) {
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const int4 v = q[i];
            auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, (c + i + D) * 1024, 0);
            q[i] = make_int4(x[0], x[1], x[2], x[3]);
            acc += v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x12345678) out[0] = acc;
}

template <int D>
void run(const int *d, long n_chunks, int *dout) {
    const int G = 256, R = G * 16;
    const long cpr = (n_chunks + R - 1) / R;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int it = 0; it < 3; ++it) k_stream<D><<<G, 1024>>>(d, n_chunks, cpr, R, dout);
    hipEventRecord(a);
    const int N = 20;
    for (int it = 0; it < N; ++it) k_stream<D><<<G, 1024>>>(d, n_chunks, cpr, R, dout);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("depth %d: %.3f ms/pass  %.0f GB/s\n", D, ms / N, n_chunks * 1024.0 / (ms / N * 1e-3) / 1e9);
}

int main() {
    const long n_chunks = 1L << 22;   // 4 GiB
    int *d, *dout;
    hipMalloc(&d, n_chunks * 1024 + 1024 * 64);
    hipMalloc(&dout, 4);
    hipMemset(d, 1, n_chunks * 1024);
    run<2>(d, n_chunks, dout);
    run<4>(d, n_chunks, dout);
    run<6>(d, n_chunks, dout);
    run<8>(d, n_chunks, dout);
    run<12>(d, n_chunks, dout);
    return 0;
}
