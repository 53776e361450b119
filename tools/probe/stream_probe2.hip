// Streaming-read ceiling of the k_step access pattern by cache policy and by region layout.
// 256 workgroups x 16 waves, 1 KiB buffer loads (16 B/lane), a register ring of depth 8, trivial
// compute.  Variants: the load's cache-policy bits (aux: 0 plain, 1 sc0, 2 nt, 16 sc1, 3 sc0|nt,
// 18 nt|sc1) with one contiguous region per wave (k_step's layout), and a layout where a
// workgroup's 16 waves read consecutive chunks of one contiguous workgroup region.
// (tools/probe; not the product)
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int D = 8;

template <int AUX, bool WG_INTERLEAVE>
__global__ void __launch_bounds__(1024) k_stream(const int *ids, long n_chunks, long cpr, int R, int *out) {
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int r = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 16 + w));
    if (r >= R) return;
    long c0, stride;
    int nc;
    if (WG_INTERLEAVE) {
        // the workgroup owns 16 * cpr consecutive chunks; wave w reads w, w+16, w+32, ...
        c0 = (long)blockIdx.x * 16 * cpr + w;
        stride = 16;
        nc = (int)cpr;
    } else {
        c0 = (long)r * cpr;
        stride = 1;
        nc = (int)cpr;
    }
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(ids + c0 * 256), 0,
                                                                       (int)(((long)nc * stride) * 1024), 0x00020000);
    int acc = 0;
    int4 q[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
        auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, (int)(i * stride * 1024), AUX);
        q[i] = make_int4(x[0], x[1], x[2], x[3]);
    }
    for (int c = 0; c < nc; c += D) {
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const int4 v = q[i];
            auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, (int)((c + i + D) * stride * 1024), AUX);
            q[i] = make_int4(x[0], x[1], x[2], x[3]);
            acc += v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x12345678) out[0] = acc;
}

template <int AUX, bool IL>
void run(const int *d, long n_chunks, int *dout, const char *name) {
    const int G = 256, R = G * 16;
    const long cpr = n_chunks / R;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int it = 0; it < 3; ++it) k_stream<AUX, IL><<<G, 1024>>>(d, n_chunks, cpr, R, dout);
    hipEventRecord(a);
    const int N = 20;
    for (int it = 0; it < N; ++it) k_stream<AUX, IL><<<G, 1024>>>(d, n_chunks, cpr, R, dout);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-28s %.3f ms/pass  %.0f GB/s\n", name, ms / N, R * cpr * 1024.0 / (ms / N * 1e-3) / 1e9);
}

int main() {
    const long n_chunks = 1L << 22;   // 4 GiB
    int *d, *dout;
    hipMalloc(&d, n_chunks * 1024 + 1024 * 64 * 16);
    hipMalloc(&dout, 4);
    hipMemset(d, 1, n_chunks * 1024 + 1024 * 64 * 16);
    for (int rep = 0; rep < 2; ++rep) {
        run<0, false>(d, n_chunks, dout, "region/wave plain");
        run<1, false>(d, n_chunks, dout, "region/wave sc0");
        run<2, false>(d, n_chunks, dout, "region/wave nt");
        run<16, false>(d, n_chunks, dout, "region/wave sc1");
        run<3, false>(d, n_chunks, dout, "region/wave sc0|nt");
        run<18, false>(d, n_chunks, dout, "region/wave nt|sc1");
        run<0, true>(d, n_chunks, dout, "region/wg plain");
        run<2, true>(d, n_chunks, dout, "region/wg nt");
    }
    return 0;
}
