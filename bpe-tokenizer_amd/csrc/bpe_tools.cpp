// bpe_tools.cpp — synthetic corpus generator for the bench and tests (include/bpe_tools.h).
#include "bpe_tools.h"

#include <cstring>
#include <thread>
#include <vector>

namespace {

inline uint32_t step(uint32_t x) {
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    return x;
}

// 32x32 matrices over GF(2), stored as columns: M(x) = XOR of col[j] for set bits j of x.
struct Mat {
    uint32_t col[32];
};

inline uint32_t apply(const Mat &m, uint32_t x) {
    uint32_t r = 0;
    for (int j = 0; j < 32; ++j)
        if (x >> j & 1u) r ^= m.col[j];
    return r;
}

inline Mat mul(const Mat &a, const Mat &b) {  // a o b
    Mat r;
    for (int j = 0; j < 32; ++j) r.col[j] = apply(a, b.col[j]);
    return r;
}

uint32_t jump(uint32_t x, uint64_t n) {
    Mat m, acc;
    for (int j = 0; j < 32; ++j) {
        m.col[j] = step(1u << j);
        acc.col[j] = 1u << j;
    }
    while (n) {
        if (n & 1) acc = mul(m, acc);
        m = mul(m, m);
        n >>= 1;
    }
    return apply(acc, x);
}

}  // namespace

extern "C" int bpe_synth_latin1(uint32_t seed, uint32_t A, uint32_t base, uint64_t skip,
                                uint8_t *out, int64_t n) {
    if (!out || n < 0 || A == 0 || A > 256 || base + A > 256) return -1;
    unsigned nt = std::thread::hardware_concurrency();
    if (nt == 0) nt = 1;
    if (nt > 16) nt = 16;
    if (n < (1 << 22)) nt = 1;
    const int64_t per = (n + nt - 1) / nt;
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t) {
        const int64_t b = t * per, e = std::min<int64_t>(n, b + per);
        if (b >= e) break;
        th.emplace_back([=]() {
            uint32_t x = jump(seed, skip + (uint64_t)b);
            for (int64_t i = b; i < e; ++i) {
                x = step(x);
                out[i] = (uint8_t)(base + (uint32_t)(((uint64_t)x * A) >> 32));
            }
        });
    }
    for (auto &t : th) t.join();
    return 0;
}
