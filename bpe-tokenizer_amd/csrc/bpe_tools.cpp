// bpe_tools.cpp — synthetic corpus generator for the bench and tests (include/bpe_tools.h).
#include "bpe_tools.h"

#include <algorithm>
#include <cmath>
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

// ---- skewed variant: Zipf-distributed words ("Zipf s=1.1 words") -------------
namespace {

inline uint32_t mix32(uint32_t x) {   // (murmur3 finaliser; seeds the per-word / per-sample streams)
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    x ^= x >> 16;
    return x ? x : 1u;
}

inline uint32_t below(uint32_t x, uint32_t n) { return (uint32_t)(((uint64_t)x * n) >> 32); }

}  // namespace

extern "C" int bpe_synth_zipf(uint32_t seed, double s, uint32_t n_words, uint64_t first_sample,
                              int64_t sample_bytes, uint8_t *out, int64_t n) {
    if (!out || n < 0 || sample_bytes <= 0 || n_words == 0 || n_words > (1u << 24) || !(s > 0))
        return -1;
    // the word list: word w is 2..8 letters a-z from its own stream
    std::vector<uint32_t> woff(n_words + 1, 0);
    std::vector<uint8_t> wchars;
    wchars.reserve((size_t)n_words * 5);
    for (uint32_t w = 0; w < n_words; ++w) {
        uint32_t x = mix32(seed ^ mix32(0x9E3779B9u * (w + 1)));
        x = step(x);
        const uint32_t len = 2 + below(x, 7);
        for (uint32_t i = 0; i < len; ++i) {
            x = step(x);
            wchars.push_back((uint8_t)('a' + below(x, 26)));
        }
        woff[w + 1] = (uint32_t)wchars.size();
    }
    // rank r (1-based) has weight r^-s
    std::vector<double> cdf(n_words);
    double acc = 0;
    for (uint32_t r = 0; r < n_words; ++r) cdf[r] = (acc += std::pow((double)(r + 1), -s));
    for (auto &v : cdf) v /= acc;
    const int64_t n_samples = (n + sample_bytes - 1) / sample_bytes;
    unsigned nt = std::thread::hardware_concurrency();
    if (nt == 0) nt = 1;
    if (nt > 16) nt = 16;
    if (n_samples < (int64_t)nt) nt = (unsigned)std::max<int64_t>(1, n_samples);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t]() {
            for (int64_t k = t; k < n_samples; k += nt) {
                // sample first_sample + k: words from its own stream, one separator after each
                // (a newline after 1 word in 16, else a space), cut at sample_bytes
                uint32_t x = mix32((uint32_t)seed + 0x9E3779B9u * (uint32_t)(first_sample + k + 1) +
                                   (uint32_t)((first_sample + k) >> 32));
                uint8_t *p = out + k * sample_bytes;
                const int64_t len = std::min<int64_t>(sample_bytes, n - k * sample_bytes);
                int64_t i = 0;
                while (i < len) {
                    x = step(x);
                    const double u = (double)x * (1.0 / 4294967296.0);
                    const uint32_t w = (uint32_t)(std::lower_bound(cdf.begin(), cdf.end(), u) -
                                                  cdf.begin());
                    const uint32_t wi = w < n_words ? w : n_words - 1;
                    for (uint32_t j = woff[wi]; j < woff[wi + 1] && i < len; ++j) p[i++] = wchars[j];
                    x = step(x);
                    if (i < len) p[i++] = (x & 15u) == 0 ? '\n' : ' ';
                }
            }
        });
    for (auto &t : th) t.join();
    return 0;
}
