/*
 * bpe_cpu_mt.cc — multi-threaded CPU restatement of the reference's BPE merge-training hot path.
 *
 * TEST INFRASTRUCTURE + CPU BASELINE ONLY.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load liboracle_mt.so; the product path
 * (libbpe.so, the N-API addon, core.js) never does.
 *
 * Reference: beenotung/bpe-tokenizer v2.2.0, /root/reference/core.ts — findNextMerge (247-326),
 * applyMerge (332-360), mergeUntil (365-383).  This is the order-free restatement of SURVEY.md
 * Appendix A (R1-R5), run on all host cores: the same full recount per merge as the reference
 * (and as the GPU engine), so its pair-scans/s is comparable with theirs.  It is pinned against
 * oracle/bpe_oracle.c (the literal scan-order restatement, itself pinned to the reference's own
 * outputs in tests/golden/) by tests/test_oracle_golden.py: every golden case and random corpora.
 *
 * Parallel layout: the samples (core.ts:106, one `corpus_in_code` string each) are cut into
 * contiguous ranges, one per thread; pairs never cross samples (core.ts:265-267), so each range
 * is counted and rewritten on its own.  Per iteration:
 *   count   — R1 (core.ts:265-293): a pair (x, y) at position i counts unless x == y sits at an
 *             odd offset of its run (the skip rule 285-290).  Pairs of ids < 256 go to a dense
 *             per-thread table; the others are appended to per-thread, per-partition key lists;
 *   reduce  — partition p (one thread) sums the lists sent to it in an open-addressing table and
 *             a 1/P slice of the dense tables, and keeps its best packed key
 *             (W << 17 | (0x1FFFF - (a + b)), after the max_length filter core.ts:270-273);
 *   select  — R2/R3 (core.ts:294-313): max W, then min a + b, then (only when pairs remain tied)
 *             the earliest last counted occurrence, found by a tie scan over the ranges;
 *   apply   — R5 (core.ts:356-359): leftmost non-overlapping rewrite of every sample in place.
 * Samples keep their start offset; a rewritten sample leaves dead space behind it, so the
 * corpus order of positions (begin + i) is unchanged and no global compaction is needed.
 */
#include <omp.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

constexpr int HOT = 256;
constexpr uint32_t EMPTY = 0xFFFFFFFFu;

inline uint64_t pack_key(uint64_t w, int32_t a, int32_t b) {
    return w ? ((w << 17) | (uint64_t)(0x1FFFF - (a + b))) : 0;
}

struct PartTable {   // open addressing, u32 key (a << 16 | b) -> u64 count
    std::vector<uint32_t> keys;
    std::vector<uint64_t> counts;
    uint32_t mask = 0;
    void reset(size_t want) {
        size_t cap = 1024;
        while (cap < 2 * want) cap <<= 1;
        if (keys.size() != cap) {
            keys.assign(cap, EMPTY);
            counts.assign(cap, 0);
        } else {
            std::fill(keys.begin(), keys.end(), EMPTY);
            std::fill(counts.begin(), counts.end(), 0);
        }
        mask = (uint32_t)(cap - 1);
    }
    void add(uint32_t key) {
        uint32_t h = (key * 0x9E3779B1u) & mask;
        for (;;) {
            if (keys[h] == key) break;
            if (keys[h] == EMPTY) {
                keys[h] = key;
                break;
            }
            h = (h + 1) & mask;
        }
        counts[h] += 1;
    }
};

struct Range {
    int64_t s0, s1;   // samples [s0, s1)
};

}  // namespace

struct cpu_bpe {
    std::vector<int32_t> ids;
    std::vector<int64_t> begin, len;   // per sample
    std::vector<int32_t> len16;
    int32_t n_tokens = 0;
    int T = 1;                         // threads == partitions
    std::vector<Range> ranges;
    std::vector<std::vector<uint32_t>> hot;            // [T][65536]
    std::vector<std::vector<std::vector<uint32_t>>> buf;   // [T][P] cold keys
    std::vector<PartTable> part;
    std::vector<uint64_t> hot_sum;                     // [65536]
    std::vector<uint64_t> part_best;
    int64_t live = 0;
};

namespace {

inline uint32_t part_of(uint32_t key, int P) {
    return (uint32_t)(((uint64_t)(key * 0x85EBCA6Bu) * (uint64_t)P) >> 32);
}

bool pair_ok(const cpu_bpe *c, int32_t a, int32_t b, int64_t max_length) {
    return !max_length || (int64_t)c->len16[a] + c->len16[b] <= max_length;
}

// R1 over one thread's samples: dense hot counts + per-partition cold key lists.
void count_range(cpu_bpe *c, int t) {
    uint32_t *hot = c->hot[t].data();
    std::memset(hot, 0, HOT * HOT * sizeof(uint32_t));
    auto &bufs = c->buf[t];
    for (auto &b : bufs) b.clear();
    const int P = c->T;
    const Range r = c->ranges[t];
    for (int64_t s = r.s0; s < r.s1; ++s) {
        const int32_t *p = c->ids.data() + c->begin[s];
        const int64_t n = c->len[s];
        if (n < 2) continue;
        int32_t prev = p[0];
        int par = 0;   // parity of prev's offset in its run of equal tokens
        for (int64_t i = 1; i < n; ++i) {
            const int32_t t2 = p[i];
            bool counted;
            if (t2 == prev) {
                counted = par == 0;   // core.ts:285-290: X X counts at even run offsets only
                par ^= 1;
            } else {
                counted = true;
                par = 0;
            }
            if (counted) {
                if ((prev | t2) < HOT) {
                    hot[(prev << 8) | t2] += 1;
                } else {
                    const uint32_t key = ((uint32_t)prev << 16) | (uint32_t)t2;
                    bufs[part_of(key, P)].push_back(key);
                }
            }
            prev = t2;
        }
    }
}

// Last counted position (begin + i, + 1; 0 = none) of each candidate in one thread's samples.
void tie_range(const cpu_bpe *c, int t, const std::vector<uint32_t> &cand, uint64_t *last) {
    const Range r = c->ranges[t];
    for (int64_t s = r.s0; s < r.s1; ++s) {
        const int32_t *p = c->ids.data() + c->begin[s];
        const int64_t n = c->len[s];
        if (n < 2) continue;
        int32_t prev = p[0];
        int par = 0;
        for (int64_t i = 1; i < n; ++i) {
            const int32_t t2 = p[i];
            bool counted;
            if (t2 == prev) {
                counted = par == 0;
                par ^= 1;
            } else {
                counted = true;
                par = 0;
            }
            if (counted) {
                const uint32_t key = ((uint32_t)prev << 16) | (uint32_t)t2;
                for (size_t j = 0; j < cand.size(); ++j)
                    if (cand[j] == key) last[j] = (uint64_t)(c->begin[s] + i - 1) + 1;
            }
            prev = t2;
        }
    }
}

// R5: leftmost non-overlapping (a, b) -> cc in every sample of one thread's range.
int64_t apply_range(cpu_bpe *c, int t, int32_t a, int32_t b, int32_t cc) {
    const Range r = c->ranges[t];
    int64_t w = 0;
    for (int64_t s = r.s0; s < r.s1; ++s) {
        int32_t *p = c->ids.data() + c->begin[s];
        const int64_t n = c->len[s];
        int64_t i = 0;
        while (i + 1 < n && !(p[i] == a && p[i + 1] == b)) ++i;   // first match (no writes)
        if (i + 1 >= n) continue;
        int64_t o = i;
        while (i < n) {
            if (i + 1 < n && p[i] == a && p[i + 1] == b) {
                p[o++] = cc;
                i += 2;
                ++w;
            } else {
                p[o++] = p[i++];
            }
        }
        c->len[s] = o;
    }
    return w;
}

}  // namespace

extern "C" {

/* A corpus (flat ids + n_samples + 1 offsets), the UTF-16 length of each of n_tokens tokens, room
 * for `extra` more tokens, `threads` OpenMP threads (<= 0: all). */
cpu_bpe *cpu_setup(cpu_bpe *c, const int64_t *off, int64_t n_samples, const int32_t *len16,
                   int32_t n_tokens, int64_t extra, int threads);

cpu_bpe *cpu_create(const int32_t *ids, const int64_t *off, int64_t n_samples, const int32_t *len16,
                    int32_t n_tokens, int64_t extra, int threads) {
    cpu_bpe *c = new cpu_bpe();
    c->ids.assign(ids, ids + off[n_samples]);
    return cpu_setup(c, off, n_samples, len16, n_tokens, extra, threads);
}

/* The same from latin1 bytes (byte b -> token map256[b]) cut into samples of sample_bytes (the
 * last one shorter), without a host copy of the int32 ids: the config-5 corpus (16 GiB of text)
 * is 64 GiB of ids.  Every token has UTF-16 length 1. */
cpu_bpe *cpu_create_latin1(const uint8_t *bytes, int64_t n, int64_t sample_bytes,
                           const int32_t *map256, int32_t n_tokens, int64_t extra, int threads) {
    cpu_bpe *c = new cpu_bpe();
    c->ids.resize(n);
    int32_t *ids = c->ids.data();
#pragma omp parallel for schedule(static) num_threads(threads > 0 ? threads : omp_get_max_threads())
    for (int64_t i = 0; i < n; ++i) ids[i] = map256[bytes[i]];
    if (sample_bytes <= 0 || sample_bytes > n) sample_bytes = n > 0 ? n : 1;
    const int64_t n_samples = (n + sample_bytes - 1) / sample_bytes;
    std::vector<int64_t> off(n_samples + 1);
    for (int64_t k = 0; k <= n_samples; ++k) off[k] = std::min(n, k * sample_bytes);
    std::vector<int32_t> len16(std::max<int32_t>(n_tokens, 1), 1);
    return cpu_setup(c, off.data(), n_samples, len16.data(), n_tokens, extra, threads);
}

cpu_bpe *cpu_setup(cpu_bpe *c, const int64_t *off, int64_t n_samples, const int32_t *len16,
                   int32_t n_tokens, int64_t extra, int threads) {
    const int64_t total = off[n_samples];
    c->begin.resize(n_samples);
    c->len.resize(n_samples);
    for (int64_t s = 0; s < n_samples; ++s) {
        c->begin[s] = off[s];
        c->len[s] = off[s + 1] - off[s];
    }
    c->len16.assign(len16, len16 + n_tokens);
    c->len16.resize((size_t)n_tokens + (size_t)std::max<int64_t>(extra, 0), 1);
    c->n_tokens = n_tokens;
    c->live = total;
    int T = threads > 0 ? threads : omp_get_max_threads();
    T = (int)std::max<int64_t>(1, std::min<int64_t>(T, std::max<int64_t>(1, n_samples)));
    c->T = T;
    // contiguous sample ranges of about total / T tokens each
    int64_t s = 0;
    for (int t = 0; t < T; ++t) {
        const int64_t target = total * (t + 1) / T;
        int64_t e = s;
        while (e < n_samples && (off[e] < target || e == s)) ++e;
        if (t == T - 1) e = n_samples;
        c->ranges.push_back({s, e});
        s = e;
    }
    c->hot.assign(T, std::vector<uint32_t>(HOT * HOT));
    c->buf.assign(T, std::vector<std::vector<uint32_t>>(T));
    c->part.resize(T);
    c->hot_sum.assign(HOT * HOT, 0);
    c->part_best.assign(T, 0);
    return c;
}

void cpu_destroy(cpu_bpe *c) { delete c; }

int64_t cpu_live(const cpu_bpe *c) { return c->live; }

int cpu_threads(const cpu_bpe *c) { return c->T; }

/* findNextMerge (core.ts:247-326): 0 and (a, b, W), or 1 when the reference returns null. */
int cpu_find_next_merge(cpu_bpe *c, int64_t max_length, int64_t min_weight, int32_t *out_a,
                        int32_t *out_b, int64_t *out_w) {
    if (min_weight == 0) min_weight = 2;                               // core.ts:256
    const int T = c->T;
#pragma omp parallel num_threads(T)
    {
        const int t = omp_get_thread_num();
        count_range(c, t);
#pragma omp barrier
        // partition t: its cold keys from every thread, and its slice of the hot bins
        size_t n = 0;
        for (int u = 0; u < T; ++u) n += c->buf[u][t].size();
        PartTable &pt = c->part[t];
        pt.reset(n);
        for (int u = 0; u < T; ++u)
            for (uint32_t k : c->buf[u][t]) pt.add(k);
        uint64_t best = 0;
        for (size_t h = 0; h <= pt.mask; ++h) {
            if (pt.keys[h] == EMPTY) continue;
            const int32_t a = (int32_t)(pt.keys[h] >> 16), b = (int32_t)(pt.keys[h] & 0xFFFF);
            if (!pair_ok(c, a, b, max_length)) continue;
            best = std::max(best, pack_key(pt.counts[h], a, b));
        }
        const int lo = HOT * HOT * t / T, hi = HOT * HOT * (t + 1) / T;
        for (int bin = lo; bin < hi; ++bin) {
            uint64_t sum = 0;
            for (int u = 0; u < T; ++u) sum += c->hot[u][bin];
            c->hot_sum[bin] = sum;
            const int32_t a = bin >> 8, b = bin & 255;
            if (sum && pair_ok(c, a, b, max_length)) best = std::max(best, pack_key(sum, a, b));
        }
        c->part_best[t] = best;
    }
    uint64_t best = 0;
    for (uint64_t b : c->part_best) best = std::max(best, b);
    if (!best) return 1;                                               // core.ts:312
    const int64_t W = (int64_t)(best >> 17);
    if (W < min_weight) return 1;                                      // core.ts:313
    // every pair sharing the best (W, a + b)
    std::vector<uint32_t> cand;
    for (int bin = 0; bin < HOT * HOT; ++bin) {
        const int32_t a = bin >> 8, b = bin & 255;
        if (c->hot_sum[bin] && pair_ok(c, a, b, max_length) && pack_key(c->hot_sum[bin], a, b) == best)
            cand.push_back(((uint32_t)a << 16) | (uint32_t)b);
    }
    for (int t = 0; t < T; ++t) {
        const PartTable &pt = c->part[t];
        if (c->part_best[t] != best) continue;
        for (size_t h = 0; h <= pt.mask; ++h) {
            if (pt.keys[h] == EMPTY) continue;
            const int32_t a = (int32_t)(pt.keys[h] >> 16), b = (int32_t)(pt.keys[h] & 0xFFFF);
            if (pair_ok(c, a, b, max_length) && pack_key(pt.counts[h], a, b) == best)
                cand.push_back(pt.keys[h]);
        }
    }
    uint32_t win = cand[0];
    if (cand.size() > 1) {
        // R3: the candidate whose last counted occurrence is earliest (core.ts:296-305)
        std::vector<uint64_t> last(T * cand.size(), 0);
#pragma omp parallel num_threads(T)
        {
            const int t = omp_get_thread_num();
            tie_range(c, t, cand, last.data() + t * cand.size());
        }
        uint64_t bp = ~0ull;
        for (size_t j = 0; j < cand.size(); ++j) {
            uint64_t l = 0;
            for (int t = 0; t < T; ++t) l = std::max(l, last[t * cand.size() + j]);
            if (l && l < bp) {
                bp = l;
                win = cand[j];
            }
        }
    }
    *out_a = (int32_t)(win >> 16);
    *out_b = (int32_t)(win & 0xFFFF);
    *out_w = W;
    return 0;
}

/* applyMerge's rewrite (core.ts:356-359) with c = cc; registers len16[cc] (core.ts:318).
 * Returns the replacement count. */
int64_t cpu_apply_merge(cpu_bpe *c, int32_t a, int32_t b, int32_t cc) {
    if ((size_t)cc >= c->len16.size()) c->len16.resize((size_t)cc + 1024, 1);
    c->len16[cc] = c->len16[a] + c->len16[b];
    c->n_tokens = std::max(c->n_tokens, cc + 1);
    int64_t w = 0;
    const int T = c->T;
#pragma omp parallel num_threads(T) reduction(+ : w)
    w += apply_range(c, omp_get_thread_num(), a, b, cc);
    c->live -= w;
    return w;
}

/* mergeUntil (core.ts:365-383): up to max_iterations (0 = unlimited) merges, (a, b, W) triples into
 * out_abw (capacity cap); *scans receives the pair-scans (live tokens summed over iterations).
 * Returns the merge count. */
int64_t cpu_merge_until(cpu_bpe *c, int64_t max_length, int64_t min_weight, int64_t max_iterations,
                        int64_t *out_abw, int64_t cap, int64_t *scans) {
    int64_t n = 0, sc = 0;
    for (int64_t it = 1; !max_iterations || it <= max_iterations; ++it) {
        int32_t a, b;
        int64_t w;
        const int64_t live = c->live;
        if (cpu_find_next_merge(c, max_length, min_weight, &a, &b, &w)) break;
        sc += live;
        cpu_apply_merge(c, a, b, c->n_tokens);
        if (n < cap) {
            out_abw[3 * n] = a;
            out_abw[3 * n + 1] = b;
            out_abw[3 * n + 2] = w;
        }
        ++n;
    }
    if (scans) *scans = sc;
    return n;
}

/* The corpus: ids_out (capacity live) and n_samples + 1 offsets. */
void cpu_read(const cpu_bpe *c, int32_t *ids_out, int64_t *off_out) {
    int64_t o = 0;
    off_out[0] = 0;
    for (size_t s = 0; s < c->begin.size(); ++s) {
        if (c->len[s])
            std::memcpy(ids_out + o, c->ids.data() + c->begin[s], c->len[s] * sizeof(int32_t));
        o += c->len[s];
        off_out[s + 1] = o;
    }
}

}  // extern "C"
