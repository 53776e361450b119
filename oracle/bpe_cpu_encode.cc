/*
 * bpe_cpu_encode.cc — the device encoder's algorithm (bpe-tokenizer_amd/csrc/bpe_encode.hip, DESIGN
 * §3d) on the host's cores: a CPU baseline for encodeToCode of a batch of texts.
 *
 * TEST INFRASTRUCTURE + CPU BASELINE ONLY.  Only tests/ and bench.py's / tools/encode_bench.py's
 * CPU legs load liboracle_enc.so; the product path never does.
 *
 * Reference: /root/reference/core.ts encodeToCode (392-409) replays every merge's replaceAll over
 * the text in list order (404-406).  For a list in which no merge's new token is an input of
 * itself or of an earlier merge (every list the reference trains: c is always a fresh index,
 * core.ts:315,484), that equals the rank-greedy form: take the lowest-ranked merge whose pair
 * occurs, rewrite all its leftmost non-overlapping occurrences, repeat (proof in DESIGN §3d).  This
 * file runs the rank-greedy form the classic way, per text on one thread: a doubly linked list of
 * the tokens and a binary heap of the adjacencies keyed (rank, position).  A rewrite only creates
 * pairs with the new token c, whose merges all rank above the current one, so popping in (rank,
 * position) order takes each rank's occurrences left to right: for x x pairs that is replaceAll's
 * leftmost non-overlapping rule (the pair at p + 1 is gone once p is merged; p + 2 is popped next).
 * O(n log n) per text; texts are spread over threads with OpenMP (dynamic schedule).
 *
 * Checked against the in-order replay oracle_encode (oracle/bpe_oracle.c) by
 * tests/test_encoder.py::test_cpu_rank_greedy_equals_replay.
 */
#include <omp.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

constexpr uint32_t NO_RANK = 0xFFFFFFFFu;

struct RankTable {   // open addressing: key (a << 16 | b) -> rank, c
    std::vector<uint64_t> slots;   // key << 32 | rank, ~0 free
    std::vector<int32_t> c_of;
    uint32_t mask = 0;
    void build(const int32_t *abc, int64_t m) {
        size_t cap = 64;
        while (cap < 2 * (size_t)m + 2) cap <<= 1;
        slots.assign(cap, ~0ull);
        mask = (uint32_t)(cap - 1);
        c_of.resize((size_t)m);
        for (int64_t r = 0; r < m; ++r) {
            const uint32_t key = ((uint32_t)abc[3 * r] << 16) | (uint32_t)abc[3 * r + 1];
            c_of[(size_t)r] = abc[3 * r + 2];
            uint32_t h = (key * 0x9E3779B1u) & mask;
            while (slots[h] != ~0ull && (uint32_t)(slots[h] >> 32) != key) h = (h + 1) & mask;
            if (slots[h] == ~0ull) slots[h] = ((uint64_t)key << 32) | (uint32_t)r;   // first rank wins
        }
    }
    uint32_t rank(int32_t a, int32_t b) const {
        const uint32_t key = ((uint32_t)a << 16) | (uint32_t)b;
        uint32_t h = (key * 0x9E3779B1u) & mask;
        for (;;) {
            const uint64_t v = slots[h];
            if (v == ~0ull) return NO_RANK;
            if ((uint32_t)(v >> 32) == key) return (uint32_t)v;
            h = (h + 1) & mask;
        }
    }
};

struct Scratch {
    std::vector<int32_t> tok;
    std::vector<int32_t> nxt, prv;
    std::vector<uint64_t> heap;   // rank << 32 | position
};

// one text: n ids in, the encoded ids out (returns their count)
int64_t encode_one(const RankTable &T, const int32_t *in, int64_t n, int32_t *out, Scratch &S) {
    if (n < 2) {
        if (n == 1) out[0] = in[0];
        return n;
    }
    S.tok.assign(in, in + n);
    S.nxt.resize((size_t)n);
    S.prv.resize((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        S.nxt[(size_t)i] = (int32_t)(i + 1 < n ? i + 1 : -1);
        S.prv[(size_t)i] = (int32_t)(i - 1);
    }
    auto &H = S.heap;
    H.clear();
    for (int64_t i = 0; i + 1 < n; ++i) {
        const uint32_t r = T.rank(S.tok[(size_t)i], S.tok[(size_t)i + 1]);
        if (r != NO_RANK) H.push_back(((uint64_t)r << 32) | (uint64_t)i);
    }
    auto cmp = [](uint64_t x, uint64_t y) { return x > y; };   // (a min-heap)
    std::make_heap(H.begin(), H.end(), cmp);
    while (!H.empty()) {
        std::pop_heap(H.begin(), H.end(), cmp);
        const uint64_t top = H.back();
        H.pop_back();
        const uint32_t r = (uint32_t)(top >> 32);
        const int32_t p = (int32_t)(uint32_t)top;
        const int32_t q = S.nxt[(size_t)p];
        // stale: p merged away (tok < 0), or its right neighbour no longer makes rank r's pair
        if (S.tok[(size_t)p] < 0 || q < 0 || T.rank(S.tok[(size_t)p], S.tok[(size_t)q]) != r) continue;
        const int32_t c = T.c_of[r];
        S.tok[(size_t)p] = c;
        S.tok[(size_t)q] = -1;
        const int32_t q2 = S.nxt[(size_t)q];
        S.nxt[(size_t)p] = q2;
        if (q2 >= 0) S.prv[(size_t)q2] = p;
        const int32_t l = S.prv[(size_t)p];
        if (l >= 0) {
            const uint32_t rl = T.rank(S.tok[(size_t)l], c);
            if (rl != NO_RANK) {
                H.push_back(((uint64_t)rl << 32) | (uint64_t)(uint32_t)l);
                std::push_heap(H.begin(), H.end(), cmp);
            }
        }
        if (q2 >= 0) {
            const uint32_t rr = T.rank(c, S.tok[(size_t)q2]);
            if (rr != NO_RANK) {
                H.push_back(((uint64_t)rr << 32) | (uint64_t)(uint32_t)p);
                std::push_heap(H.begin(), H.end(), cmp);
            }
        }
    }
    int64_t k = 0;
    for (int32_t i = 0; i >= 0; i = S.nxt[(size_t)i]) out[k++] = S.tok[(size_t)i];
    return k;
}

}  // namespace

extern "C" {

// encodeToCode of n_texts texts (ids[off[k] .. off[k+1])) through the merges abc (a, b, c per
// rank) on `threads` threads (<= 0: all): out[out_off[k] .. out_off[k+1]) (out holds off[n] ids).
// Returns the threads used.
int cpu_encode_batch(const int32_t *ids, const int64_t *off, int64_t n_texts, const int32_t *abc,
                     int64_t n_merges, int32_t *out, int64_t *out_off, int threads) {
    RankTable T;
    T.build(abc, n_merges);
    if (threads <= 0) threads = omp_get_max_threads();
    std::vector<int64_t> len((size_t)std::max<int64_t>(n_texts, 1));
    // each text encodes in place in out at its input offset, then the results are packed
#pragma omp parallel num_threads(threads)
    {
        Scratch S;
#pragma omp for schedule(dynamic, 64)
        for (int64_t k = 0; k < n_texts; ++k)
            len[(size_t)k] = encode_one(T, ids + off[k], off[k + 1] - off[k], out + (off[k] - off[0]), S);
    }
    int64_t o = 0;
    out_off[0] = 0;
    for (int64_t k = 0; k < n_texts; ++k) {
        if (o != off[k] - off[0]) std::memmove(out + o, out + (off[k] - off[0]), (size_t)len[(size_t)k] * 4);
        o += len[(size_t)k];
        out_off[k + 1] = o;
    }
    return threads;
}

}  // extern "C"
