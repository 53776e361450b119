// bpe_engine.hip — libbpe: host side of the MI355X BPE merge-training engine + the C ABI of
// include/bpe.h.  One context = one HIP device + one stream + one corpus shard in HBM.
//
// The corpus is never compacted per merge: chunks stay left-packed and a merge rewrites only the
// chunks it touches.  One streaming kernel (k_step) does both halves of an iteration:
//   applyMerge(a, b, c)   (core.ts:332-360)  -> k_step<MERGE>: apply to every chunk, then count the
//                                               post-merge pairs, k_runs, k_reduce_hot
//   findNextMerge(opts)   (core.ts:247-326)  -> (k_step<plain> only if no counts are cached)
//                                               k_argmax_hot/cold, k_collect, [k_tie (rule R3)]
// so a mergeUntil iteration streams the corpus exactly once.
#include "bpe_kernels.hip.h"
#include "bpe_pix.hip.h"
#include "bpe.h"
#include "bpe_multi.h"
#include "bpe_tools.h"

namespace bpe_step {
// (csrc/bpe_step.hip: the C3 hot path's pass, compiled with its own flags; the structures are
// the ones of bpe_kernels.hip.h, passed untyped)
hipError_t launch_step_loop_table(unsigned grid, hipStream_t s, int32_t *ids, int64_t n_chunks,
                                  int64_t cpr, int R, const void *carry, const void *ctl,
                                  uint32_t *partials, unsigned long long *spill, const void *ct,
                                  void *sums, unsigned long long *replaced);
hipError_t launch_step_table(int merge, unsigned grid, hipStream_t s, int32_t *ids, int64_t n_chunks,
                             int64_t cpr, int R, const void *carry, int32_t ma, int32_t mb,
                             int32_t mc, uint32_t *partials, unsigned long long *spill,
                             const void *ct, const uint32_t *heavy, void *sums,
                             unsigned long long *replaced);
}

#include <algorithm>
#include <chrono>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

using namespace bpe;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return fail(e_ == hipErrorOutOfMemory ? BPE_ERR_OOM : BPE_ERR_HIP,             \
                        std::string("bpe native: ") + #expr + ": " + hipGetErrorString(e_)); \
    } while (0)

inline void dfree(void *p) {
    if (p) (void)hipFree(p);
}

// mergeUntil iterations the device runs per host round trip (each ends in one sync)
constexpr int64_t LOOP_BATCH = 64;
// apply-only replay: merges per host round trip (their replacement counts come back together)
constexpr int64_t REPLAY_BATCH = 256;

static_assert(TABLE_BINS == BPE_TABLE_BINS && HOT_BINS == BPE_HOT_BINS, "include/bpe.h table layout");
static_assert(MAX_CAND == BPE_MAX_CAND && LOOP_BATCH == BPE_LOOP_BATCH, "include/bpe.h rank loop sizes");
static_assert(XCHG_HDR == BPE_XCHG_HDR && XCHG_WORDS == BPE_XCHG_WORDS && TIE_WORDS == BPE_TIE_WORDS &&
                  DELTA_ROWS == BPE_DELTA_ROWS,
              "include/bpe.h exchange layout");

template <typename T>
int dev_alloc(T **p, size_t n) {
    *p = nullptr;
    if (n == 0) n = 1;
    hipError_t e = hipMalloc((void **)p, n * sizeof(T));
    if (e != hipSuccess)
        return fail(e == hipErrorOutOfMemory ? BPE_ERR_OOM : BPE_ERR_HIP,
                    std::string("bpe native: hipMalloc: ") + hipGetErrorString(e));
    return BPE_OK;
}

}  // namespace

struct bpe_ctx {
    // a corpus sharded over several devices (bpe_create_multi): every entry point forwards to
    // csrc/bpe_multi.cpp, which drives one single-device context per shard
    bpe_multi *multi = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;
    // corpus: n_chunks left-packed chunks + one all-SEP spare chunk
    int32_t *d_ids = nullptr, *d_tmp = nullptr;
    int64_t cap_slots = 0;
    int64_t n_chunks = 0;
    int64_t live_slots = 0;    // live slots (tokens + SEPs)
    int64_t n_samples = 0;
    int64_t n_live = 0;        // live tokens
    bool packed = true;        // live slots are a dense prefix (only the last chunk has a tail)
    // vocabulary
    std::vector<int32_t> h_len16;
    std::vector<int64_t> h_count;      // occurrences per token in the corpus (exact)
    int32_t *d_len16 = nullptr;
    int64_t cap_vocab = 0;
    int64_t len16_lo = 0;      // h_len16[len16_lo:] is not yet on the device
    // pass state
    uint32_t *d_partials = nullptr;
    int partials_wg = 0;         // workgroups the partial slab can hold
    unsigned long long *d_spill = nullptr, *d_hot = nullptr, *d_total = nullptr;   // d_hot: TABLE_BINS
    uint32_t *d_heavy = nullptr;
    RegionSum *d_sums = nullptr;
    RegionCarry *d_carry = nullptr;
    int64_t *d_outoff = nullptr;
    Result *d_res = nullptr, *h_res = nullptr;
    int2 *d_cand = nullptr;
    ColdTable cold{};
    // [0] n_used, [1] overflow, [2] n_blist, [3] sel_n0, [4] dead, [5] n_recomputed (ColdTable)
    uint32_t *d_cold_flags = nullptr;
    uint64_t cold_cap = 0;
    // an applied merge whose replacement count is still on the device (settled at the next sync)
    bool pending = false;
    int32_t pend_a = 0, pend_b = 0, pend_c = 0;
    int64_t pend_expect = -1;    // W the replacement count must equal (mergeUntil), -1 = any
    int2 *h_cand = nullptr;      // pinned: first MAX_CAND candidates come back with the Result
    bool counts_valid = false;   // d_hot + cold table describe the current corpus
    // d_hot's sketch half is an upper bound of the cold pairs' counts.  A MODE_FUSED pass leaves
    // it garbage (its LDS half holds the refresh hash there): every reader of the sketch recounts
    // first (table_ok)
    bool sketch_valid = false;
    uint64_t cold_used = 0;      // n_used of the cold table last reported to the host
    // The cold table holds the exact count of EVERY cold pair and is kept so merge by merge
    // (cold_refresh) instead of being rebuilt by exact passes: entered after consecutive exact
    // passes (a corpus whose winners are pairs of merged tokens, e.g. Zipf words)
    bool cold_exact = false;
    int exact_streak = 0;
    // with the cold table maintained, merge passes count incrementally (MODE_INCR: the hot bins are
    // maintained too, and a pass counts only the pairs the merge can change); BPE_FUSED=1 keeps
    // the full hot recount with the cold refresh riding along (MODE_FUSED) instead
    bool use_incr = true;
    // mergeUntil on the position index (bpe_set_mode BPE_MODE_INCREMENTAL, BPE_PIX=1): O(W) work
    // per merge instead of a pass (bpe_pix.hip.h)
    bool use_pix = false;
    struct PixState *pix = nullptr;
    bool carry_valid = false;    // d_sums / d_carry describe the current corpus and geometry
    int64_t cpr = 0;
    int R = 0, G = 0;
    int64_t last_replaced = 0;
    // best hot key of d_hot computed by the last k_reduce_table (valid for best_ml)
    bool best_ready = false;
    int64_t best_ml = 0;
    int64_t opt_max_length = 0;   // max_length of the last find (the reduce's filter)
    // stats: kernel spans are timed with events read back lazily (no sync in the merge loop)
    bool stats_on = false;
    bool span_mute = false;   // the device loop's untimed iterations (events cost ~µs each)
    uint64_t span_tick = 0;
    bpe_stats stats{};
    struct Span {
        hipEvent_t a, b;
        int kind;   // 0 stream pass, 1 selection, 2 tie pass
    };
    std::vector<Span> spans;
    std::vector<hipEvent_t> ev_pool;
    // device-resident mergeUntil loop: control block + merge log (pinned host mirrors)
    LoopCtl *d_ctl = nullptr, *h_ctl = nullptr;
    long long *d_log = nullptr, *h_log = nullptr;
    unsigned int *d_ticket = nullptr;   // last-block tickets (k_tie_fused, k_select_maint; zero between launches)
    BlockBest *d_brec = nullptr;        // k_select_maint's per-block bests
    // apply-only replay: per-merge replacement counts
    unsigned long long *d_repl = nullptr, *h_repl = nullptr;
    // sharded device loop (one rank): the caller's all-reduced exchange buffer (include/bpe.h
    // BPE_XCHG_*: header + this shard's table, or + the delta rows) and tie positions
    unsigned long long *rl_table = nullptr, *rl_tie = nullptr;
    int rl_rank = 0, rl_world = 1;
    int64_t rl_base = 0, rl_enqueued = 0, rl_max_length = 0;
    int64_t rl_words = 0;   // words of the exchange all-reduced per iteration (this batch)
    bool rl_open = false;
    // d_hot and the cold table hold the GLOBAL counts of a sharded corpus, replicated on every
    // rank (bpe_set_global_counts): the rank loop keeps them merge by merge from the all-reduced
    // delta rows.  Anything that needs this shard's own counts leaves that state first.
    bool rl_global = false;
    // the last batch's last merge left its delta rows in rl_table, not yet all-reduced: the next
    // batch's first exchange carries them (same buffer)
    bool rl_delta_pending = false;
    int32_t rl_last_a = 0, rl_last_b = 0, rl_last_c = 0;
    int64_t rl_last_w = -1;
    // the cold table holds this shard's exact count of every cold pair (bpe_cold_counts)
    bool cold_list = false;
    // the global state of a sharded corpus lives in the position index (bpe_set_mode
    // BPE_MODE_INCREMENTAL, bpe_pix.hip.h): c->pix holds this shard's lists and the GLOBAL counts
    // between rank loop batches, and the corpus is in the index's slot layout until it is dropped
    bool rl_pix = false;
    uint64_t pix_min_cap = 0;    // (the next index build's least table size)
    // sharded incremental mode, compact exchange: entries of L and of R the next batch's exchange
    // holds (0: not known yet, every token id; sized from the largest need of the batches before)
    // the lane layout of the sharded incremental exchange: the last merge's count (0: unknown),
    // the layout {bits, lanes per word, right side's first word} of this batch and of the batch
    // whose last merge's lanes are pending
    unsigned long long pix_w_last = 0;
    uint32_t pix_lane[3] = {0, 0, 0}, pix_lane_prev[3] = {0, 0, 0};
    int64_t pix_nw_last = 0;   // words the last rank-loop batch all-reduced (its pending merge's)
    bool pix_first_pending = false;
};

namespace {

int set_device(bpe_ctx *c) {
    HIP_TRY(hipSetDevice(c->device));
    return BPE_OK;
}

}  // namespace
int pix_finish(bpe_ctx *c);
namespace {

// Before anything that reads or updates this shard's own counts: global tables (the sharded
// maintained state) are dropped, and the next use recounts.  A sharded position index is dropped
// too: the corpus goes back to the chunk layout.
int leave_global(bpe_ctx *c) {
    if (!c->rl_global) return BPE_OK;
    c->rl_global = false;
    c->rl_delta_pending = false;
    c->counts_valid = c->sketch_valid = c->best_ready = false;
    c->cold_exact = false;
    c->cold_list = false;
    if (c->rl_pix) {
        c->rl_pix = false;
        return pix_finish(c);
    }
    return BPE_OK;
}
#define LEAVE_GLOBAL(c)                   \
    do {                                  \
        const int lg_ = leave_global(c);  \
        if (lg_) return lg_;              \
    } while (0)

void geometry(bpe_ctx *c) {
    const int64_t nc = std::max<int64_t>(1, c->n_chunks);
    c->cpr = (nc + MAX_REGIONS - 1) / MAX_REGIONS;
    c->R = (int)((nc + c->cpr - 1) / c->cpr);
    c->G = (c->R + WAVES_PER_WG - 1) / WAVES_PER_WG;
}

// Capacity for `chunks` data chunks + the spare chunk, in both buffers.  Preserves the data.
int ensure_chunks(bpe_ctx *c, int64_t chunks) {
    const int64_t want = (chunks + 1) * CHUNK;
    if (want <= c->cap_slots) return BPE_OK;
    int64_t cap = std::max<int64_t>(want, c->cap_slots * 3 / 2);
    cap = (cap + CHUNK - 1) / CHUNK * CHUNK;
    int32_t *ids, *tmp;
    int rc;
    if ((rc = dev_alloc(&ids, cap))) return rc;
    if ((rc = dev_alloc(&tmp, cap))) {
        dfree(ids);
        return rc;
    }
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)ids, SEP, cap, c->stream));
    if (c->d_ids && c->n_chunks)
        HIP_TRY(hipMemcpyAsync(ids, c->d_ids, c->n_chunks * CHUNK * sizeof(int32_t),
                               hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    dfree(c->d_ids);
    dfree(c->d_tmp);
    c->d_ids = ids;
    c->d_tmp = tmp;
    c->cap_slots = cap;
    return BPE_OK;
}

// After writing live slots [0, live_slots) densely: TOMB to the end of the last chunk, SEP spare.
int seal_packed(bpe_ctx *c) {
    c->n_chunks = (c->live_slots + CHUNK - 1) / CHUNK;
    const int64_t end = c->n_chunks * CHUNK;
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)(c->d_ids + end), SEP, CHUNK, c->stream));
    if (end > c->live_slots) {
        k_seal<<<1, CHUNK, 0, c->stream>>>(c->d_ids, c->live_slots);
        HIP_TRY(hipGetLastError());
    }
    c->packed = true;
    c->counts_valid = c->carry_valid = false;
    c->cold_exact = false;
    c->rl_global = c->rl_delta_pending = false;
    c->cold_list = false;
    geometry(c);
    return BPE_OK;
}

void mark_len16(bpe_ctx *c, int64_t i) { c->len16_lo = std::min(c->len16_lo, i); }

// Room for ids [0, n) in the device length table (the host tables are not extended).
int ensure_len16_cap(bpe_ctx *c, int64_t n) {
    if (n > c->cap_vocab) {
        int64_t cap = std::max<int64_t>(n, std::max<int64_t>(1024, c->cap_vocab * 2));
        dfree(c->d_len16);
        int rc = dev_alloc(&c->d_len16, cap);
        if (rc) return rc;
        c->cap_vocab = cap;
        c->len16_lo = 0;   // a fresh device buffer
    }
    return BPE_OK;
}

int ensure_vocab(bpe_ctx *c, int64_t n) {
    if ((int64_t)c->h_len16.size() < n) {
        mark_len16(c, (int64_t)c->h_len16.size());
        c->h_len16.resize(n, 1);
        c->h_count.resize(n, 0);
    }
    return ensure_len16_cap(c, n);
}

// The UTF-16 length table is read on the device only by the max_length filter (core.ts:270-273),
// so it is brought up to date lazily and incrementally (a merge adds one entry).
int sync_len16(bpe_ctx *c, int64_t max_length) {
    const int64_t n = (int64_t)c->h_len16.size();
    if (!max_length || c->len16_lo >= n) return BPE_OK;
    if (c->h_len16.empty()) return BPE_OK;
    HIP_TRY(hipMemcpyAsync(c->d_len16 + c->len16_lo, c->h_len16.data() + c->len16_lo,
                           (n - c->len16_lo) * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    c->len16_lo = n;
    return BPE_OK;
}

// Upper bound on distinct cold pairs in the next pass: every counted pair with an id >= HOT
// involves a cold-token occurrence, and each occurrence sits in at most two pairs.  `extra` bounds
// the occurrences of a token created by the pass itself.
// grid of the scans over the cold table's dense view (>= HOT_BINS / 256 for k_collect)
constexpr int COLD_GRID = 1024;
static_assert(COLD_GRID * 256 >= HOT_BINS, "k_collect covers the hot bins");
static_assert(COLD_GRID <= TK_GROUP * TK_MAX_GROUPS && (MAX_REGIONS + 3) / 4 <= TK_GROUP * TK_MAX_GROUPS,
              "grid_last's counters cover k_select_maint's and k_tie_fused's grids");

// Empties the cold table: free slots, zero dense counts (the invariant past n_used), n_used = 0.
int cold_clear(bpe_ctx *c) {
    c->cold_list = false;
    HIP_TRY(hipMemsetAsync(c->cold.slots, 0xFF, c->cold_cap * sizeof(unsigned long long), c->stream));
    HIP_TRY(hipMemsetAsync(c->cold.dcounts, 0, c->cold_cap * sizeof(unsigned long long), c->stream));
    HIP_TRY(hipMemsetAsync(c->d_cold_flags, 0, 5 * sizeof(uint32_t), c->stream));
    // (the block maxima: no block flagged; the next selection of a batch is a full scan)
    HIP_TRY(hipMemsetAsync(c->cold.bdirty, 0, (c->cold_cap / CB + 1) * sizeof(uint32_t), c->stream));
    c->cold_used = 0;
    return BPE_OK;
}

// the cold table's capacity for a pass that creates at most `extra` cold-token occurrences
uint64_t cold_cap_for(const bpe_ctx *c, uint64_t extra, uint64_t min_cap = 0) {
    uint64_t s = extra;
    for (size_t t = HOT; t < c->h_count.size(); ++t) s += (uint64_t)std::max<int64_t>(0, c->h_count[t]);
    uint64_t need = 2 * s + 16;
    const uint64_t V = c->h_len16.size() + 1;
    need = std::min<uint64_t>(need, V * V);
    need = std::min<uint64_t>(need, (uint64_t)c->n_live + 16);
    uint64_t cap = 1024;
    while (cap < 2 * need || cap < min_cap) cap <<= 1;
    return cap;
}

// (reallocates empty when it grows: the contents are lost, cold_rebuild keeps them)
int ensure_cold(bpe_ctx *c, uint64_t extra, uint64_t min_cap = 0) {
    const uint64_t cap = cold_cap_for(c, extra, min_cap);
    if (cap <= c->cold_cap) return BPE_OK;
    if (cap > (1ull << 31)) return fail(BPE_ERR_OOM, "bpe native: cold pair table too large");
    HIP_TRY(hipStreamSynchronize(c->stream));
    dfree(c->cold.slots);
    dfree(c->cold.dkeys);
    dfree(c->cold.dcounts);
    dfree(c->cold.bmax);
    dfree(c->cold.bdirty);
    dfree(c->cold.blist);
    int rc;
    if ((rc = dev_alloc(&c->cold.slots, cap))) return rc;
    if ((rc = dev_alloc(&c->cold.dkeys, cap))) return rc;
    if ((rc = dev_alloc(&c->cold.dcounts, cap))) return rc;
    if ((rc = dev_alloc(&c->cold.bmax, cap / CB + 1))) return rc;
    if ((rc = dev_alloc(&c->cold.bdirty, cap / CB + 1))) return rc;
    if ((rc = dev_alloc(&c->cold.blist, cap / CB + 1))) return rc;
    c->cold_cap = cap;
    c->cold.mask = (uint32_t)(cap - 1);
    int lg = 0;
    while ((1ull << lg) < cap) ++lg;
    c->cold.shift = 32 - lg;
    c->cold.n_used = c->d_cold_flags;
    c->cold.overflow = c->d_cold_flags + 1;
    c->cold.n_blist = c->d_cold_flags + 2;
    c->cold.sel_n0 = c->d_cold_flags + 3;
    c->cold.dead = c->d_cold_flags + 4;
    c->cold.n_recomputed = c->d_cold_flags + 5;
    c->counts_valid = false;
    c->cold_exact = false;
    return cold_clear(c);
}

// The maintained cold table rebuilt from itself (round 5): its live claims (a count > 0: every
// cold pair of the corpus, the table being exact) gathered out, then loaded into a cleared table
// of at least min_cap slots and four times their number, so that the dead claims and the holes go
// and the fill drops to a quarter.  The exact pass over the corpus it replaces took 8 ms on 1 GiB
// of zipf words, plus the table-state iterations until the maintained state was entered again.
// BPE_COLD_REBUILD=0: the exact pass instead (A/B; read per call).  (Rebuilding also ahead of a
// batch at half fill, so that the batch hands no iteration over for it, timed 0.2 % slower on
// zipf C3: profiles/r05_ab_cold_rebuild.txt)
bool cold_rebuild_on() {
    const char *e = getenv("BPE_COLD_REBUILD");
    return !e || atoi(e) != 0;
}

int cold_rebuild(bpe_ctx *c, uint64_t min_cap) {
    hipStream_t s = c->stream;
    uint32_t flags[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(flags, c->d_cold_flags, sizeof flags, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (flags[1]) return fail(BPE_ERR_STATE, "bpe native: cold pair table overflow");
    const uint64_t n = std::min<uint64_t>(flags[0], c->cold_cap);
    // (the temporary lists are freed on every way out, HIP_TRY's early returns included)
    struct Scratch {
        hipStream_t s;
        uint32_t *keys = nullptr, *d_m = nullptr;
        unsigned long long *counts = nullptr;
        ~Scratch() {
            (void)hipStreamSynchronize(s);
            dfree(keys);
            dfree(counts);
            dfree(d_m);
        }
    } t{s};
    int rc;
    if ((rc = dev_alloc(&t.keys, std::max<uint64_t>(n, 1))) ||
        (rc = dev_alloc(&t.counts, std::max<uint64_t>(n, 1))) || (rc = dev_alloc(&t.d_m, 1)))
        return rc;
    HIP_TRY(hipMemsetAsync(t.d_m, 0, sizeof(uint32_t), s));
    k_cold_gather<<<COLD_GRID, 256, 0, s>>>(c->cold, t.keys, t.counts, t.d_m);
    HIP_TRY(hipGetLastError());
    uint32_t m = 0;
    HIP_TRY(hipMemcpyAsync(&m, t.d_m, sizeof m, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    // (a table that grows is reallocated empty, which drops the maintained state: restored once
    // the live claims are back)
    const bool counts_valid = c->counts_valid, cold_exact = c->cold_exact;
    for (int attempt = 0;; ++attempt) {
        if ((rc = ensure_cold(c, 0, std::max<uint64_t>(min_cap, 4 * (uint64_t)m + 4096)))) return rc;
        if ((rc = cold_clear(c))) return rc;
        if (m) k_load_cold<<<COLD_GRID, 256, 0, s>>>(c->cold, t.keys, t.counts, m);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(flags, c->d_cold_flags, sizeof flags, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (!flags[1]) break;
        if (attempt == 2) return fail(BPE_ERR_STATE, "bpe native: cold pair table overflow");
        min_cap = 2 * c->cold_cap;
    }
    c->cold_used = flags[0];
    c->counts_valid = counts_valid;
    c->cold_exact = cold_exact;
    if (c->stats_on) c->stats.cold_rebuilds += 1;
    return BPE_OK;
}

float ev_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

hipEvent_t take_event(bpe_ctx *c) {
    hipEvent_t e = nullptr;
    if (!c->ev_pool.empty()) {
        e = c->ev_pool.back();
        c->ev_pool.pop_back();
    } else if (hipEventCreate(&e) != hipSuccess) {
        e = nullptr;
    }
    return e;
}

// Starts a timed span on the stream (nullptr when stats are off).
constexpr uint64_t SPAN_EVERY = 8;

hipEvent_t span_begin(bpe_ctx *c) {
    if (!c->stats_on || c->span_mute) return nullptr;
    hipEvent_t e = take_event(c);
    if (e) (void)hipEventRecord(e, c->stream);
    return e;
}

// Reads every finished span into the stats and recycles the events.
int flush_spans(bpe_ctx *c) {
    if (c->spans.empty()) return BPE_OK;
    HIP_TRY(hipEventSynchronize(c->spans.back().b));
    for (auto &sp : c->spans) {
        const double ms = ev_ms(sp.a, sp.b);
        if (sp.kind == 0 || sp.kind == 2) {   // (2: a maintained-state pass, MODE_INCR)
            c->stats.step_ms += ms;
            c->stats.step_timed += 1;
            if (sp.kind == 2) {
                c->stats.incr_ms += ms;
                c->stats.incr_timed += 1;
            }
        }
        else c->stats.select_ms += ms;
        c->ev_pool.push_back(sp.a);
        c->ev_pool.push_back(sp.b);
    }
    c->spans.clear();
    return BPE_OK;
}

int span_end(bpe_ctx *c, hipEvent_t a, int kind) {
    if (!a) return BPE_OK;
    hipEvent_t b = take_event(c);
    if (!b) return fail(BPE_ERR_HIP, "bpe native: event");
    HIP_TRY(hipEventRecord(b, c->stream));
    c->spans.push_back({a, b, kind});
    if (c->spans.size() >= 1024) return flush_spans(c);
    return BPE_OK;
}

// One streaming pass: (optionally apply the merge a,b -> cc, then) count every pair, stitch the
// region boundaries and reduce the hot table.  Leaves counts + carries valid for the new corpus.
// With a merge, *replaced receives the number of replacements.
int settle(bpe_ctx *c);
int settle_with(bpe_ctx *c, unsigned long long R);
int maybe_compact(bpe_ctx *c);

// One 160 KiB slab per workgroup of a counting pass (for the current geometry).
int ensure_partials(bpe_ctx *c) {
    geometry(c);
    if (c->G > c->partials_wg) {
        HIP_TRY(hipStreamSynchronize(c->stream));
        dfree(c->d_partials);
        c->d_partials = nullptr;
        c->partials_wg = 0;
        int rc = dev_alloc(&c->d_partials, (size_t)c->G * HIST_WORDS);
        if (rc) return rc;
        c->partials_wg = c->G;
    }
    return BPE_OK;
}

// fused: a merge pass that also refreshes the maintained cold table (MODE_FUSED; the caller
// invalidates the pairs with a side a or b before it and syncs the dense view after it)
int run_pass(bpe_ctx *c, bool merge, int32_t a, int32_t b, int32_t cc, int64_t *replaced,
             bool fused = false) {
    int rc;
    if (merge && c->pending)
        if ((rc = settle(c))) return rc;
    if ((rc = ensure_partials(c))) return rc;
    c->cold_list = false;   // (fused and incremental passes update the cold table)
    if ((rc = sync_len16(c, c->opt_max_length))) return rc;   // the reduce's max_length filter
    hipStream_t s = c->stream;
    // the spill is zero here: zeroed once at create, then by every k_reduce_table
    HIP_TRY(hipMemsetAsync(c->d_res, 0, sizeof(Result), s));
    hipEvent_t e_step = span_begin(c);
    const bool incr = merge && fused && c->use_incr;
    if (incr) {
        k_incr_invalidate<<<COLD_GRID, 256, 0, s>>>(c->cold, c->d_hot, a, b);
        if (a == b)
            k_step<MERGE_XX, MODE_INCR><<<c->G, WG, 0, s>>>(
                c->d_ids, c->n_chunks, c->cpr, c->R, c->d_carry, a, b, cc, c->d_partials,
                c->d_spill, c->cold, c->d_heavy, c->d_sums, &c->d_res->replaced, c->d_hot);
        else
            k_step<MERGE_XY, MODE_INCR><<<c->G, WG, 0, s>>>(
                c->d_ids, c->n_chunks, c->cpr, c->R, c->d_carry, a, b, cc, c->d_partials,
                c->d_spill, c->cold, c->d_heavy, c->d_sums, &c->d_res->replaced, c->d_hot);
    } else if (merge && fused && a == b)
        k_step<MERGE_XX, MODE_FUSED><<<c->G, WG, 0, s>>>(
            c->d_ids, c->n_chunks, c->cpr, c->R, c->d_carry, a, b, cc, c->d_partials, c->d_spill,
            c->cold, c->d_heavy, c->d_sums, &c->d_res->replaced);
    else if (merge && fused)
        k_step<MERGE_XY, MODE_FUSED><<<c->G, WG, 0, s>>>(
            c->d_ids, c->n_chunks, c->cpr, c->R, c->d_carry, a, b, cc, c->d_partials, c->d_spill,
            c->cold, c->d_heavy, c->d_sums, &c->d_res->replaced);
    else
        HIP_TRY(bpe_step::launch_step_table(!merge ? NO_MERGE : a == b ? MERGE_XX : MERGE_XY, c->G,
                                            s, c->d_ids, c->n_chunks, c->cpr, c->R, c->d_carry,
                                            merge ? a : -1, merge ? b : -1, merge ? cc : -1,
                                            c->d_partials, c->d_spill, &c->cold, c->d_heavy,
                                            c->d_sums, &c->d_res->replaced));
    HIP_TRY(hipGetLastError());
    if ((rc = span_end(c, e_step, 0))) return rc;
    hipEvent_t e_red = span_begin(c);
    if (incr) {
        // the touched pairs into the maintained tables, then the best hot key
        k_runs<MODE_INCR><<<(c->R + 255) / 256, 256, 0, s>>>(
            c->d_sums, c->R, c->d_carry, c->d_spill, c->cold, c->d_heavy, nullptr, a, b, cc,
            c->d_hot);
        k_reduce_rows<<<4 * INCR_RLIM / 2 / RR_COLS, 256, 0, s>>>(
            c->d_partials, c->G, c->d_spill, c->d_hot, c->cold, a, b, cc);
        k_argmax_hot<<<HOT_BINS / 256, 256, 0, s>>>(c->d_hot, c->d_len16, c->opt_max_length,
                                                    c->d_res);
    } else {
        if (merge && fused)
            k_runs<MODE_FUSED><<<(c->R + 255) / 256, 256, 0, s>>>(
                c->d_sums, c->R, c->d_carry, c->d_spill, c->cold, c->d_heavy, nullptr, a, b, cc);
        else
            k_runs<MODE_TABLE><<<(c->R + 255) / 256, 256, 0, s>>>(
                c->d_sums, c->R, c->d_carry, c->d_spill, c->cold, c->d_heavy, nullptr);
        k_reduce_table<<<HIST_WORDS / REDUCE_WORDS_PER_BLOCK, REDUCE_THREADS, 0, s>>>(
            c->d_partials, c->G, c->d_spill, c->d_hot, c->d_len16, c->opt_max_length, c->d_res,
            nullptr);
    }
    HIP_TRY(hipGetLastError());
    if ((rc = span_end(c, e_red, 1))) return rc;
    c->best_ready = true;
    c->best_ml = c->opt_max_length;
    if (c->stats_on) {
        c->stats.step_launches += 1;
        c->stats.step_slots += c->n_chunks * CHUNK;
        c->stats.step_live += c->n_live;
    }
    if (merge) {
        // the replacement count stays on the device until the next sync point (settle)
        c->pending = true;
        c->pend_a = a;
        c->pend_b = b;
        c->pend_c = cc;
        c->pend_expect = -1;
        if (replaced) {
            int rc2 = settle(c);
            if (rc2) return rc2;
            *replaced = c->last_replaced;
        }
    }
    c->counts_valid = true;
    c->carry_valid = true;
    c->sketch_valid = !(merge && fused);
    if (merge && fused && c->stats_on) c->stats.fused_passes += 1;
    return BPE_OK;
}

// d_hot holds this corpus's counts with a usable sketch (the hot bins and the sketch bound)
bool table_ok(const bpe_ctx *c) { return c->counts_valid && c->sketch_valid; }

// Host accounting of an applied merge once its replacement count R is known.
int settle_with(bpe_ctx *c, unsigned long long Ru) {
    if (!c->pending) return BPE_OK;
    c->pending = false;
    const int64_t R = (int64_t)Ru;
    c->last_replaced = R;
    c->n_live -= R;
    c->live_slots -= R;
    c->h_count[c->pend_a] -= R;
    c->h_count[c->pend_b] -= R;
    c->h_count[c->pend_c] += R;
    if (R) c->packed = false;
    if (c->pend_expect >= 0 && R != c->pend_expect)
        return fail(BPE_ERR_STATE, "bpe native: replacement count != W");
    return BPE_OK;
}

int settle(bpe_ctx *c) {
    // (a sharded position index between rank loop batches: anything else reads the chunk layout)
    if (c->rl_pix && !c->rl_open) LEAVE_GLOBAL(c);
    if (!c->pending) return BPE_OK;
    unsigned long long R = 0;
    HIP_TRY(hipMemcpyAsync(&R, &c->d_res->replaced, sizeof R, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return settle_with(c, R);
}

// Moves the live slots to a dense prefix (when dead slots waste too much of the stream, and
// before appending to a merged corpus).  Needs valid region sums; leaves counts valid (they do
// not depend on the layout) but invalidates the carries (the geometry changes).
int compact(bpe_ctx *c) {
    int rc;
    if (c->packed) return BPE_OK;
    if (!c->carry_valid)
        if ((rc = run_pass(c, false, 0, 0, 0, nullptr))) return rc;
    hipStream_t s = c->stream;
    k_scan_live<<<1, 1024, 0, s>>>(c->d_sums, c->R, c->d_outoff, c->d_total);
    // (no fill of the target first: k_compact writes the live prefix and seal_packed the last
    // chunk's tail and the spare chunk, the only slots past the prefix that anything reads.  A
    // fill of the whole buffer cost ~0.7 ms per compaction, 58 of them on zipf C3)
    k_compact<<<(c->R + 3) / 4, 256, 0, s>>>(c->d_ids, c->n_chunks, c->cpr, c->R, c->d_outoff,
                                             c->d_tmp);
    HIP_TRY(hipGetLastError());
    unsigned long long total = 0;
    HIP_TRY(hipMemcpyAsync(&total, c->d_total, sizeof total, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if ((int64_t)total != c->live_slots)
        return fail(BPE_ERR_STATE, "bpe native: compaction lost slots");
    std::swap(c->d_ids, c->d_tmp);
    const bool counts = c->counts_valid, cold_exact = c->cold_exact, sketch = c->sketch_valid;
    const bool glob = c->rl_global, pend = c->rl_delta_pending, list = c->cold_list;
    if ((rc = seal_packed(c))) return rc;
    c->counts_valid = counts;
    c->sketch_valid = sketch;
    c->cold_exact = cold_exact;
    c->rl_global = glob;
    c->rl_delta_pending = pend;
    c->cold_list = list;
    if (c->stats_on) c->stats.compactions += 1;
    return BPE_OK;
}

// Dead slots past the compaction threshold.
bool compaction_due(const bpe_ctx *c);

int maybe_compact(bpe_ctx *c) {
    if (!compaction_due(c)) return BPE_OK;
    int rc = compact(c);
    if (rc) return rc;
    return run_pass(c, false, 0, 0, 0, nullptr);         // rebuild carries for the new layout
}

bool compaction_due(const bpe_ctx *c) {
    const int64_t slots = c->n_chunks * CHUNK;
    if (c->packed || slots < (1 << 20)) return false;
    // dead slots cost a pass as much as live ones: re-pack once they are 1% of the stream (a
    // compaction costs about three passes; at C3 merge rates that is every ~700 merges; 3% timed
    // 0.8% slower per pass over the full C3 run)
    static const int keep_pct = [] {
        const char *v = getenv("BPE_COMPACT_LIVE_PCT");   // (A/B knob: live share kept, 90..99)
        const int p = v ? atoi(v) : 99;
        return p >= 90 && p <= 99 ? p : 99;
    }();
    return c->live_slots * 100 < slots * keep_pct;
}

// Exact counts of the cold pairs in the sketch buckets marked in d_heavy, into the sparse table
// (one more streaming pass; only when some bucket could still reach the best hot count).
int exact_pass(bpe_ctx *c) {
    int rc;
    c->cold_exact = false;   // (the table is rebuilt for the marked buckets only)
    if ((rc = ensure_cold(c, 0))) return rc;
    if (!c->carry_valid)
        if ((rc = run_pass(c, false, 0, 0, 0, nullptr))) return rc;
    geometry(c);
    hipStream_t s = c->stream;
    uint32_t flags[2] = {0, 0};
    for (int attempt = 0;; ++attempt) {
        if ((rc = cold_clear(c))) return rc;
        k_step<NO_MERGE, MODE_EXACT><<<c->G, WG, 0, s>>>(
            c->d_ids, c->n_chunks, c->cpr, c->R, c->d_carry, -1, -1, -1, c->d_partials,
            c->d_spill, c->cold, c->d_heavy, c->d_sums, &c->d_res->replaced);
        k_runs<MODE_EXACT><<<(c->R + 255) / 256, 256, 0, s>>>(c->d_sums, c->R, c->d_carry,
                                                              c->d_spill, c->cold, c->d_heavy,
                                                              nullptr);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(flags, c->d_cold_flags, sizeof flags, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (!flags[1]) break;
        // the distinct pairs fit by construction; claims that lost a race (holes) did not:
        // a table twice as large, and the pass again
        if (attempt == 2) return fail(BPE_ERR_STATE, "bpe native: cold pair table overflow");
        if ((rc = ensure_cold(c, 0, 2 * c->cold_cap))) return rc;
    }
    c->cold_used = flags[0];
    if (c->stats_on) c->stats.exact_passes += 1;
    return BPE_OK;
}

// select_from_table: the maintained cold table overflowed, select again after a recount
constexpr int SELECT_RETRY = 100;

// Best hot pair + heavy sketch buckets for `table` (a [TABLE_BINS] u64 table on the device);
// then, when some bucket is heavy, the exact pass; then every pair sharing the best key.
// Leaves the Result in h_res and the candidates in `cand`.
int select_from_table(bpe_ctx *c, const unsigned long long *table, int64_t max_length,
                      bool local, std::vector<int2> &cand, hipEvent_t e_sel) {
    int rc;
    if ((rc = sync_len16(c, max_length))) return rc;
    hipStream_t s = c->stream;
    const bool maintained = local && c->cold_exact;
    if (maintained) {
        // the maintained cold table holds every cold pair exactly (the sketch is not consulted):
        // best hot key, then the cold argmax and every pair sharing the best, one host round trip
        if (table == c->d_hot && c->best_ready && c->best_ml == max_length) {
            HIP_TRY(hipMemsetAsync(&c->d_res->n_cand, 0, 2 * sizeof(unsigned), s));
        } else {
            k_select<<<1, 1024, 0, s>>>(table, c->d_len16, max_length, c->d_res, c->d_cand,
                                       c->d_heavy);
            HIP_TRY(hipMemsetAsync(&c->d_res->n_cand, 0, sizeof(unsigned), s));
        }
        c->best_ready = false;
        HIP_TRY(hipMemsetAsync(&c->d_res->cold_dead, 0, sizeof(unsigned long long), s));
        k_argmax_cold<<<COLD_GRID, 256, 0, s>>>(c->cold, c->d_len16, max_length, c->d_res);
        k_collect<<<COLD_GRID, 256, 0, s>>>(table, c->cold, c->d_len16, max_length, c->d_res,
                                            c->d_cand);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(c->h_res, c->d_res, sizeof(Result), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(c->h_cand, c->d_cand, MAX_CAND * sizeof(int2), hipMemcpyDeviceToHost, s));
        if ((rc = span_end(c, e_sel, 1))) return rc;
        HIP_TRY(hipStreamSynchronize(s));
        if ((rc = settle_with(c, c->h_res->replaced))) return rc;
        const uint64_t flags = c->h_res->cold_flags;
        c->cold_used = flags & 0xFFFFFFFFu;
        if (flags >> 32) {
            // a refresh claimed more slots than the table has: this selection cannot be
            // trusted.  Leave the maintained state; the caller recounts and selects again (plain
            // pass, then exact passes that rebuild the table)
            c->cold_exact = false;
            c->counts_valid = false;
            c->exact_streak = 1;
            return SELECT_RETRY;
        }
        if ((flags & 0xFFFFFFFFu) * 4 > c->cold_cap * 3 ||
            2 * c->h_res->cold_dead > (flags & 0xFFFFFFFFu) + 65536) {
            // too full to probe well, or mostly claims whose pair is gone (every scan streams
            // them): this selection has read it (its result is on the host); rebuilt from its
            // own live claims, it stays the maintained table (BPE_COLD_REBUILD=0: the exact pass
            // over the corpus at the next selection, as before round 5)
            if (cold_rebuild_on()) {
                if ((rc = cold_rebuild(c, 0))) return rc;
            } else {
                c->cold_exact = false;
                c->exact_streak = 1;
            }
        }
    } else if (local && table == c->d_hot && c->best_ready && c->best_ml == max_length) {
        // the reduce already left the best hot key in the Result: collect its pairs and the
        // heavy sketch buckets with the whole chip
        HIP_TRY(hipMemsetAsync(&c->d_res->n_cand, 0, 2 * sizeof(unsigned), s));
        k_select_multi<<<TABLE_BINS / 256, 256, 0, s>>>(table, c->d_len16, max_length, c->d_res,
                                                        c->d_cand, c->d_heavy, nullptr);
    } else {
        k_select<<<1, 1024, 0, s>>>(table, c->d_len16, max_length, c->d_res, c->d_cand, c->d_heavy);
    }
    if (!maintained) {
    c->best_ready = false;
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(c->h_res, c->d_res, sizeof(Result), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(c->h_cand, c->d_cand, MAX_CAND * sizeof(int2), hipMemcpyDeviceToHost, s));
    if ((rc = span_end(c, e_sel, 1))) return rc;
    HIP_TRY(hipStreamSynchronize(s));
    if ((rc = settle_with(c, c->h_res->replaced))) return rc;   // a pending apply's R came along
    if (local && !c->h_res->n_heavy && !c->cold_exact) c->exact_streak = 0;
    if (local && (c->h_res->n_heavy || c->cold_exact)) {
        // some cold pair may still reach W: count those exactly (or read the maintained table),
        // then recollect hot + cold
        if (!c->cold_exact) {
            // the second exact pass in a row counts every cold pair and keeps the table
            const bool full = ++c->exact_streak >= 2;
            if (full) HIP_TRY(hipMemsetAsync(c->d_heavy, 0xFF, HEAVY_WORDS * sizeof(uint32_t), s));
            if ((rc = exact_pass(c))) return rc;
            c->cold_exact = full;
        } else {
            uint32_t flags[2] = {0, 0};
            HIP_TRY(hipMemcpyAsync(flags, c->d_cold_flags, sizeof flags, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            if (flags[1]) return fail(BPE_ERR_STATE, "bpe native: cold pair table overflow");
            if ((uint64_t)flags[0] * 4 > c->cold_cap * 3) {
                // too full to probe well: this selection still reads it, the next one rebuilds it
                c->cold_exact = false;
                c->exact_streak = 1;
            }
        }
        HIP_TRY(hipMemsetAsync(&c->d_res->n_cand, 0, sizeof(unsigned), s));
        k_argmax_cold<<<COLD_GRID, 256, 0, s>>>(c->cold, c->d_len16, max_length, c->d_res);
        k_collect<<<COLD_GRID, 256, 0, s>>>(table, c->cold, c->d_len16, max_length, c->d_res,
                                                 c->d_cand);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(c->h_res, c->d_res, sizeof(Result), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(c->h_cand, c->d_cand, MAX_CAND * sizeof(int2), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    }
    const unsigned n_cand = std::min<unsigned>(c->h_res->n_cand, CAND_CAP);
    cand.assign(c->h_cand, c->h_cand + std::min<unsigned>(n_cand, MAX_CAND));
    if (n_cand > (unsigned)MAX_CAND) {
        cand.resize(n_cand);
        HIP_TRY(hipMemcpy(cand.data(), c->d_cand, n_cand * sizeof(int2), hipMemcpyDeviceToHost));
    }
    return BPE_OK;
}

// R3 pass(es): last counted occurrence (slot + 1, 0 = none) of each candidate on this corpus.
// cand: the candidate list in device memory.
int tie_positions(bpe_ctx *c, const int2 *cand, unsigned n_cand, unsigned long long *last) {
    int rc;
    if (!c->carry_valid)
        if ((rc = run_pass(c, false, 0, 0, 0, nullptr))) return rc;
    hipStream_t s = c->stream;
    for (unsigned j0 = 0; j0 < n_cand; j0 += MAX_CAND) {
        const unsigned nb = std::min<unsigned>(MAX_CAND, n_cand - j0);
        TieArgs A;
        memset(&A, 0, sizeof A);
        A.ids = c->d_ids;
        A.n_chunks = c->n_chunks;
        A.cpr = c->cpr;
        A.R = c->R;
        A.n_cand = (int)nb;
        A.carry = c->d_carry;
        A.cand = cand + j0;
        A.res = c->d_res;
        A.ctl = nullptr;
        HIP_TRY(hipMemsetAsync(c->d_res, 0, sizeof(Result), s));
        c->best_ready = false;   // the Result is reused
        hipEvent_t e_tie = span_begin(c);
        if (c->n_live > 0) k_tie<<<(c->R + 3) / 4, 256, 0, s>>>(A);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(c->h_res, c->d_res, sizeof(Result), hipMemcpyDeviceToHost, s));
        if ((rc = span_end(c, e_tie, 2))) return rc;
        HIP_TRY(hipStreamSynchronize(s));
        if (c->stats_on) c->stats.tie_passes += 1;
        for (unsigned j = 0; j < nb; ++j) last[j0 + j] = c->h_res->last[j];
    }
    return BPE_OK;
}

int do_find(bpe_ctx *c, int64_t max_length, int64_t min_weight, int32_t *a, int32_t *b,
            int64_t *w) {
    if (min_weight == 0) min_weight = 2;                              // core.ts:256
    int rc;
    LEAVE_GLOBAL(c);
    // with a maintained cold table the selection settles a pending merge from the Result it
    // copies back anyway, so the host does not wait for the merge pass before enqueueing it
    const bool deferred = c->pending && c->cold_exact && c->counts_valid;
    if (!deferred) {
        if ((rc = settle(c))) return rc;
        if (c->n_live < 2) return BPE_NO_MERGE;
    }
    // (the maintained cold table does not read the sketch; every other selection does)
    if (!(c->cold_exact ? c->counts_valid : table_ok(c)))
        if ((rc = run_pass(c, false, 0, 0, 0, nullptr))) return rc;
    c->opt_max_length = max_length;
    hipEvent_t e_sel = span_begin(c);
    std::vector<int2> cand;
    rc = select_from_table(c, c->d_hot, max_length, true, cand, e_sel);
    if (rc == SELECT_RETRY) {
        if ((rc = run_pass(c, false, 0, 0, 0, nullptr))) return rc;
        rc = select_from_table(c, c->d_hot, max_length, true, cand, nullptr);
    }
    if (rc) return rc;
    if (c->stats_on) {
        c->stats.iterations += 1;
        c->stats.live_tokens += c->n_live;
    }
    const Result res = *c->h_res;
    if (res.best == 0) return BPE_NO_MERGE;                            // core.ts:312
    const int64_t W = (int64_t)(res.best >> 17);
    if (W < min_weight) return BPE_NO_MERGE;                           // core.ts:313
    const unsigned n_cand = (unsigned)cand.size();
    if (n_cand == 0 || res.n_cand > (unsigned)CAND_CAP)
        return fail(BPE_ERR_STATE, "bpe native: bad candidate count");
    int32_t ba = cand[0].x, bb = cand[0].y;
    if (n_cand > 1) {
        // R3: several pairs share W and a+b -> the one whose last counted occurrence is earliest
        // (the pair that reached W first in the reference's scan, core.ts:296-305)
        std::vector<unsigned long long> last(n_cand);
        if ((rc = tie_positions(c, c->d_cand, n_cand, last.data()))) return rc;
        unsigned long long best_pos = ~0ull;
        for (unsigned j = 0; j < n_cand; ++j) {
            if (last[j] && last[j] < best_pos) {
                best_pos = last[j];
                ba = cand[j].x;
                bb = cand[j].y;
            }
        }
        if (best_pos == ~0ull) return fail(BPE_ERR_STATE, "bpe native: tie pass found no occurrence");
    }
    *a = ba;
    *b = bb;
    *w = W;
    return BPE_OK;
}

int register_merge(bpe_ctx *c, int32_t a, int32_t b, int32_t cc);

int do_apply(bpe_ctx *c, int32_t a, int32_t b, int32_t cc, int64_t *replaced) {
    int rc;
    LEAVE_GLOBAL(c);
    if ((rc = register_merge(c, a, b, cc))) return rc;                 // core.ts:315-318
    if (replaced) *replaced = 0;
    if ((rc = settle(c))) return rc;
    if ((rc = maybe_compact(c))) return rc;
    if (c->n_live < 2) return BPE_OK;
    if (!c->carry_valid)
        if ((rc = run_pass(c, false, 0, 0, 0, nullptr))) return rc;
    // a maintained cold table is refreshed by the merge pass itself: the pairs with a side in
    // {a, b, cc} are the only ones whose count the merge changes (every other pair keeps its
    // occurrences and its run parity), so those lose their count before the pass and the pass
    // counts them again on the merged corpus.  A table that has to grow is rebuilt by a full
    // exact pass at the next selection instead.
    bool fused = false;
    if (c->cold_exact) {
        const int64_t na = c->h_count[a], nb = c->h_count[b];
        const uint64_t bound = (uint64_t)std::max<int64_t>(0, a == b ? na / 2 : std::min(na, nb));
        // the refresh claims at most 2 * bound new slots (holes included): it must fit the
        // table's 3/4 fill limit, which counts every claim made since the last rebuild
        const uint64_t V = c->h_len16.size() + 1;
        const uint64_t claims = std::min<uint64_t>(2 * bound, V * V) + 64;
        if (cold_rebuild_on() &&
            (cold_cap_for(c, bound) > c->cold_cap || c->cold_used + claims > c->cold_cap / 4 * 3)) {
            // a table that has to grow, or has no room for the refresh: rebuilt from its own
            // live claims, with room for both
            if ((rc = cold_rebuild(c, std::max(cold_cap_for(c, bound), 2 * claims)))) return rc;
        }
        const uint64_t cap1 = c->cold_cap;
        if ((rc = ensure_cold(c, bound))) return rc;
        const bool room = c->cold_used + claims <= c->cold_cap / 4 * 3 && c->cold_cap == cap1;
        fused = c->cold_exact && room && !getenv("BPE_DEBUG_NO_FUSED");
        if (!fused) {
            c->cold_exact = false;
            c->exact_streak = 1;   // (the next exact pass rebuilds the whole table)
        }
    }
    if (fused && !c->use_incr) k_cold_invalidate<<<COLD_GRID, 256, 0, c->stream>>>(c->cold, a, b);
    if ((rc = run_pass(c, true, a, b, cc, replaced, fused))) return rc;
    return BPE_OK;
}

// Up to n mergeUntil iterations with the decisions kept on the device (core.ts:367-384): per
// iteration k_select_multi, k_decide, [k_tie, k_decide] and the pass (k_step_loop, k_runs,
// k_reduce_table), every kernel reading the merge from the LoopCtl, and one host sync at the end.
// With a maintained cold table (skewed corpora) the selection is k_argmax_cold + k_collect over
// that table and the pass is the fused one (k_cold_invalidate, k_step_loop<MODE_FUSED>,
// k_runs<MODE_FUSED>), as in the host path.
// The merges go to out_abw[3 * i ...]; *status is the LoopStatus the batch ended with (LOOP_RUN:
// all n done; LOOP_HOST: the next iteration needs the host path).  The host tables are brought up
// to date from the log.
int loop_batch(bpe_ctx *c, int64_t max_length, int64_t min_weight, int64_t n, int64_t *out_abw,
               int64_t *n_done, int *status) {
    int rc;
    *n_done = 0;
    *status = LOOP_DONE;
    LEAVE_GLOBAL(c);
    if ((rc = settle(c))) return rc;
    c->cold_list = false;
    c->opt_max_length = max_length;
    const bool maint = c->cold_exact && c->counts_valid && c->carry_valid &&
                       !getenv("BPE_DEBUG_NO_FUSED");
    // (A/B and checking knob: every maintained selection a full scan of the cold table)
    static const bool sel_full = getenv("BPE_SEL_FULL") != nullptr;
    if (!maint) c->cold_exact = false;
    if (!maint && (!table_ok(c) || !c->carry_valid))
        if ((rc = run_pass(c, false, 0, 0, 0, nullptr))) return rc;
    const int64_t base = (int64_t)c->h_len16.size();
    if ((rc = ensure_len16_cap(c, base + n))) return rc;
    // the device table must be exact below `base`: k_decide extends it
    if (c->len16_lo < base) {
        HIP_TRY(hipMemcpyAsync(c->d_len16 + c->len16_lo, c->h_len16.data() + c->len16_lo,
                               (base - c->len16_lo) * sizeof(int32_t), hipMemcpyHostToDevice,
                               c->stream));
        c->len16_lo = base;
    }
    geometry(c);
    hipStream_t s = c->stream;
    if (maint) {
        // (k_select_maint takes the best over the hot bins itself)
        HIP_TRY(hipMemsetAsync(c->d_res, 0, sizeof(Result), s));
    } else if (c->best_ready && c->best_ml == max_length) {
        // keep the reduce's best key, clear the rest of the Result
        HIP_TRY(hipMemsetAsync(&c->d_res->n_cand, 0, sizeof(Result) - offsetof(Result, n_cand), s));
    } else {
        HIP_TRY(hipMemsetAsync(c->d_res, 0, sizeof(Result), s));
        k_argmax_hot<<<HOT_BINS / 256, 256, 0, s>>>(c->d_hot, c->d_len16, max_length, c->d_res);
    }
    LoopCtl *h = c->h_ctl;
    memset(h, 0, sizeof *h);
    h->status = LOOP_RUN;
    h->next_id = (int32_t)base;
    h->w = -1;
    h->min_weight = min_weight;
    h->max_id = BPE_MAX_VOCAB;
    h->maintained = maint ? 1 : 0;
    h->cold_cap = c->cold_cap;
    HIP_TRY(hipMemcpyAsync(c->d_ctl, h, sizeof *h, hipMemcpyHostToDevice, s));
    TieArgs A;
    memset(&A, 0, sizeof A);
    A.ids = c->d_ids;
    A.n_chunks = c->n_chunks;
    A.cpr = c->cpr;
    A.R = c->R;
    A.carry = c->d_carry;
    A.cand = c->d_cand;
    A.res = c->d_res;
    A.ctl = c->d_ctl;
    for (int64_t i = 0; i < n; ++i) {
        // the spans of every SPAN_EVERY-th iteration only: each event record costs the stream
        // a few microseconds, about 3% of an iteration with all six
        c->span_mute = (c->span_tick++ % SPAN_EVERY) != 0;
        hipEvent_t e_sel = span_begin(c);
        if (maint) {
            // best key over the hot bins and the cold table, its pairs, the table's flags
            // a full scan of the cold table on the first selection of the batch and every
            // SEL_FULL_EVERY-th (its dead claims), else the block maxima on a grid of one
            // workgroup per 256 hot bins
            const bool full = !c->use_incr || sel_full || i % SEL_FULL_EVERY == 0;
            k_select_maint<<<full ? COLD_GRID : HOT_BINS / 256, 256, 0, s>>>(
                c->d_hot, c->cold, c->d_len16, max_length, c->d_res, c->d_cand, c->d_brec,
                c->d_ticket, c->d_ctl, full ? 1 : 0);
        } else {
            k_select_multi<<<TABLE_BINS / 256, 256, 0, s>>>(c->d_hot, c->d_len16, max_length,
                                                            c->d_res, c->d_cand, c->d_heavy,
                                                            c->d_ctl);
        }
        // the decision, the R3 tie pass when tied, and its commit: one launch
        k_tie_fused<<<(c->R + 3) / 4, 256, 0, s>>>(A, c->d_len16, c->d_log, c->d_ticket);
        // (the maintained tables' entries touching the merge, zeroed for the pass to recount:
        // timed with the selection, so that the pass's span is the pass kernel alone)
        if (maint && c->use_incr)
            k_incr_invalidate<<<COLD_GRID, 256, 0, s>>>(c->cold, c->d_hot, -1, -1, c->d_ctl,
                                                        c->d_len16, max_length);
        else if (maint)
            k_cold_invalidate<<<COLD_GRID, 256, 0, s>>>(c->cold, -1, -1, c->d_ctl);
        HIP_TRY(hipGetLastError());
        if ((rc = span_end(c, e_sel, 1))) return rc;
        hipEvent_t e_step = span_begin(c);
        if (maint && c->use_incr) {
            k_step_loop<MODE_INCR><<<c->G, WG, 0, s>>>(c->d_ids, c->n_chunks, c->cpr, c->R,
                                                       c->d_carry, c->d_ctl, c->d_partials,
                                                       c->d_spill, c->cold, c->d_sums,
                                                       &c->d_res->replaced, c->d_hot);
        } else if (maint) {
            k_step_loop<MODE_FUSED><<<c->G, WG, 0, s>>>(c->d_ids, c->n_chunks, c->cpr, c->R,
                                                        c->d_carry, c->d_ctl, c->d_partials,
                                                        c->d_spill, c->cold, c->d_sums,
                                                        &c->d_res->replaced);
        } else {
            HIP_TRY(bpe_step::launch_step_loop_table(c->G, s, c->d_ids, c->n_chunks, c->cpr, c->R,
                                                     c->d_carry, c->d_ctl, c->d_partials,
                                                     c->d_spill, &c->cold, c->d_sums,
                                                     &c->d_res->replaced));
        }
        HIP_TRY(hipGetLastError());
        if ((rc = span_end(c, e_step, maint && c->use_incr ? 2 : 0))) return rc;
        hipEvent_t e_red = span_begin(c);
        if (maint && c->use_incr) {
            k_runs<MODE_INCR><<<(c->R + 255) / 256, 256, 0, s>>>(c->d_sums, c->R, c->d_carry,
                                                                 c->d_spill, c->cold, c->d_heavy,
                                                                 c->d_ctl, -1, -1, -1, c->d_hot);
            k_reduce_rows<<<4 * INCR_RLIM / 2 / RR_COLS, 256, 0, s>>>(
                c->d_partials, c->G, c->d_spill, c->d_hot, c->cold, -1, -1, -1, c->d_ctl);
        } else {
            if (maint)
                k_runs<MODE_FUSED><<<(c->R + 255) / 256, 256, 0, s>>>(c->d_sums, c->R, c->d_carry,
                                                                      c->d_spill, c->cold,
                                                                      c->d_heavy, c->d_ctl);
            else
                k_runs<MODE_TABLE><<<(c->R + 255) / 256, 256, 0, s>>>(c->d_sums, c->R, c->d_carry,
                                                                      c->d_spill, c->cold,
                                                                      c->d_heavy, c->d_ctl);
            k_reduce_table<<<HIST_WORDS / REDUCE_WORDS_PER_BLOCK, REDUCE_THREADS, 0, s>>>(
                c->d_partials, c->G, c->d_spill, c->d_hot, c->d_len16, max_length, c->d_res,
                c->d_ctl);
        }
        HIP_TRY(hipGetLastError());
        if ((rc = span_end(c, e_red, 1))) return rc;
    }
    c->span_mute = false;
    HIP_TRY(hipMemcpyAsync(h, c->d_ctl, sizeof *h, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(c->h_res, c->d_res, sizeof(Result), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(c->h_log, c->d_log, LOG_WORDS * n * sizeof(long long),
                           hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const int64_t nd = h->n_done;
    if (h->status == LOOP_ERROR)
        return fail(BPE_ERR_STATE, "bpe native: device loop: replacement count != W, or a tie "
                                   "pass found no occurrence");
    if (nd < 0 || nd > n) return fail(BPE_ERR_STATE, "bpe native: device loop: bad merge count");
    // the last merge's replacement count is checked here (the others were, on the device)
    if (h->status == LOOP_RUN && nd > 0 && c->h_res->replaced != (unsigned long long)h->w)
        return fail(BPE_ERR_STATE, "bpe native: replacement count != W");
    c->h_len16.resize(base + nd, 1);
    c->h_count.resize(base + nd, 0);
    for (int64_t i = 0; i < nd; ++i) {
        const int32_t a = (int32_t)c->h_log[LOG_WORDS * i], b = (int32_t)c->h_log[LOG_WORDS * i + 1];
        const int64_t W = c->h_log[LOG_WORDS * i + 2];
        const int64_t cc = base + i;
        c->h_len16[cc] = c->h_len16[a] + c->h_len16[b];                // core.ts:318
        if (c->stats_on) {
            c->stats.iterations += 1;
            c->stats.live_tokens += c->n_live;
        }
        c->n_live -= W;
        c->live_slots -= W;
        c->h_count[a] -= W;
        c->h_count[b] -= W;
        c->h_count[cc] += W;
        if (W) c->packed = false;
        if (c->stats_on) {
            c->stats.step_launches += 1;
            c->stats.step_slots += c->n_chunks * CHUNK;
            c->stats.step_live += c->n_live;
            if (maint && c->use_incr) {
                c->stats.incr_launches += 1;
                c->stats.incr_live += c->n_live;
            }
        }
        out_abw[3 * i] = a;
        out_abw[3 * i + 1] = b;
        out_abw[3 * i + 2] = W;
    }
    c->len16_lo = base + nd;   // k_decide wrote the new lengths on the device
    if (maint) {
        c->cold_used = c->h_res->cold_flags & 0xFFFFFFFFu;   // (as of the last selection)
        if (c->stats_on) {
            c->stats.cold_used = std::max<int64_t>(c->stats.cold_used, (int64_t)c->cold_used);
            uint32_t nr = 0;
            HIP_TRY(hipMemcpy(&nr, c->cold.n_recomputed, sizeof nr, hipMemcpyDeviceToHost));
            c->stats.sel_blocks = nr;   // (cumulative since the context was made)
        }
        if (nd) c->sketch_valid = false;                     // (fused passes)
        if (c->stats_on) c->stats.fused_passes += nd;
    }
    if (c->stats_on) {
        c->stats.tie_passes += h->n_tie;
        c->stats.unscreened_passes += h->n_unscreened;
        c->stats.tie_tail += h->n_tail;
        c->stats.tie_lone += h->n_lone;
        c->stats.loop_host += h->n_host;
    }
    c->last_replaced = nd ? c->h_log[LOG_WORDS * (nd - 1) + 2] : c->last_replaced;
    // every early-ended batch of the table state leaves the last reduce's best key in the Result
    // (the maintained state selects with k_select_maint: nothing is left ready)
    c->best_ready = !maint;
    c->best_ml = max_length;
    c->counts_valid = c->carry_valid = true;
    if (!maint) c->sketch_valid = true;
    *n_done = nd;
    *status = h->status;
    return BPE_OK;
}

// ---- the device loop on one rank of a sharded corpus ------------------------
// Per iteration the caller enqueues, on this context's stream: all-reduce(SUM) of the exchange
// buffer's first *n_words words, rank_loop_select, all-reduce(MAX) of the BPE_TIE_WORDS tie words,
// rank_loop_decide, rank_loop_count.  Nothing syncs the host until rank_loop_end, which reads the
// batch's merges back.  Two states, the same on every rank:
//  - table (the streaming pass's full recount): the exchange is the header + this shard's 81920-bin
//    table, summed into the global table every rank selects from;
//  - maintained (after bpe_set_global_counts: skewed corpora, large vocabularies): every rank
//    holds the global hot and cold tables; a merge (a, b) -> c zeroes the pairs touching a or b
//    in them, each shard recounts the pairs with a side in {a, b, c} on its own corpus (MODE_INCR)
//    into delta rows, and the summed rows are added to every rank's tables (k_apply_delta).
// The header's first word is this shard's replacement count of the merge just applied: summed,
// it must equal W (checked on the device by the next decision, and for the batch's last merge by
// the host from the log).
int carry_pass(bpe_ctx *c);
}  // namespace
int pix_rank_begin(bpe_ctx *c, int64_t max_length, int64_t min_weight, unsigned long long *xchg,
                   unsigned long long *tie, int rank, int world, int64_t *n_words);
int pix_rank_select(bpe_ctx *c);
int pix_rank_decide(bpe_ctx *c);
int pix_rank_count(bpe_ctx *c);
int pix_rank_end(bpe_ctx *c, int64_t *out, int64_t cap, int64_t *n_done, int *status);
int pix_set_global(bpe_ctx *c, const unsigned long long *table, const uint32_t *keys,
                   const unsigned long long *counts, int64_t n);
namespace {

int rank_loop_begin(bpe_ctx *c, int64_t max_length, int64_t min_weight, unsigned long long *xchg,
                    unsigned long long *tie, int rank, int world, int64_t *n_words) {
    int rc;
    if (c->rl_pix && c->rl_global) {
        if (!c->rl_delta_pending || xchg == c->rl_table)
            return pix_rank_begin(c, max_length, min_weight, xchg, tie, rank, world, n_words);
        LEAVE_GLOBAL(c);   // (another exchange buffer: the last merge's delta rows are not in it)
    }
    if ((rc = settle(c))) return rc;
    const bool glob = c->rl_global;
    c->opt_max_length = max_length;
    if (glob) {
        // the global tables stay: a compaction keeps every count, and the carries are rebuilt
        // without a counting pass (it would write this shard's counts over the global table)
        if (compaction_due(c)) {
            if (!c->carry_valid)
                if ((rc = carry_pass(c))) return rc;
            if ((rc = compact(c))) return rc;
        }
        if (!c->carry_valid)
            if ((rc = carry_pass(c))) return rc;
        if (c->rl_delta_pending && xchg != c->rl_table) {
            // (another exchange buffer: the last merge's delta rows are not in it)
            LEAVE_GLOBAL(c);
            return rank_loop_begin(c, max_length, min_weight, xchg, tie, rank, world, n_words);
        }
    } else {
        c->cold_exact = false;
        if ((rc = maybe_compact(c))) return rc;
        if (!table_ok(c) || !c->carry_valid)
            if ((rc = run_pass(c, false, 0, 0, 0, nullptr))) return rc;
    }
    if ((rc = ensure_partials(c))) return rc;
    const int64_t base = (int64_t)c->h_len16.size();
    if ((rc = ensure_len16_cap(c, base + LOOP_BATCH))) return rc;
    if (c->len16_lo < base) {
        HIP_TRY(hipMemcpyAsync(c->d_len16 + c->len16_lo, c->h_len16.data() + c->len16_lo,
                               (base - c->len16_lo) * sizeof(int32_t), hipMemcpyHostToDevice,
                               c->stream));
        c->len16_lo = base;
    }
    hipStream_t s = c->stream;
    HIP_TRY(hipMemsetAsync(c->d_res, 0, sizeof(Result), s));
    LoopCtl *h = c->h_ctl;
    memset(h, 0, sizeof *h);
    h->status = LOOP_RUN;
    h->next_id = (int32_t)base;
    h->w = -1;
    h->min_weight = min_weight == 0 ? 2 : min_weight;                   // core.ts:256
    h->sharded = 1;
    h->max_id = BPE_MAX_VOCAB;
    h->last_rank = rank == world - 1;
    h->maintained = glob ? 1 : 0;
    h->cold_cap = c->cold_cap;
    int64_t nw;
    if (glob) {
        // the delta rows of every token id a merge of this batch can see (<= base + LOOP_BATCH)
        nw = XCHG_HDR + DELTA_ROWS * std::min<int64_t>(BPE_MAX_VOCAB, base + LOOP_BATCH + 1);
        if (c->rl_delta_pending) {
            // the last batch's last merge: its rows go into this batch's first exchange
            h->a = c->rl_last_a;
            h->b = c->rl_last_b;
            h->c = c->rl_last_c;
            h->w = c->rl_last_w;
        } else {
            // all of it: the rows past this batch's words must be zero when later batches reach
            // them (k_apply_delta only zeroes the rows it consumes; the buffer may hold anything)
            HIP_TRY(hipMemsetAsync(xchg, 0, XCHG_WORDS * sizeof(unsigned long long), s));
        }
    } else {
        nw = XCHG_HDR + TABLE_BINS;
        HIP_TRY(hipMemsetAsync(xchg, 0, XCHG_HDR * sizeof(unsigned long long), s));
        HIP_TRY(hipMemcpyAsync(xchg + XCHG_HDR, c->d_hot, TABLE_BINS * sizeof(unsigned long long),
                               hipMemcpyDeviceToDevice, s));
    }
    HIP_TRY(hipMemcpyAsync(c->d_ctl, h, sizeof *h, hipMemcpyHostToDevice, s));
    c->rl_delta_pending = false;
    c->cold_list = false;
    c->rl_table = xchg;
    c->rl_tie = tie;
    c->rl_rank = rank;
    c->rl_world = world;
    c->rl_base = base;
    c->rl_enqueued = 0;
    c->rl_max_length = max_length;
    c->rl_open = true;
    c->best_ready = false;
    *n_words = nw;
    return BPE_OK;
}

// From the all-reduced exchange: the global table (or the maintained tables after the delta),
// the best key, its pairs, the proposal (or the tie pass, whose positions go to `tie` with this
// rank's vote for the all-reduce(MAX)).
int rank_loop_select(bpe_ctx *c) {
    if (!c->rl_open || c->rl_enqueued >= LOOP_BATCH)
        return fail(BPE_ERR_STATE, "bpe native: rank loop not begun, or its batch is full");
    if (c->rl_pix) return pix_rank_select(c);
    hipStream_t s = c->stream;
    const int64_t ml = c->rl_max_length;
    hipEvent_t e_sel = span_begin(c);
    if (c->rl_global) {
        k_apply_delta<<<COLD_GRID, 256, 0, s>>>(c->rl_table, c->d_hot, c->cold, c->d_ctl);
        // the block maxima of the cold table, as in the single-corpus device loop (round 5: was
        // k_argmax_hot + k_argmax_cold + k_collect, two scans of every claimed cold pair per merge,
        // which grew with the vocabulary).  The summed delta rows re-add the pairs of a and b that
        // k_incr_invalidate zeroed (to at most their old count: their blocks were flagged when the
        // zeroed entry may have been the max) and claim the pairs of c (new claims at the end of
        // the dense view), exactly the changes the incremental form recomputes.  A full scan on the
        // first selection of a batch and every SEL_FULL_EVERY-th (its dead claims).
        static const bool sel_full = getenv("BPE_SEL_FULL") != nullptr;
        const bool full = sel_full || c->rl_enqueued % SEL_FULL_EVERY == 0;
        k_select_maint<<<full ? COLD_GRID : HOT_BINS / 256, 256, 0, s>>>(
            c->d_hot, c->cold, c->d_len16, ml, c->d_res, c->d_cand, c->d_brec, c->d_ticket,
            c->d_ctl, full ? 1 : 0);
    } else {
        const unsigned long long *table = c->rl_table + XCHG_HDR;
        k_argmax_hot<<<HOT_BINS / 256, 256, 0, s>>>(table, c->d_len16, ml, c->d_res, c->d_ctl);
        k_select_multi<<<TABLE_BINS / 256, 256, 0, s>>>(table, c->d_len16, ml, c->d_res, c->d_cand,
                                                        c->d_heavy, c->d_ctl);
    }
    k_decide<<<1, 64, 0, s>>>(c->d_ctl, c->d_res, c->d_cand, c->d_len16, c->d_log, 0, nullptr,
                              c->rl_table);
    TieArgs A;
    memset(&A, 0, sizeof A);
    A.ids = c->d_ids;
    A.n_chunks = c->n_chunks;
    A.cpr = c->cpr;
    A.R = c->R;
    A.carry = c->d_carry;
    A.cand = c->d_cand;
    A.res = c->d_res;
    A.ctl = c->d_ctl;
    k_tie<<<(c->R + 3) / 4, 256, 0, s>>>(A);
    k_tie_export<<<1, 64, 0, s>>>(c->d_ctl, c->d_res, c->rl_tie, c->rl_rank);
    HIP_TRY(hipGetLastError());
    return span_end(c, e_sel, 1);
}

// After the all-reduce(MAX) of `tie`: the decision, the same on every rank.
int rank_loop_decide(bpe_ctx *c) {
    if (!c->rl_open) return fail(BPE_ERR_STATE, "bpe native: rank loop not begun");
    if (c->rl_pix) return pix_rank_decide(c);
    k_decide<<<1, 64, 0, c->stream>>>(c->d_ctl, c->d_res, c->d_cand, c->d_len16, c->d_log, 1,
                                      c->rl_tie, c->rl_table);
    HIP_TRY(hipGetLastError());
    return BPE_OK;
}

// Applies the decided merge to this shard and counts it: this shard's table (or delta rows) and
// its replacement count into the exchange buffer.
int rank_loop_count(bpe_ctx *c) {
    if (!c->rl_open) return fail(BPE_ERR_STATE, "bpe native: rank loop not begun");
    if (c->rl_pix) return pix_rank_count(c);
    hipStream_t s = c->stream;
    unsigned long long *x = c->rl_table;
    hipEvent_t e_step = span_begin(c);
    if (c->rl_global) {
        k_incr_invalidate<<<COLD_GRID, 256, 0, s>>>(c->cold, c->d_hot, -1, -1, c->d_ctl, c->d_len16,
                                                    c->rl_max_length);
        k_step_loop<MODE_INCR><<<c->G, WG, 0, s>>>(c->d_ids, c->n_chunks, c->cpr, c->R, c->d_carry,
                                                   c->d_ctl, c->d_partials, c->d_spill, c->cold,
                                                   c->d_sums, &c->d_res->replaced, c->d_hot, x);
    } else {
        HIP_TRY(bpe_step::launch_step_loop_table(c->G, s, c->d_ids, c->n_chunks, c->cpr, c->R,
                                                 c->d_carry, c->d_ctl, c->d_partials, c->d_spill,
                                                 &c->cold, c->d_sums, &c->d_res->replaced));
    }
    HIP_TRY(hipGetLastError());
    int rc;
    if ((rc = span_end(c, e_step, 0))) return rc;
    hipEvent_t e_red = span_begin(c);
    if (c->rl_global) {
        k_runs<MODE_INCR><<<(c->R + 255) / 256, 256, 0, s>>>(c->d_sums, c->R, c->d_carry, c->d_spill,
                                                             c->cold, c->d_heavy, c->d_ctl, -1, -1,
                                                             -1, c->d_hot, x);
        k_reduce_rows<<<4 * INCR_RLIM / 2 / RR_COLS, 256, 0, s>>>(
            c->d_partials, c->G, c->d_spill, c->d_hot, c->cold, -1, -1, -1, c->d_ctl, x,
            &c->d_res->replaced);
    } else {
        k_runs<MODE_TABLE><<<(c->R + 255) / 256, 256, 0, s>>>(c->d_sums, c->R, c->d_carry,
                                                              c->d_spill, c->cold, c->d_heavy,
                                                              c->d_ctl);
        k_reduce_table<<<HIST_WORDS / REDUCE_WORDS_PER_BLOCK, REDUCE_THREADS, 0, s>>>(
            c->d_partials, c->G, c->d_spill, x + XCHG_HDR, c->d_len16, c->rl_max_length, nullptr,
            c->d_ctl, x, &c->d_res->replaced, &c->d_res->bin_max);
    }
    HIP_TRY(hipGetLastError());
    c->rl_enqueued += 1;
    return span_end(c, e_red, 1);
}

// Syncs, reads the batch's merges back (out_abwr: (a, b, W, this shard's replacement count)
// quadruples) and updates the host tables with this shard's counts.  *status: LOOP_RUN (every
// enqueued iteration merged), LOOP_DONE (no pair qualifies), LOOP_HOST (the next iteration needs
// the host protocol).
int rank_loop_end(bpe_ctx *c, int64_t *out, int64_t cap, int64_t *n_done, int *status) {
    if (!c->rl_open) return fail(BPE_ERR_STATE, "bpe native: rank loop not begun");
    if (c->rl_pix) return pix_rank_end(c, out, cap, n_done, status);
    c->rl_open = false;
    hipStream_t s = c->stream;
    LoopCtl *h = c->h_ctl;
    HIP_TRY(hipMemcpyAsync(h, c->d_ctl, sizeof *h, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(c->h_res, c->d_res, sizeof(Result), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(c->h_log, c->d_log, LOG_WORDS * LOOP_BATCH * sizeof(long long),
                           hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const bool glob = c->rl_global;
    if (h->status == LOOP_ERROR) {
        const bool was_global = glob;
        static const bool dbg = getenv("BPE_DEBUG_GLOBAL") != nullptr;
        if (dbg) {
            HIP_TRY(hipMemcpy(c->h_log, c->d_log, LOG_WORDS * LOOP_BATCH * sizeof(long long),
                              hipMemcpyDeviceToHost));
            for (int64_t i = 0; i < h->n_done && i < LOOP_BATCH; ++i)
                fprintf(stderr, "[bpe debug] rank %d batch merge %lld: (%lld, %lld) W %lld rep %lld\n",
                        c->rl_rank, (long long)i, c->h_log[4 * i], c->h_log[4 * i + 1],
                        c->h_log[4 * i + 2], c->h_log[4 * i + 3]);
            fprintf(stderr, "[bpe debug] rank %d ctl: a %d b %d c %d w %lld tie %d vote %d base %lld\n",
                    c->rl_rank, h->a, h->b, h->c, (long long)h->w, h->tie, h->vote, (long long)c->rl_base);
        }
        LEAVE_GLOBAL(c);
        c->counts_valid = false;
        char msg[256];
        if (h->err == 1)
            snprintf(msg, sizeof msg, "bpe native: rank loop: the shards' replacement counts sum to "
                     "%llu, not W = %llu (merge %lld of the batch, %s state)", h->err_got, h->err_want,
                     (long long)h->n_done, was_global ? "maintained" : "table");
        else
            snprintf(msg, sizeof msg, "bpe native: rank loop: a tie pass found no occurrence (merge "
                     "%lld of the batch, %s state)", (long long)h->n_done, was_global ? "maintained" : "table");
        return fail(BPE_ERR_STATE, msg);
    }
    const int64_t nd = h->n_done;
    if (nd < 0 || nd > c->rl_enqueued) return fail(BPE_ERR_STATE, "bpe native: rank loop: bad merge count");
    const int64_t base = c->rl_base;
    c->h_len16.resize(base + nd, 1);
    c->h_count.resize(base + nd, 0);
    for (int64_t i = 0; i < nd; ++i) {
        const long long *m = c->h_log + LOG_WORDS * i;
        const int32_t a = (int32_t)m[0], b = (int32_t)m[1];
        const int64_t W = m[2];
        // this shard's replacement count (the last merge's is still in the Result)
        const int64_t R = m[3] >= 0 ? m[3] : (int64_t)c->h_res->replaced;
        const int64_t cc = base + i;
        c->h_len16[cc] = c->h_len16[a] + c->h_len16[b];                // core.ts:318
        if (c->stats_on) {
            c->stats.iterations += 1;
            c->stats.live_tokens += c->n_live;
        }
        c->n_live -= R;
        c->live_slots -= R;
        c->h_count[a] -= R;
        c->h_count[b] -= R;
        c->h_count[cc] += R;
        if (R) c->packed = false;
        if (c->stats_on) {
            c->stats.step_launches += 1;
            c->stats.step_slots += c->n_chunks * CHUNK;
            c->stats.step_live += c->n_live;
            if (glob) c->stats.fused_passes += 1;
        }
        if (i < cap) {
            out[4 * i] = a;
            out[4 * i + 1] = b;
            out[4 * i + 2] = W;
            out[4 * i + 3] = R;
        }
    }
    c->len16_lo = base + nd;
    if (c->stats_on) {
        c->stats.tie_passes += h->n_tie;
        c->stats.unscreened_passes += h->n_unscreened;
        c->stats.tie_tail += h->n_tail;
        c->stats.tie_lone += h->n_lone;
        c->stats.loop_host += h->n_host;
    }
    c->carry_valid = true;   // (the last pass's carries)
    c->best_ready = false;
    const bool all = h->status == LOOP_RUN && nd == c->rl_enqueued;
    if (glob) {
        if (all && nd > 0) {
            // the last merge's delta rows wait in the exchange buffer for the next batch's first
            // all-reduce
            const long long *m = c->h_log + LOG_WORDS * (nd - 1);
            c->rl_delta_pending = true;
            c->rl_last_a = (int32_t)m[0];
            c->rl_last_b = (int32_t)m[1];
            c->rl_last_c = (int32_t)(base + nd - 1);
            c->rl_last_w = m[2];
        } else if (!all) {
            LEAVE_GLOBAL(c);   // (the host path takes over: this shard's counts are recounted)
        }
    } else if (all && nd > 0) {
        // the last count left this shard's table in the exchange buffer, not summed since
        HIP_TRY(hipMemcpyAsync(c->d_hot, c->rl_table + XCHG_HDR, TABLE_BINS * sizeof(unsigned long long),
                               hipMemcpyDeviceToDevice, s));
        c->counts_valid = c->sketch_valid = true;
    } else if (nd > 0 || !all) {
        // (the exchange buffer was summed again after the batch ended: recount when needed)
        c->counts_valid = false;
    }
    *n_done = nd;
    *status = h->status;
    return BPE_OK;
}

// This shard's exact count of every cold pair (an id >= 256), for the global tables of the
// sharded maintained state: one exact streaming pass (kept: a second call with a bigger buffer
// exports the same list without another pass).
int cold_counts(bpe_ctx *c, uint32_t *keys, unsigned long long *counts, int64_t cap, int64_t *n) {
    int rc;
    LEAVE_GLOBAL(c);
    if ((rc = settle(c))) return rc;
    if (!c->cold_list) {
        hipStream_t s = c->stream;
        if (c->n_live >= 2) {
            HIP_TRY(hipMemsetAsync(c->d_heavy, 0xFF, HEAVY_WORDS * sizeof(uint32_t), s));
            if ((rc = exact_pass(c))) return rc;
        } else {
            if ((rc = cold_clear(c))) return rc;
            c->cold_used = 0;
        }
        c->cold_list = true;
    }
    *n = (int64_t)c->cold_used;
    if (*n > cap) return BPE_OK;
    if (*n) {
        if (!keys || !counts) return fail(BPE_ERR_ARG, "bpe native: null cold buffers");
        k_export_cold<<<256, 256, 0, c->stream>>>(c->cold, keys, counts);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    return BPE_OK;
}

// Loads the global maintained state of a sharded corpus: the hot bins of the global table and
// the cold pairs of every shard (duplicates summed).  The next rank loop batch keeps them.
int set_global_counts(bpe_ctx *c, const unsigned long long *table, const uint32_t *keys,
                      const unsigned long long *counts, int64_t n) {
    int rc;
    LEAVE_GLOBAL(c);
    if ((rc = settle(c))) return rc;
    if (n < 0 || (n && (!keys || !counts))) return fail(BPE_ERR_ARG, "bpe native: bad global counts");
    if (c->use_pix) return pix_set_global(c, table, keys, counts, n);   // (the incremental mode)
    hipStream_t s = c->stream;
    // room for every distinct pair at half fill, and for the claims of the merges to come (the
    // decisions hand over to the host before 3/4 fill)
    if ((rc = ensure_cold(c, 0, 4 * (uint64_t)n + 4096))) return rc;
    for (int attempt = 0;; ++attempt) {
        if ((rc = cold_clear(c))) return rc;
        HIP_TRY(hipMemcpyAsync(c->d_hot, table, HOT_BINS * sizeof(unsigned long long),
                               hipMemcpyDeviceToDevice, s));
        if (n) k_load_cold<<<1024, 256, 0, s>>>(c->cold, keys, counts, n);
        HIP_TRY(hipGetLastError());
        uint32_t flags[2] = {0, 0};
        HIP_TRY(hipMemcpyAsync(flags, c->d_cold_flags, sizeof flags, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (!flags[1] && (uint64_t)flags[0] * 4 <= c->cold_cap) {
            c->cold_used = flags[0];
            break;
        }
        if (attempt == 2) return fail(BPE_ERR_STATE, "bpe native: global cold table overflow");
        if ((rc = ensure_cold(c, 0, 2 * c->cold_cap))) return rc;
    }
    c->rl_global = true;
    c->rl_delta_pending = false;
    c->counts_valid = true;
    c->sketch_valid = false;
    c->cold_exact = false;   // (the single-context maintained state is not this one)
    c->best_ready = false;
    return BPE_OK;
}

// Carries (RegionCarry) for the current corpus and geometry without counting pairs.
int carry_pass(bpe_ctx *c) {
    geometry(c);
    hipStream_t s = c->stream;
    k_apply<NO_MERGE><<<c->G, WG, 0, s>>>(c->d_ids, c->n_chunks, c->cpr, c->R, c->d_carry, -1, -1,
                                          -1, c->d_sums, nullptr);
    k_runs<MODE_NONE><<<(c->R + 255) / 256, 256, 0, s>>>(c->d_sums, c->R, c->d_carry, nullptr,
                                                         c->cold, nullptr, nullptr);
    HIP_TRY(hipGetLastError());
    c->carry_valid = true;
    return BPE_OK;
}

// Checks a merge (a, b) -> cc against the vocabulary and registers cc (core.ts:315-318).
int register_merge(bpe_ctx *c, int32_t a, int32_t b, int32_t cc) {
    if (a < 0 || b < 0 || cc < 0 || cc >= BPE_MAX_VOCAB)
        return fail(cc >= BPE_MAX_VOCAB ? BPE_ERR_VOCAB : BPE_ERR_ARG,
                    "bpe native: token id out of range (vocab is limited to 55295 tokens)");
    if (a >= (int64_t)c->h_len16.size() || b >= (int64_t)c->h_len16.size())
        return fail(BPE_ERR_ARG, "bpe native: apply_merge with an unregistered token");
    int rc;
    if ((rc = ensure_vocab(c, (int64_t)cc + 1))) return rc;
    c->h_len16[cc] = c->h_len16[a] + c->h_len16[b];
    mark_len16(c, cc);
    return BPE_OK;
}

// applyMerge without counting, for a run of merges (restoreMerge replay, core.ts:477-494; batch
// encoding, core.ts:392-409): one apply-only streaming pass per merge (k_apply + k_runs for the
// carries), their replacement counts read back once per REPLAY_BATCH merges.  With count_after
// the last merge is applied by the fused apply + count pass, so a find that follows needs no
// extra pass.  replaced (may be null) receives each merge's replacement count.
int replay(bpe_ctx *c, const int32_t *abc, int64_t n, int64_t *replaced, bool count_after) {
    int rc;
    LEAVE_GLOBAL(c);
    if ((rc = settle(c))) return rc;
    const int64_t n_plain = count_after ? n - 1 : n;
    for (int64_t i0 = 0; i0 < n_plain;) {
        if ((rc = maybe_compact(c))) return rc;
        if (!c->carry_valid)
            if ((rc = carry_pass(c))) return rc;
        const int64_t nb = std::min<int64_t>(REPLAY_BATCH, n_plain - i0);
        for (int64_t j = 0; j < nb; ++j) {
            const int32_t *m = abc + 3 * (i0 + j);
            if ((rc = register_merge(c, m[0], m[1], m[2]))) return rc;
        }
        geometry(c);
        hipStream_t s = c->stream;
        HIP_TRY(hipMemsetAsync(c->d_repl, 0, nb * sizeof(unsigned long long), s));
        for (int64_t j = 0; j < nb; ++j) {
            const int32_t *m = abc + 3 * (i0 + j);
            if (m[0] == m[1])
                k_apply<MERGE_XX><<<c->G, WG, 0, s>>>(c->d_ids, c->n_chunks, c->cpr, c->R,
                                                      c->d_carry, m[0], m[1], m[2], c->d_sums,
                                                      c->d_repl + j);
            else
                k_apply<MERGE_XY><<<c->G, WG, 0, s>>>(c->d_ids, c->n_chunks, c->cpr, c->R,
                                                      c->d_carry, m[0], m[1], m[2], c->d_sums,
                                                      c->d_repl + j);
            k_runs<MODE_NONE><<<(c->R + 255) / 256, 256, 0, s>>>(c->d_sums, c->R, c->d_carry,
                                                                 nullptr, c->cold, nullptr, nullptr);
        }
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(c->h_repl, c->d_repl, nb * sizeof(unsigned long long),
                               hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        for (int64_t j = 0; j < nb; ++j) {
            const int32_t *m = abc + 3 * (i0 + j);
            const int64_t R = (int64_t)c->h_repl[j];
            c->n_live -= R;
            c->live_slots -= R;
            c->h_count[m[0]] -= R;
            c->h_count[m[1]] -= R;
            c->h_count[m[2]] += R;
            if (R) c->packed = false;
            if (replaced) replaced[i0 + j] = R;
        }
        c->counts_valid = false;
        c->cold_exact = false;
        c->best_ready = false;
        i0 += nb;
    }
    if (count_after && n > 0) {
        const int32_t *m = abc + 3 * (n - 1);
        int64_t R = 0;
        if ((rc = do_apply(c, m[0], m[1], m[2], &R))) return rc;
        if (replaced) replaced[n - 1] = R;
    }
    return BPE_OK;
}

int append_begin(bpe_ctx *c, int64_t extra_slots) {
    int rc;
    if ((rc = settle(c))) return rc;
    if (!c->packed)
        if ((rc = compact(c))) return rc;
    return ensure_chunks(c, (c->live_slots + extra_slots + CHUNK - 1) / CHUNK);
}

}  // namespace

int bpe_fail(int code, const char *msg) { return fail(code, msg); }

// a multi-device context forwards the call; per-shard entry points refuse it
// Device scratch freed on scope exit (the sample index is a rare, host-facing operation).
struct Scratch {
    std::vector<void *> p;
    template <typename T>
    int get(T **out, size_t n) {
        int rc = dev_alloc(out, n);
        if (!rc) p.push_back(*out);
        return rc;
    }
    ~Scratch() {
        for (void *q : p) dfree(q);
    }
};

// Where every sample ends: slot_end[i] = the slot of sample i's terminator, live_end[i] = the
// live tokens of samples 0..i.  Two reads of the corpus (k_census, k_sep_emit), one host sync.
int sample_ends(bpe_ctx *c, std::vector<int64_t> &slot_end, std::vector<int64_t> &live_end) {
    int rc;
    if ((rc = settle(c))) return rc;
    const int64_t ns = c->n_samples;
    slot_end.assign(ns, 0);
    live_end.assign(ns, 0);
    if (!ns) return BPE_OK;
    geometry(c);
    Scratch t;
    int64_t *d_live, *d_seps, *d_slot, *d_lend;
    if ((rc = t.get(&d_live, c->R)) || (rc = t.get(&d_seps, c->R)) || (rc = t.get(&d_slot, ns)) ||
        (rc = t.get(&d_lend, ns)))
        return rc;
    hipStream_t s = c->stream;
    const int blocks = (c->R + 3) / 4;
    k_census<<<blocks, 256, 0, s>>>(c->d_ids, c->n_chunks, c->cpr, c->R, d_live, d_seps);
    k_scan_pair<<<1, 1024, 0, s>>>(c->R, d_live, d_seps);
    k_sep_emit<<<blocks, 256, 0, s>>>(c->d_ids, c->n_chunks, c->cpr, c->R, d_live, d_seps, ns,
                                      d_slot, d_lend);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(slot_end.data(), d_slot, ns * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(live_end.data(), d_lend, ns * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (live_end[ns - 1] != c->n_live)
        return fail(BPE_ERR_STATE, "bpe native: corpus layout mismatch (sample index)");
    return BPE_OK;
}

int sample_lengths(bpe_ctx *c, int64_t *lens, int64_t cap) {
    if (cap < c->n_samples || (c->n_samples && !lens))
        return fail(BPE_ERR_ARG, "bpe native: sample_lengths buffer too small");
    std::vector<int64_t> se, le;
    int rc = sample_ends(c, se, le);
    if (rc) return rc;
    for (int64_t i = 0; i < c->n_samples; ++i) lens[i] = le[i] - (i ? le[i - 1] : 0);
    return BPE_OK;
}

// Live ids of samples idx[0..n), packed in that order: one gather of their slot ranges on the
// device, one copy back, the dead slots dropped on the host.
int read_samples(bpe_ctx *c, const int64_t *idx, int64_t n, int32_t *ids_out, int64_t ids_cap,
                 int64_t *off) {
    if (n < 0 || (n && !idx) || !off) return fail(BPE_ERR_ARG, "bpe native: bad read_samples arguments");
    off[0] = 0;
    if (!n) return BPE_OK;
    std::vector<int64_t> se, le;
    int rc = sample_ends(c, se, le);
    if (rc) return rc;
    std::vector<int64_t> src(n), len(n), dst(n + 1);
    int64_t need = 0;
    dst[0] = 0;
    for (int64_t k = 0; k < n; ++k) {
        const int64_t i = idx[k];
        if (i < 0 || i >= c->n_samples) return fail(BPE_ERR_ARG, "bpe native: sample index out of range");
        src[k] = i ? se[i - 1] + 1 : 0;
        len[k] = se[i] - src[k];
        dst[k + 1] = dst[k] + len[k];
        need += le[i] - (i ? le[i - 1] : 0);
    }
    if (ids_cap < need || (need && !ids_out))
        return fail(BPE_ERR_ARG, "bpe native: read_samples buffer too small");
    const int64_t total = dst[n];
    std::vector<int32_t> buf(total);
    if (total) {
        Scratch t;
        int64_t *d_src, *d_len, *d_dst;
        int32_t *d_out;
        if ((rc = t.get(&d_src, n)) || (rc = t.get(&d_len, n)) || (rc = t.get(&d_dst, n)) ||
            (rc = t.get(&d_out, total)))
            return rc;
        hipStream_t s = c->stream;
        HIP_TRY(hipMemcpyAsync(d_src, src.data(), n * sizeof(int64_t), hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(d_len, len.data(), n * sizeof(int64_t), hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(d_dst, dst.data(), n * sizeof(int64_t), hipMemcpyHostToDevice, s));
        k_gather_ranges<<<(unsigned)std::min<int64_t>(n, 1 << 16), 256, 0, s>>>(c->d_ids, d_src, d_len,
                                                                                d_dst, n, d_out);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(buf.data(), d_out, total * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    int64_t o = 0;
    for (int64_t k = 0; k < n; ++k) {
        for (int64_t j = dst[k]; j < dst[k + 1]; ++j)
            if (buf[j] >= 0) ids_out[o++] = buf[j];
        off[k + 1] = o;
    }
    if (o != need) return fail(BPE_ERR_STATE, "bpe native: corpus layout mismatch (read_samples)");
    return BPE_OK;
}

// ================================================================================================
// The incremental mergeUntil on the position index (bpe_pix.hip.h)
// ================================================================================================
struct PixState {
    PixCorpus C{};
    PixTable T{};
    PixBufs B{};
    PixCtl *d_ctl = nullptr, *h_ctl = nullptr;
    long long *d_log = nullptr, *h_log = nullptr;
    uint64_t cap = 0;
    int64_t max_length = 0;
    std::vector<void *> owned;
};
constexpr int64_t PIX_BATCH = 256;      // merges per host round trip
constexpr int PIX_NOT_ELIGIBLE = 100;   // (internal) the corpus does not fit the index

void pix_free(bpe_ctx *c) {
    PixState *P = c->pix;
    if (!P) return;
    for (void *q : P->owned) dfree(q);
    if (P->h_ctl) (void)hipHostFree(P->h_ctl);
    if (P->h_log) (void)hipHostFree(P->h_log);
    delete P;
    c->pix = nullptr;
}

template <typename T>
int pix_alloc(PixState *P, T **out, size_t n) {
    int rc = dev_alloc(out, n);
    if (!rc) P->owned.push_back(*out);
    return rc;
}

// The index of the current corpus: the slot array is the compacted corpus itself (d_ids, n live
// slots), links i -> i +- 1, and every pair's list from a counting scatter into the pair table
// (bpe_pix.hip.h, index build): run starts per block and their carries, then per position its
// pair's slot, list length and count, a pool segment per pair, and the positions into the
// segments.  A table that fills past a quarter is built again four times larger.
int pix_build_timed(bpe_ctx *c, int64_t max_length);

int pix_build(bpe_ctx *c, int64_t max_length) {
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = pix_build_timed(c, max_length);
    if (c->stats_on && rc == BPE_OK)
        c->stats.pix_build_ms +=
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

int pix_build_timed(bpe_ctx *c, int64_t max_length) {
    int rc;
    if ((rc = settle(c))) return rc;
    if (!c->packed)
        if ((rc = compact(c))) return rc;
    const int64_t n = c->live_slots;
    // positions and pool offsets are 32-bit (PIX_NONE = 2^32 - 1 is no position; the margin keeps
    // a block's end, block * PB + PB, below 2^32); the vocabulary key is two 16-bit ids
    // (a shard of a sharded corpus may hold fewer than two slots: its index is just empty)
    if (n > (int64_t)PIX_MAX_SLOTS || c->h_len16.size() > 0xFFFF) return PIX_NOT_ELIGIBLE;
    if ((rc = ensure_vocab(c, (int64_t)c->h_len16.size()))) return rc;
    if ((rc = sync_len16(c, 1))) return rc;
    pix_free(c);
    PixState *P = c->pix = new PixState();
    P->max_length = max_length;
    hipStream_t s = c->stream;
    const uint32_t N = (uint32_t)n;
    PixCorpus &C = P->C;
    C.tok = c->d_ids;
    C.n = N;
    if ((rc = pix_alloc(P, &C.nxt, N)) || (rc = pix_alloc(P, &C.prv, N))) return rc;
    const uint64_t pool_cap = std::min<uint64_t>(0xFFFFFFF0ull, (uint64_t)N + std::max<uint64_t>(N / 2, 1u << 22));
    PixBufs &B = P->B;
    if ((rc = pix_alloc(P, &B.pool, pool_cap))) return rc;
    const uint32_t nblk = (N + PB - 1) / PB;
    uint32_t *carry;
    if ((rc = pix_alloc(P, &carry, nblk))) return rc;
    k_pix_build_links<<<4096, 256, 0, s>>>(C, carry);
    k_pix_scan_max<<<1, 1024, 0, s>>>(carry, nblk);
    HIP_TRY(hipGetLastError());
    if ((rc = pix_alloc(P, &P->d_ctl, 1)) || (rc = pix_alloc(P, &P->d_log, PIX_LOG * PIX_BATCH))) return rc;
    HIP_TRY(hipHostMalloc((void **)&P->h_ctl, sizeof(PixCtl), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void **)&P->h_log, PIX_LOG * PIX_BATCH * sizeof(long long), hipHostMallocDefault));
    // the hot passes' scratch: per workgroup and half a slab of 32768 counts (then offsets), the
    // hot pairs' totals, slots and uncounted (x, x) occurrences
    Scratch hs;
    const int G = (int)std::max<uint32_t>(1, std::min<uint32_t>(PH_WG_MAX, nblk));
    uint32_t *slab, *htot, *hslot, *hseg, *bucket, *xoff;
    unsigned long long *oddxx;
    if ((rc = hs.get(&slab, (size_t)2 * G * PH_HALF)) || (rc = hs.get(&htot, 65536)) ||
        (rc = hs.get(&hslot, 65536)) || (rc = hs.get(&oddxx, 256)) || (rc = hs.get(&hseg, 65536)) ||
        (rc = hs.get(&bucket, 257)) || (rc = hs.get(&xoff, (size_t)G * 256)))
        return rc;
    // the pair table: room for the current pairs and the ones merges will add (a shard of a
    // sharded corpus: also every pair of the other shards, pix_min_cap)
    uint64_t cap = 1u << 20;
    while (cap < (uint64_t)N / 8 || cap < c->pix_min_cap) cap <<= 1;
    PixTable &T = P->T;
    for (int attempt = 0;; ++attempt) {
        if (cap >= (1ull << 31)) return PIX_NOT_ELIGIBLE;   // (slot numbers keep PIX_OWNER free)
        P->cap = cap;
        T = PixTable{};
        T.mask = (uint32_t)(cap - 1);
        T.len16 = c->d_len16;
        T.ml = max_length;
        T.nblocks = (uint32_t)(cap / PIX_B);
        T.nsuper = (T.nblocks + PIX_SB - 1) / PIX_SB;
        if ((rc = pix_alloc(P, &T.keys, cap)) || (rc = pix_alloc(P, &T.cnt, cap)) ||
            (rc = pix_alloc(P, &T.off, cap)) || (rc = pix_alloc(P, &T.len, cap)) ||
            (rc = pix_alloc(P, &T.fill, cap)) || (rc = pix_alloc(P, &T.bmax, T.nblocks)) ||
            (rc = pix_alloc(P, &T.sbmax, T.nsuper)) || (rc = pix_alloc(P, &T.bdirty, T.nblocks)) ||
            (rc = pix_alloc(P, &T.sbdirty, T.nsuper)))
            return rc;
        HIP_TRY(hipMemsetAsync(T.keys, 0xFF, cap * sizeof(uint32_t), s));
        HIP_TRY(hipMemsetAsync(T.cnt, 0, cap * sizeof(unsigned long long), s));
        HIP_TRY(hipMemsetAsync(T.len, 0, cap * sizeof(uint32_t), s));
        HIP_TRY(hipMemsetAsync(T.bdirty, 0, T.nblocks * sizeof(uint32_t), s));
        HIP_TRY(hipMemsetAsync(T.sbdirty, 0, T.nsuper * sizeof(uint32_t), s));
        HIP_TRY(hipMemsetAsync(oddxx, 0, 256 * sizeof(unsigned long long), s));
        PixCtl *h = P->h_ctl;
        memset(h, 0, sizeof *h);
        h->status = PIX_RUN;
        h->max_length = max_length;
        h->max_id = BPE_MAX_VOCAB;
        h->next_id = (int32_t)c->h_len16.size();
        h->pool_cap = pool_cap;
        h->used_cap = cap / 10 * 7;
        HIP_TRY(hipMemcpyAsync(P->d_ctl, h, sizeof *h, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemsetAsync(slab, 0, (size_t)2 * G * PH_HALF * sizeof(uint32_t), s));
        k_pix_hot_count<<<G, PH_T, 0, s>>>(C, T, P->d_ctl, carry, slab, oddxx);
        k_pix_hot_xoff<<<256, 256, 0, s>>>(slab, G, xoff);
        k_pix_hot_scan<<<2 * PH_HALF / 256, 256, 0, s>>>(slab, G, htot);
        k_pix_hot_claim<<<65536 / 256, 256, 0, s>>>(T, P->d_ctl, htot, oddxx, hslot);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(h, P->d_ctl, sizeof *h, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (!h->err && h->used * 4 <= cap) break;
        // too full to probe well: a table four times larger
        for (void *q : {(void *)T.keys, (void *)T.cnt, (void *)T.off, (void *)T.len, (void *)T.fill,
                        (void *)T.bmax, (void *)T.sbmax, (void *)T.bdirty, (void *)T.sbdirty}) {
            P->owned.erase(std::find(P->owned.begin(), P->owned.end(), q));
            dfree(q);
        }
        cap <<= 2;
        if (attempt == 3) return PIX_NOT_ELIGIBLE;
    }
    // the hot pairs' segments in (x, y) order (buckets by first token), then the cold pairs'
    k_pix_hot_seg<<<1, 1024, 0, s>>>(T, P->d_ctl, htot, hslot, hseg, bucket);
    k_pix_build_alloc<<<4096, 256, 0, s>>>(T, P->d_ctl, (uint32_t)cap, 1);
    HIP_TRY(hipGetLastError());
    // The two-level fill when no first token holds more than 1/32 of the hot positions (a
    // workgroup per bucket does the second level); else the per-pair cursors (k_pix_hot_fill)
    uint32_t hb[257];
    HIP_TRY(hipMemcpyAsync(hb, bucket, sizeof hb, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    uint32_t bmax = 0;
    for (int x = 0; x < 256; ++x) bmax = std::max(bmax, hb[x + 1] - hb[x]);
    uint2 *stage = nullptr;
    const bool two_level = hb[256] > 0 && (uint64_t)bmax * 32 <= (uint64_t)hb[256] + (1u << 20) &&
                           !getenv("BPE_PIX_FILL_PAIRS") && hs.get(&stage, hb[256]) == BPE_OK;
    if (!two_level) (void)hipGetLastError();   // (a failed staging allocation is not an error)
    if (two_level) {
        k_pix_fill_x<<<G, PH_T, 0, s>>>(C, T, B, xoff, bucket, stage);
        k_pix_fill_y<<<256, 1024, 0, s>>>(B, hseg, bucket, stage);
    } else {
        for (int half = 0; half < 2; ++half)
            k_pix_hot_fill<<<G, PH_T, 0, s>>>(C, T, B, half, slab, hslot);
    }
    HIP_TRY(hipGetLastError());
    // per-merge buffers
    B.site_cap = (uint32_t)std::min<uint64_t>(N / 2 + 16, 1u << 26);
    B.ent_cap = 2 * B.site_cap + 16;
    if ((rc = pix_alloc(P, &B.sites, B.site_cap)) || (rc = pix_alloc(P, &B.ent, B.ent_cap)) ||
        (rc = pix_alloc(P, &B.dblocks, T.nblocks)) || (rc = pix_alloc(P, &B.dsuper, T.nsuper)))
        return rc;
    k_pix_bmax_all<<<4096, 256, 0, s>>>(T);
    k_pix_sbmax<<<1024, 256, 0, s>>>(T, B, P->d_ctl, 1);
    HIP_TRY(hipGetLastError());
    PixCtl *h = P->h_ctl;
    HIP_TRY(hipMemcpyAsync(h, P->d_ctl, sizeof *h, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (h->status != PIX_RUN) return fail(BPE_ERR_STATE, "bpe native: position index: pair table full");
    if (h->pool_top > (uint64_t)N) return fail(BPE_ERR_STATE, "bpe native: position index: bad pair lists");
    c->counts_valid = c->carry_valid = c->best_ready = false;
    c->cold_exact = false;
    if (c->stats_on) c->stats.pix_builds += 1;
    return BPE_OK;
}

// The corpus back into the chunk layout: the live slots of the slot array, in order, as a dense
// prefix (then the streaming path's state is rebuilt on its next use).
int pix_finish(bpe_ctx *c) {
    PixState *P = c->pix;
    if (!P) return BPE_OK;
    hipStream_t s = c->stream;
    const uint32_t N = P->C.n;
    {
        Scratch t;
        uint32_t *cnt, *d_total;
        const uint32_t nblk = (N + PB - 1) / PB;
        int rc;
        if ((rc = t.get(&cnt, nblk)) || (rc = t.get(&d_total, 1))) return rc;
        // (no fill first: the scatter writes the live prefix, seal_packed the rest that is read)
        k_pix_live_count<<<4096, 256, 0, s>>>(c->d_ids, N, cnt);
        k_pix_scan_sum<<<1, 1024, 0, s>>>(cnt, nblk, d_total);
        k_pix_live_scatter<<<4096, 256, 0, s>>>(c->d_ids, N, cnt, c->d_tmp);
        HIP_TRY(hipGetLastError());
        uint32_t nsel = 0;
        HIP_TRY(hipMemcpyAsync(&nsel, d_total, sizeof nsel, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if ((int64_t)nsel != c->live_slots)
            return fail(BPE_ERR_STATE, "bpe native: position index: live slots lost");
    }
    std::swap(c->d_ids, c->d_tmp);
    pix_free(c);
    return seal_packed(c);
}

int pix_reserve(bpe_ctx *c);

// mergeUntil on the index: batches of PIX_BATCH merges, one host round trip each.  An iteration
// the index cannot take (PIX_HOST) runs on the streaming path, and the index is rebuilt after it.
int pix_merge_until(bpe_ctx *c, int64_t max_length, int64_t min_weight, int64_t max_iterations,
                    int64_t *out_abw, int64_t cap, int64_t *n_merges) {
    int rc;
    int64_t n = 0;
    const int64_t mw = min_weight == 0 ? 2 : min_weight;                  // core.ts:256
    int builds = 0;
    bool just_built = false;
    LEAVE_GLOBAL(c);
    // Heavy merges first on the stream: a merge costs the index O(W) (plus contention on the
    // new pairs' slots when W is large), the stream one pass whatever W.  While the next merge's
    // W exceeds max(2^16, n_live / 8192) (C3: 131 K against W = 16 K, so never; a skewed corpus's
    // first merges replace millions), the streaming path takes it (findNextMerge + applyMerge),
    // and the index is built once the merges get light.  Zipf C3, incremental mode: 1.34 ms/merge
    // without the prefix; 0.585 / 0.363 / 0.309 / 0.432 with n_live / 512 / 2048 / 8192 / 32768
    // (tools/pix_wdiv.sh), against 0.394 for the stream alone.
    static const int64_t w_div = [] {
        const char *v = getenv("BPE_PIX_WDIV");   // (A/B knob)
        const long long d = v ? atoll(v) : 8192;
        return (int64_t)(d > 0 ? d : 8192);
    }();
    while (!c->pix && (!max_iterations || n < max_iterations)) {
        if ((rc = settle(c))) return rc;
        if (c->n_live < 2) break;
        int32_t a, b;
        int64_t w;
        rc = do_find(c, max_length, min_weight, &a, &b, &w);
        if (rc == BPE_NO_MERGE) {
            *n_merges = n;
            return settle(c);
        }
        if (rc) return rc;
        if (w <= (int64_t)1 << 16 || w * w_div <= c->n_live) break;   // light: the index from here
        const int32_t cc = (int32_t)c->h_len16.size();
        if ((rc = do_apply(c, a, b, cc, nullptr))) return rc;
        if (c->pending) c->pend_expect = w;
        if ((rc = settle(c))) return rc;
        if (n < cap) {
            out_abw[3 * n] = a;
            out_abw[3 * n + 1] = b;
            out_abw[3 * n + 2] = w;
        }
        ++n;
    }
    while (!max_iterations || n < max_iterations) {                      // core.ts:374-378
        if (!c->pix || c->pix->max_length != max_length) {
            if ((rc = pix_finish(c))) return rc;
            if ((rc = settle(c))) return rc;
            if (c->n_live < 2) break;
            rc = pix_build(c, max_length);
            ++builds;
            just_built = true;
            if (rc == BPE_ERR_OOM) {
                // (the index does not fit next to the corpus: the stream needs no extra memory)
                if (c->pix) {
                    (void)hipStreamSynchronize(c->stream);
                    pix_free(c);
                }
                rc = PIX_NOT_ELIGIBLE;
            }
            if (rc == PIX_NOT_ELIGIBLE) {
                pix_free(c);
                *n_merges = n;
                return PIX_NOT_ELIGIBLE;   // the caller goes on with the streaming loop
            }
            if (rc) return rc;
        }
        if (builds && !just_built)
            if ((rc = pix_reserve(c))) return rc;   // (grow the pool / table in place)
        just_built = false;
        PixState *P = c->pix;
        hipStream_t s = c->stream;
        const int64_t base = (int64_t)c->h_len16.size();
        int64_t want = std::min<int64_t>(PIX_BATCH, BPE_MAX_VOCAB - base);
        if (max_iterations) want = std::min<int64_t>(want, max_iterations - n);
        if ((rc = ensure_len16_cap(c, base + std::max<int64_t>(want, 1)))) return rc;
        if ((rc = sync_len16(c, 1))) return rc;
        int status = PIX_HOST;
        int64_t nd = 0;
        if (want > 0) {
            P->T.len16 = c->d_len16;   // (ensure_len16_cap may have moved it)
            k_pix_begin<<<1, 1, 0, s>>>(P->d_ctl, want, (int32_t)base, mw);
            for (int64_t i = 0; i < want; ++i) {
                k_pix_select<<<1, 1024, 0, s>>>(P->T, P->B, P->d_ctl);
                k_pix_sites<<<PIX_GRID, 256, 0, s>>>(P->C, P->T, P->B, P->d_ctl);
                k_pix_alloc<<<PIX_GRID, 256, 0, s>>>(P->T, P->B, P->d_ctl);
                k_pix_apply<<<PIX_GRID, 256, 0, s>>>(P->C, P->T, P->B, P->d_ctl, P->d_log);
            }
            HIP_TRY(hipGetLastError());
            PixCtl *h = P->h_ctl;
            HIP_TRY(hipMemcpyAsync(h, P->d_ctl, sizeof *h, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipMemcpyAsync(P->h_log, P->d_log, PIX_LOG * want * sizeof(long long),
                                   hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            status = h->status;
            nd = h->n_done;
            if (status == PIX_ERROR) {
                char msg[160];
                snprintf(msg, sizeof msg, "bpe native: position index inconsistent (code %d)", h->err);
                return fail(BPE_ERR_STATE, msg);
            }
            if (nd < 0 || nd > want) return fail(BPE_ERR_STATE, "bpe native: position index: bad merge count");
            c->h_len16.resize(base + nd, 1);
            c->h_count.resize(base + nd, 0);
            for (int64_t i = 0; i < nd; ++i, ++n) {
                const int32_t a = (int32_t)P->h_log[PIX_LOG * i], b = (int32_t)P->h_log[PIX_LOG * i + 1];
                const int64_t W = P->h_log[PIX_LOG * i + 2];
                const int64_t cc = base + i;
                c->h_len16[cc] = c->h_len16[a] + c->h_len16[b];            // core.ts:318
                if (c->stats_on) {
                    c->stats.iterations += 1;
                    c->stats.live_tokens += c->n_live;
                    c->stats.pix_merges += 1;
                }
                c->n_live -= W;
                c->live_slots -= W;
                c->h_count[a] -= W;
                c->h_count[b] -= W;
                c->h_count[cc] += W;
                if (n < cap) {
                    out_abw[3 * n] = a;
                    out_abw[3 * n + 1] = b;
                    out_abw[3 * n + 2] = W;
                }
            }
            c->len16_lo = base + nd;   // pix_commit wrote the new lengths on the device
            if (status == PIX_DONE) break;
            if (status == PIX_RUN || status == PIX_PAUSE) continue;
            if (c->stats_on) c->stats.pix_host += 1;
        }
        if (max_iterations && n >= max_iterations) break;
        // PIX_HOST: this iteration on the streaming path, then a fresh index
        if ((rc = pix_finish(c))) return rc;
        if (builds > 64 && builds > n / 16) {
            *n_merges = n;
            return PIX_NOT_ELIGIBLE;   // (the index keeps failing here: stay on the stream)
        }
        int32_t a, b;
        int64_t w;
        rc = do_find(c, max_length, min_weight, &a, &b, &w);
        if (rc == BPE_NO_MERGE) break;
        if (rc) return rc;
        const int32_t cc = (int32_t)c->h_len16.size();
        if ((rc = do_apply(c, a, b, cc, nullptr))) return rc;
        if (c->pending) c->pend_expect = w;
        if ((rc = settle(c))) return rc;
        if (n < cap) {
            out_abw[3 * n] = a;
            out_abw[3 * n + 1] = b;
            out_abw[3 * n + 2] = w;
        }
        ++n;
    }
    if ((rc = pix_finish(c))) return rc;
    *n_merges = n;
    return settle(c);
}

// ================================================================================================
// A shard of a sharded corpus in the incremental mode: the position index inside the rank loop
// (bpe_pix.hip.h, "a shard of a sharded corpus").  The index holds this shard's lists and every
// pair's GLOBAL count; each merge's count changes travel as delta rows.
// ================================================================================================

// bpe_set_global_counts in the incremental mode: this shard's index, then the global counts (the
// summed table's hot bins, every shard's cold pairs) in place of its own.
int pix_set_global(bpe_ctx *c, const unsigned long long *table, const uint32_t *keys,
                   const unsigned long long *counts, int64_t n) {
    int rc;
    // every pair of the corpus at most half the table (n counts a pair once per shard holding it;
    // pix_reserve grows the table in place as merges add pairs)
    c->pix_min_cap = 2 * (uint64_t)(HOT_BINS + n);
    // (BPE_PIX_FORCE_OOM=1, tests: the build fails as if out of device memory)
    rc = getenv("BPE_PIX_FORCE_OOM") ? BPE_ERR_OOM : pix_build(c, c->opt_max_length);
    c->pix_min_cap = 0;
    if (rc == PIX_NOT_ELIGIBLE || rc == BPE_ERR_OOM) {
        if (c->pix) {
            (void)hipStreamSynchronize(c->stream);
            pix_free(c);
        }
        return fail(BPE_ERR_NOFIT, "bpe native: the position index does not fit this shard "
                                   "(use the streaming mode)");
    }
    if (rc) return rc;
    PixState *P = c->pix;
    hipStream_t s = c->stream;
    HIP_TRY(hipMemsetAsync(P->T.cnt, 0, P->cap * sizeof(unsigned long long), s));
    k_pix_load_global<<<1024, 256, 0, s>>>(P->T, P->d_ctl, table, keys, counts, n);
    k_pix_bmax_all<<<4096, 256, 0, s>>>(P->T);
    k_pix_sbmax<<<1024, 256, 0, s>>>(P->T, P->B, P->d_ctl, 1);
    HIP_TRY(hipGetLastError());
    PixCtl *h = P->h_ctl;
    HIP_TRY(hipMemcpyAsync(h, P->d_ctl, sizeof *h, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (h->err || h->used * 2 > P->cap) {
        pix_free(c);
        return fail(BPE_ERR_STATE, "bpe native: position index: the global pairs overflow the table");
    }
    c->rl_global = true;
    c->rl_pix = true;
    c->rl_delta_pending = false;
    c->pix_w_last = 0;   // (the first batch's lanes: full words)
    c->counts_valid = c->sketch_valid = c->best_ready = false;
    c->cold_exact = false;
    return BPE_OK;
}

// Room for the next batch, grown in place (no hand-off, no rebuild): the pool when less than an
// eighth of the corpus is left of it (the new segments of a merge take two entries per site), the
// pair table (rehashed twice as large) past 45 % fill.  Between batches, with no tie pending (a
// decided tie names its pair by slot).  A shard of a sharded corpus grows its own index alone.
int pix_reserve(bpe_ctx *c) {
    PixState *P = c->pix;
    hipStream_t s = c->stream;
    PixCtl *h = P->h_ctl;
    HIP_TRY(hipMemcpyAsync(h, P->d_ctl, sizeof *h, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (h->status != PIX_RUN && h->status != PIX_PAUSE) return BPE_OK;
    const uint64_t N = P->C.n;
    const uint64_t slack = std::max<uint64_t>(N / 8, 1u << 20);
    if (h->pool_top + slack > h->pool_cap && h->pool_cap < 0xFFFFFFF0ull) {
        const uint64_t ncap = std::min<uint64_t>(0xFFFFFFF0ull, h->pool_cap + std::max<uint64_t>(N / 2, 4 * slack));
        uint32_t *np = nullptr;
        int rc = dev_alloc(&np, ncap);
        if (rc == BPE_OK) {
            HIP_TRY(hipMemcpyAsync(np, P->B.pool, h->pool_top * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
            HIP_TRY(hipStreamSynchronize(s));
            P->owned.erase(std::find(P->owned.begin(), P->owned.end(), (void *)P->B.pool));
            dfree(P->B.pool);
            P->B.pool = np;
            P->owned.push_back(np);
            h->pool_cap = ncap;
            HIP_TRY(hipMemcpyAsync(&P->d_ctl->pool_cap, &h->pool_cap, sizeof h->pool_cap,
                                   hipMemcpyHostToDevice, s));
        } else {
            (void)hipGetLastError();   // (no memory: the pool fills, and the batch hands over)
        }
    }
    if (h->used * 20 > P->cap * 9 && h->tie == PIX_TIE_NONE && P->cap * 2 < (1ull << 31)) {
        const uint64_t ncap = P->cap * 2;
        PixTable T = P->T;
        T.mask = (uint32_t)(ncap - 1);
        T.nblocks = (uint32_t)(ncap / PIX_B);
        T.nsuper = (T.nblocks + PIX_SB - 1) / PIX_SB;
        std::vector<void *> fresh;
        auto get = [&](auto **q, size_t n) {
            const int r = dev_alloc(q, n);
            if (r == BPE_OK) fresh.push_back(*q);
            return r;
        };
        uint32_t *dblocks = nullptr, *dsuper = nullptr;
        if (get(&T.keys, ncap) || get(&T.cnt, ncap) || get(&T.off, ncap) || get(&T.len, ncap) ||
            get(&T.fill, ncap) || get(&T.bmax, T.nblocks) || get(&T.sbmax, T.nsuper) ||
            get(&T.bdirty, T.nblocks) || get(&T.sbdirty, T.nsuper) || get(&dblocks, T.nblocks) ||
            get(&dsuper, T.nsuper)) {
            for (void *q : fresh) dfree(q);
            (void)hipGetLastError();
            return BPE_OK;   // (no memory: the table fills, and the batch hands over)
        }
        HIP_TRY(hipMemsetAsync(T.keys, 0xFF, ncap * sizeof(uint32_t), s));
        HIP_TRY(hipMemsetAsync(T.bdirty, 0, T.nblocks * sizeof(uint32_t), s));
        HIP_TRY(hipMemsetAsync(T.sbdirty, 0, T.nsuper * sizeof(uint32_t), s));
        k_pix_rehash<<<4096, 256, 0, s>>>(P->T, T, P->d_ctl, (uint32_t)P->cap);
        // (the old table's dirty lists name its blocks: every block max is recomputed instead)
        h->n_dblocks = h->n_dsuper = 0;
        h->used_cap = ncap / 10 * 7;
        HIP_TRY(hipMemcpyAsync(&P->d_ctl->n_dblocks, &h->n_dblocks, 2 * sizeof(uint32_t),
                               hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(&P->d_ctl->used_cap, &h->used_cap, sizeof h->used_cap,
                               hipMemcpyHostToDevice, s));
        PixBufs B = P->B;
        B.dblocks = dblocks;
        B.dsuper = dsuper;
        k_pix_bmax_all<<<4096, 256, 0, s>>>(T);
        k_pix_sbmax<<<1024, 256, 0, s>>>(T, B, P->d_ctl, 1);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(h, P->d_ctl, sizeof *h, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (h->err) return fail(BPE_ERR_STATE, "bpe native: position index: rehash overflow");
        for (void *q : {(void *)P->T.keys, (void *)P->T.cnt, (void *)P->T.off, (void *)P->T.len,
                        (void *)P->T.fill, (void *)P->T.bmax, (void *)P->T.sbmax, (void *)P->T.bdirty,
                        (void *)P->T.sbdirty, (void *)P->B.dblocks, (void *)P->B.dsuper}) {
            P->owned.erase(std::find(P->owned.begin(), P->owned.end(), q));
            dfree(q);
        }
        for (void *q : fresh) P->owned.push_back(q);
        P->T = T;
        P->B = B;
        P->cap = ncap;
    }
    return BPE_OK;
}

int pix_rank_begin(bpe_ctx *c, int64_t max_length, int64_t min_weight, unsigned long long *xchg,
                   unsigned long long *tie, int rank, int world, int64_t *n_words) {
    int rc;
    PixState *P = c->pix;
    hipStream_t s = c->stream;
    if ((rc = pix_reserve(c))) return rc;
    const int64_t base = (int64_t)c->h_len16.size();
    if ((rc = ensure_len16_cap(c, base + LOOP_BATCH))) return rc;
    if ((rc = sync_len16(c, 1))) return rc;
    P->T.len16 = c->d_len16;
    if (P->max_length != max_length) {
        // (the selection keys filter on max_length: every block max again)
        P->max_length = max_length;
        P->T.ml = max_length;
        c->pix_w_last = 0;   // (pairs the filter held back may now count more than the last W)
        k_pix_bmax_all<<<4096, 256, 0, s>>>(P->T);
        k_pix_sbmax<<<1024, 256, 0, s>>>(P->T, P->B, P->d_ctl, 1);
    }
    P->T.delta = xchg;
    // the exchange: the lane layout (a count per token id and side, in lanes as wide as the last
    // merge's count needs, bpe_pix.hip.h), or (BPE_XCHG_DENSE=1, A/B and checks) six dense rows per
    // token id
    const bool dense = getenv("BPE_XCHG_DENSE") != nullptr;   // (read per batch: tests switch it)
    const int64_t ids = std::min<int64_t>(BPE_MAX_VOCAB, base + LOOP_BATCH + 1);
    int64_t nw;
    // (the last batch's pending merge keeps its own layout for its decode, and its words)
    c->pix_first_pending = c->rl_delta_pending;
    for (int i = 0; i < 3; ++i) c->pix_lane_prev[i] = c->pix_lane[i];
    // (a pending merge's rows span the words of its own batch's layout, lanes or dense rows: this
    // batch all-reduces at least those, whatever layout it takes itself)
    const int64_t prev_words = c->rl_delta_pending ? c->pix_nw_last : 0;
    if (dense) {
        P->T.lane_w = P->T.lane_q = P->T.lane_base = 0;
        nw = std::max<int64_t>(XCHG_HDR + DELTA_ROWS * ids, prev_words);
    } else {
        uint32_t w = c->pix_w_last ? 64u - (uint32_t)__builtin_clzll(c->pix_w_last) : 64u;
        // (BPE_XCHG_LANE_BITS=n, tests: lanes of at most n bits after a known count, so that
        // counts outgrow them, pause the batch and the next one takes full words)
        if (const char *lb = getenv("BPE_XCHG_LANE_BITS"))
            if (c->pix_w_last) w = std::max(1u, std::min<uint32_t>(w, (uint32_t)atoi(lb)));
        const uint32_t q = 64u / w;
        P->T.lane_w = w;
        P->T.lane_q = q;
        P->T.lane_base = (uint32_t)((ids + q - 1) / q);
        nw = std::max<int64_t>(XCHG_HDR + PIX_XCHG_SPECIAL + 2 * (int64_t)P->T.lane_base, prev_words);
    }
    c->pix_nw_last = nw;
    c->pix_lane[0] = P->T.lane_w;
    c->pix_lane[1] = P->T.lane_q;
    c->pix_lane[2] = P->T.lane_base;
    // (delta pending: the last batch's last merge's rows are in xchg, for this batch's first
    // all-reduce; else all of it zero: the rows past this batch's words are read by later ones)
    if (!c->rl_delta_pending)
        HIP_TRY(hipMemsetAsync(xchg, 0, XCHG_WORDS * sizeof(unsigned long long), s));
    k_pix_rank_begin<<<1, 1, 0, s>>>(P->d_ctl, LOOP_BATCH, (int32_t)base,
                                     min_weight == 0 ? 2 : min_weight);   // core.ts:256
    HIP_TRY(hipGetLastError());
    c->opt_max_length = max_length;
    c->rl_table = xchg;
    c->rl_tie = tie;
    c->rl_rank = rank;
    c->rl_world = world;
    c->rl_base = base;
    c->rl_enqueued = 0;
    c->rl_max_length = max_length;
    c->rl_open = true;
    *n_words = nw;
    return BPE_OK;
}

int pix_rank_select(bpe_ctx *c) {
    PixState *P = c->pix;
    hipStream_t s = c->stream;
    hipEvent_t e = span_begin(c);
    // (the batch's first iteration decodes the last batch's pending merge in its layout)
    PixTable T = P->T;
    if (c->rl_enqueued == 0 && c->pix_first_pending) {
        T.lane_w = c->pix_lane_prev[0];
        T.lane_q = c->pix_lane_prev[1];
        T.lane_base = c->pix_lane_prev[2];
    }
    k_pix_apply_delta<<<PIX_GRID, 256, 0, s>>>(T, P->B, P->d_ctl, c->rl_table);
    k_pix_dirty<<<PIX_GRID, 256, 0, s>>>(P->T, P->B, P->d_ctl);
    k_pix_select<<<1, 1024, 0, s>>>(P->T, P->B, P->d_ctl);
    k_pix_sites<<<PIX_GRID, 256, 0, s>>>(P->C, P->T, P->B, P->d_ctl);
    k_pix_export<<<1, 64, 0, s>>>(P->d_ctl, c->rl_table, c->rl_tie, c->rl_rank);
    HIP_TRY(hipGetLastError());
    return span_end(c, e, 1);
}

int pix_rank_decide(bpe_ctx *c) {
    (void)c;   // (the decision is made by k_pix_alloc's block 0 in pix_rank_count)
    return BPE_OK;
}

int pix_rank_count(bpe_ctx *c) {
    PixState *P = c->pix;
    hipStream_t s = c->stream;
    hipEvent_t e = span_begin(c);
    k_pix_alloc<<<PIX_GRID, 256, 0, s>>>(P->T, P->B, P->d_ctl, c->rl_tie);   // (+ k_pix_decide)
    k_pix_apply<<<PIX_GRID, 256, 0, s>>>(P->C, P->T, P->B, P->d_ctl, P->d_log);
    HIP_TRY(hipGetLastError());
    c->rl_enqueued += 1;
    return span_end(c, e, 0);
}

int pix_rank_end(bpe_ctx *c, int64_t *out, int64_t cap, int64_t *n_done, int *status) {
    c->rl_open = false;
    PixState *P = c->pix;
    hipStream_t s = c->stream;
    PixCtl *h = P->h_ctl;
    HIP_TRY(hipMemcpyAsync(h, P->d_ctl, sizeof *h, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(P->h_log, P->d_log, PIX_LOG * std::max<int64_t>(1, c->rl_enqueued) * sizeof(long long),
                           hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (h->status == PIX_ERROR) {
        const int err = h->err;
        const unsigned long long got = h->n_check, W = h->W;
        LEAVE_GLOBAL(c);
        char msg[200];
        if (err == 21)
            snprintf(msg, sizeof msg, "bpe native: rank loop (incremental): the shards' replacement "
                     "counts sum to %llu, not W = %llu", got, W);
        else
            snprintf(msg, sizeof msg, "bpe native: rank loop (incremental): position index "
                     "inconsistent (code %d)", err);
        return fail(BPE_ERR_STATE, msg);
    }
    const int64_t nd = h->n_done;
    if (nd < 0 || nd > c->rl_enqueued) return fail(BPE_ERR_STATE, "bpe native: rank loop: bad merge count");
    const int64_t base = c->rl_base;
    c->h_len16.resize(base + nd, 1);
    c->h_count.resize(base + nd, 0);
    for (int64_t i = 0; i < nd; ++i) {
        const long long *m = P->h_log + PIX_LOG * i;
        const int32_t a = (int32_t)m[0], b = (int32_t)m[1];
        const int64_t W = m[2], R = m[3];
        const int64_t cc = base + i;
        c->h_len16[cc] = c->h_len16[a] + c->h_len16[b];                // core.ts:318
        if (c->stats_on) {
            c->stats.iterations += 1;
            c->stats.live_tokens += c->n_live;
            c->stats.pix_merges += 1;
        }
        c->n_live -= R;
        c->live_slots -= R;
        c->h_count[a] -= R;
        c->h_count[b] -= R;
        c->h_count[cc] += R;
        if (i < cap) {
            out[4 * i] = a;
            out[4 * i + 1] = b;
            out[4 * i + 2] = W;
            out[4 * i + 3] = R;
        }
    }
    c->len16_lo = base + nd;   // (pix_commit wrote the new lengths on the device)
    const int st = h->status == PIX_DONE ? LOOP_DONE : h->status == PIX_HOST ? LOOP_HOST : LOOP_RUN;
    // the next batch's lanes: the last merge's count bounds every later one's (and each of its
    // per-neighbour counts); a count past the lanes (lane_over) takes full words once
    if (nd > 0) c->pix_w_last = (unsigned long long)P->h_log[PIX_LOG * (nd - 1) + 2];
    if (h->lane_over) {
        c->pix_w_last = 0;
        HIP_TRY(hipMemsetAsync(&P->d_ctl->lane_over, 0, sizeof(uint32_t), s));
    }
    if (st != LOOP_RUN) {
        static const bool dbg = getenv("BPE_DEBUG_PIX") != nullptr;
        if (dbg)
            fprintf(stderr, "[bpe debug] rank %d: incremental rank loop hands over after %lld merges "
                    "(status %d, code %d, used %llu of %llu, pool %llu of %llu, candidates %u)\n",
                    c->rl_rank, (long long)nd, h->status, h->err, h->used, h->used_cap, h->pool_top,
                    h->pool_cap, h->n_cand);
        if (c->stats_on && st == LOOP_HOST) c->stats.pix_host += 1;
        LEAVE_GLOBAL(c);   // (the host takes over: the corpus back to the chunk layout)
    } else {
        c->rl_delta_pending = h->merged != 0;
    }
    *n_done = nd;
    *status = st;
    return BPE_OK;
}

#define MULTI(call) \
    if (c && c->multi) return multi_##call
#define NOT_MULTI                                                                          \
    if (c && c->multi)                                                                     \
        return fail(BPE_ERR_STATE, "bpe native: a per-shard entry point on a multi-device " \
                                   "context (drive its shards through bpe_create instead)")

// ================================================================================================
// C ABI
// ================================================================================================
extern "C" {

int bpe_version(void) { return 200; }

int bpe_last_error(char *buf, size_t cap) {
    if (!buf || !cap) return BPE_ERR_ARG;
    snprintf(buf, cap, "%s", g_err.c_str());
    return BPE_OK;
}

int bpe_device_count(int *n) {
    if (!n) return fail(BPE_ERR_ARG, "bpe native: null argument");
    int k = 0;
    if (hipGetDeviceCount(&k) != hipSuccess) k = 0;
    *n = k;
    return BPE_OK;
}

int bpe_create(bpe_ctx **out, int device) {
    if (!out) return fail(BPE_ERR_ARG, "bpe native: null argument");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return fail(BPE_ERR_HIP, "bpe native: no HIP device available (MI355X required)");
    if (device < 0 || device >= n) return fail(BPE_ERR_ARG, "bpe native: bad device index");
    bpe_ctx *c = new bpe_ctx();
    c->device = device;
    c->use_incr = !getenv("BPE_FUSED");
    c->use_pix = getenv("BPE_PIX") && atoi(getenv("BPE_PIX")) > 0;
    int rc;
    auto bail = [&](int code) {
        bpe_destroy(c);
        return code;
    };
    if ((rc = set_device(c))) return bail(rc);
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(BPE_ERR_HIP, "bpe native: hipStreamCreate failed"));
    if ((rc = dev_alloc(&c->d_spill, TABLE_BINS))) return bail(rc);
    if (hipMemset(c->d_spill, 0, TABLE_BINS * sizeof(unsigned long long)) != hipSuccess)
        return bail(fail(BPE_ERR_HIP, "bpe native: hipMemset failed"));
    if ((rc = dev_alloc(&c->d_hot, TABLE_BINS))) return bail(rc);
    if ((rc = dev_alloc(&c->d_heavy, HEAVY_WORDS))) return bail(rc);
    if ((rc = dev_alloc(&c->d_total, 2))) return bail(rc);
    if ((rc = dev_alloc(&c->d_sums, MAX_REGIONS))) return bail(rc);
    if ((rc = dev_alloc(&c->d_carry, MAX_REGIONS))) return bail(rc);
    if ((rc = dev_alloc(&c->d_outoff, MAX_REGIONS))) return bail(rc);
    if ((rc = dev_alloc(&c->d_res, 1))) return bail(rc);
    if ((rc = dev_alloc(&c->d_cand, CAND_CAP))) return bail(rc);
    if ((rc = dev_alloc(&c->d_cold_flags, 8))) return bail(rc);
    if (hipHostMalloc((void **)&c->h_cand, MAX_CAND * sizeof(int2), hipHostMallocDefault) != hipSuccess)
        return bail(fail(BPE_ERR_HIP, "bpe native: hipHostMalloc failed"));
    if (hipHostMalloc((void **)&c->h_res, sizeof(Result), hipHostMallocDefault) != hipSuccess)
        return bail(fail(BPE_ERR_HIP, "bpe native: hipHostMalloc failed"));
    if ((rc = dev_alloc(&c->d_ctl, 1))) return bail(rc);
    if ((rc = dev_alloc(&c->d_ticket, TICKET_WORDS))) return bail(rc);
    if ((rc = dev_alloc(&c->d_brec, COLD_GRID))) return bail(rc);
    if (hipMemset(c->d_ticket, 0, TICKET_WORDS * sizeof(unsigned int)) != hipSuccess)
        return bail(fail(BPE_ERR_HIP, "bpe native: memset failed"));
    if ((rc = dev_alloc(&c->d_repl, REPLAY_BATCH))) return bail(rc);
    if (hipHostMalloc((void **)&c->h_repl, REPLAY_BATCH * sizeof(unsigned long long),
                      hipHostMallocDefault) != hipSuccess)
        return bail(fail(BPE_ERR_HIP, "bpe native: hipHostMalloc failed"));
    if ((rc = dev_alloc(&c->d_log, LOG_WORDS * LOOP_BATCH))) return bail(rc);
    if (hipHostMalloc((void **)&c->h_ctl, sizeof(LoopCtl), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void **)&c->h_log, LOG_WORDS * LOOP_BATCH * sizeof(long long), hipHostMallocDefault) !=
            hipSuccess)
        return bail(fail(BPE_ERR_HIP, "bpe native: hipHostMalloc failed"));
    if (hipMemset(c->d_cold_flags, 0, 32) != hipSuccess)
        return bail(fail(BPE_ERR_HIP, "bpe native: memset failed"));
    if ((rc = ensure_chunks(c, 1))) return bail(rc);
    if ((rc = ensure_vocab(c, 0))) return bail(rc);
    if ((rc = ensure_cold(c, 0))) return bail(rc);
    if ((rc = seal_packed(c))) return bail(rc);
    *out = c;
    return BPE_OK;
}

int bpe_create_multi(bpe_ctx **out, int n_shards, const int *devices, int reduce) {
    if (!out) return fail(BPE_ERR_ARG, "bpe native: null argument");
    *out = nullptr;
    bpe_multi *m = nullptr;
    int rc = multi_create(&m, n_shards, devices, reduce);
    if (rc) return rc;
    bpe_ctx *c = new bpe_ctx();
    c->multi = m;
    *out = c;
    return BPE_OK;
}

int bpe_shard_count(bpe_ctx *c, int *n) {
    if (!c || !n) return fail(BPE_ERR_ARG, "bpe native: null argument");
    MULTI(shard_count(c->multi, n));
    *n = 1;
    return BPE_OK;
}

int bpe_destroy(bpe_ctx *c) {
    if (!c) return BPE_OK;
    if (c->multi) {
        multi_destroy(c->multi);
        delete c;
        return BPE_OK;
    }
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    rank_rccl_forget(c);
    pix_free(c);
    void *ptrs[] = {c->d_ids, c->d_tmp, c->d_len16, c->d_partials, c->d_spill, c->d_hot,
                    c->d_total, c->d_sums, c->d_carry, c->d_outoff, c->d_res, c->d_cand,
                    c->d_heavy, c->d_cold_flags, c->cold.slots, c->cold.dkeys, c->cold.dcounts,
                    c->cold.bmax, c->cold.bdirty, c->cold.blist,
                    c->d_ctl, c->d_log, c->d_repl, c->d_ticket, c->d_brec};
    for (void *p : ptrs) dfree(p);
    if (c->h_res) (void)hipHostFree(c->h_res);
    if (c->h_cand) (void)hipHostFree(c->h_cand);
    if (c->h_ctl) (void)hipHostFree(c->h_ctl);
    if (c->h_log) (void)hipHostFree(c->h_log);
    if (c->h_repl) (void)hipHostFree(c->h_repl);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto &sp : c->spans) c->ev_pool.insert(c->ev_pool.end(), {sp.a, sp.b});
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return BPE_OK;
}

int bpe_set_token_len16(bpe_ctx *c, int32_t id, int32_t len16) {
    MULTI(set_token_len16(c->multi, id, len16));
    if (!c || id < 0 || len16 < 0) return fail(BPE_ERR_ARG, "bpe native: bad token registration");
    if (id >= BPE_MAX_VOCAB)
        return fail(BPE_ERR_VOCAB, "bpe native: vocab is limited to 55295 tokens (UTF-16 surrogates)");
    int rc = set_device(c);
    if (rc) return rc;
    if ((rc = ensure_vocab(c, (int64_t)id + 1))) return rc;
    if (c->h_len16[id] != len16) {
        c->h_len16[id] = len16;
        mark_len16(c, id);
    }
    return BPE_OK;
}

int bpe_num_tokens(bpe_ctx *c, int32_t *n) {
    if (c && n) MULTI(num_tokens(c->multi, n));
    if (!c || !n) return fail(BPE_ERR_ARG, "bpe native: null argument");
    *n = (int32_t)c->h_len16.size();
    return BPE_OK;
}

int bpe_add_sample(bpe_ctx *c, const int32_t *ids, int64_t n) {
    if (n >= 0 && (n == 0 || ids)) MULTI(add_sample(c->multi, ids, n));
    if (!c || n < 0 || (n > 0 && !ids)) return fail(BPE_ERR_ARG, "bpe native: bad sample");
    int rc = set_device(c);
    if (rc) return rc;
    int32_t mx = -1;
    for (int64_t i = 0; i < n; ++i) {
        if (ids[i] < 0 || ids[i] >= BPE_MAX_VOCAB)
            return fail(BPE_ERR_ARG, "bpe native: token id out of range in sample");
        mx = std::max(mx, ids[i]);
    }
    if ((rc = ensure_vocab(c, (int64_t)mx + 1))) return rc;
    if ((rc = append_begin(c, n + 1))) return rc;
    std::vector<int32_t> buf(ids, ids + n);
    buf.push_back(SEP);
    HIP_TRY(hipMemcpyAsync(c->d_ids + c->live_slots, buf.data(), buf.size() * sizeof(int32_t),
                           hipMemcpyHostToDevice, c->stream));
    for (int64_t i = 0; i < n; ++i) c->h_count[ids[i]] += 1;
    c->live_slots += n + 1;
    c->n_samples += 1;
    c->n_live += n;
    if ((rc = seal_packed(c))) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return BPE_OK;
}

int bpe_add_latin1(bpe_ctx *c, const uint8_t *bytes, int64_t n, int64_t sample_bytes,
                   int32_t char_to_id[256], int32_t *n_tokens_io, int64_t char_hist[256]) {
    if (!c || n < 0 || (n > 0 && !bytes) || !char_to_id || !n_tokens_io || sample_bytes < 0)
        return fail(BPE_ERR_ARG, "bpe native: bad latin1 ingest arguments");
    MULTI(add_latin1(c->multi, bytes, n, sample_bytes, char_to_id, n_tokens_io, char_hist));
    int rc = set_device(c);
    if (rc) return rc;
    if (n == 0) {
        if (char_hist) memset(char_hist, 0, 256 * sizeof(int64_t));
        return bpe_add_sample(c, nullptr, 0);
    }
    if (sample_bytes == 0 || sample_bytes > n) sample_bytes = n;
    const int64_t n_smp = (n + sample_bytes - 1) / sample_bytes;
    if ((rc = append_begin(c, n + n_smp))) return rc;
    hipStream_t s = c->stream;
    uint8_t *d_bytes = nullptr;
    unsigned long long *d_stats = nullptr;   // first[256] + hist[256]
    int32_t *d_map = nullptr;
    if ((rc = dev_alloc(&d_bytes, n))) return rc;
    if ((rc = dev_alloc(&d_stats, 512)) || (rc = dev_alloc(&d_map, 256))) {
        dfree(d_bytes);
        dfree(d_stats);
        return rc;
    }
    auto cleanup = [&]() {
        (void)hipStreamSynchronize(s);
        dfree(d_bytes);
        dfree(d_stats);
        dfree(d_map);
    };
    std::vector<unsigned long long> st(512);
    if (hipMemcpyAsync(d_bytes, bytes, n, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemsetAsync(d_stats, 0xFF, 256 * sizeof(unsigned long long), s) != hipSuccess ||
        hipMemsetAsync(d_stats + 256, 0, 256 * sizeof(unsigned long long), s) != hipSuccess) {
        cleanup();
        return fail(BPE_ERR_HIP, "bpe native: latin1 upload failed");
    }
    const int blocks = (int)std::min<int64_t>(2048, (n + 65535) / 65536);
    k_byte_stats<<<blocks, 256, 0, s>>>(d_bytes, n, d_stats, d_stats + 256);
    if (hipMemcpyAsync(st.data(), d_stats, 512 * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                       s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        cleanup();
        return fail(BPE_ERR_HIP, "bpe native: latin1 stats failed");
    }
    // first-appearance order for unseen chars (core.ts:186-199)
    std::vector<std::pair<unsigned long long, int>> fresh;
    for (int ch = 0; ch < 256; ++ch)
        if (st[256 + ch] && char_to_id[ch] < 0) fresh.push_back({st[ch], ch});
    std::sort(fresh.begin(), fresh.end());
    int32_t next = *n_tokens_io;
    for (auto &p : fresh) {
        if (next >= BPE_MAX_VOCAB) {
            cleanup();
            return fail(BPE_ERR_VOCAB, "bpe native: vocab limit");
        }
        char_to_id[p.second] = next++;
    }
    if ((rc = ensure_vocab(c, next))) {
        cleanup();
        return rc;
    }
    for (int ch = 0; ch < 256; ++ch) {
        if (st[256 + ch] == 0) continue;
        const int32_t id = char_to_id[ch];
        c->h_count[id] += (int64_t)st[256 + ch];
        if (id >= *n_tokens_io) {
            c->h_len16[id] = 1;
            mark_len16(c, id);
        }
    }
    *n_tokens_io = next;
    if (char_hist)
        for (int ch = 0; ch < 256; ++ch) char_hist[ch] = (int64_t)st[256 + ch];
    if (hipMemcpyAsync(d_map, char_to_id, 256 * sizeof(int32_t), hipMemcpyHostToDevice, s) !=
        hipSuccess) {
        cleanup();
        return fail(BPE_ERR_HIP, "bpe native: map upload failed");
    }
    k_expand_latin1<<<4096, 256, 0, s>>>(d_bytes, n, sample_bytes, d_map,
                                         c->d_ids + c->live_slots);
    hipError_t e = hipGetLastError();
    cleanup();
    if (e != hipSuccess) return fail(BPE_ERR_HIP, "bpe native: latin1 expand failed");
    c->live_slots += n + n_smp;
    c->n_samples += n_smp;
    c->n_live += n;
    if ((rc = seal_packed(c))) return rc;
    HIP_TRY(hipStreamSynchronize(s));
    return BPE_OK;
}

int bpe_clear_corpus(bpe_ctx *c) {
    MULTI(clear_corpus(c->multi));
    if (!c) return fail(BPE_ERR_ARG, "bpe native: null context");
    int rc = set_device(c);
    if (rc) return rc;
    if ((rc = settle(c))) return rc;
    c->live_slots = c->n_samples = c->n_live = 0;
    std::fill(c->h_count.begin(), c->h_count.end(), 0);
    if ((rc = seal_packed(c))) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return BPE_OK;
}

int bpe_corpus_size(bpe_ctx *c, int64_t *n_samples, int64_t *n_tokens) {
    MULTI(corpus_size(c->multi, n_samples, n_tokens));
    if (!c) return fail(BPE_ERR_ARG, "bpe native: null context");
    int rc = set_device(c);
    if (rc) return rc;
    if ((rc = settle(c))) return rc;
    if (n_samples) *n_samples = c->n_samples;
    if (n_tokens) *n_tokens = c->n_live;
    return BPE_OK;
}

int bpe_read_corpus(bpe_ctx *c, int32_t *ids_out, int64_t ids_cap, int64_t *sample_off,
                    int64_t off_cap) {
    if (!c) return fail(BPE_ERR_ARG, "bpe native: null context");
    MULTI(read_corpus(c->multi, ids_out, ids_cap, sample_off, off_cap));
    if (ids_cap < c->n_live || off_cap < c->n_samples + 1 || (c->n_live && !ids_out) || !sample_off)
        return fail(BPE_ERR_ARG, "bpe native: read_corpus buffers too small");
    int rc = set_device(c);
    if (rc) return rc;
    if ((rc = settle(c))) return rc;
    const int64_t slots = c->n_chunks * CHUNK;
    std::vector<int32_t> buf(slots);
    if (slots)
        HIP_TRY(hipMemcpy(buf.data(), c->d_ids, slots * sizeof(int32_t), hipMemcpyDeviceToHost));
    int64_t o = 0, sidx = 0;
    sample_off[0] = 0;
    for (int64_t i = 0; i < slots; ++i) {
        const int32_t v = buf[i];
        if (v < SEP) continue;   // dead slot (TOMB or a tail tag)
        if (v == SEP) {
            if (sidx >= c->n_samples) return fail(BPE_ERR_STATE, "bpe native: corpus layout mismatch");
            sample_off[++sidx] = o;
        } else {
            if (o >= c->n_live) return fail(BPE_ERR_STATE, "bpe native: corpus layout mismatch");
            ids_out[o++] = v;
        }
    }
    if (sidx != c->n_samples || o != c->n_live)
        return fail(BPE_ERR_STATE, "bpe native: corpus layout mismatch");
    return BPE_OK;
}

int bpe_sample_lengths(bpe_ctx *c, int64_t *lens, int64_t cap) {
    if (!c) return fail(BPE_ERR_ARG, "bpe native: null context");
    MULTI(sample_lengths(c->multi, lens, cap));
    int rc = set_device(c);
    if (rc) return rc;
    return sample_lengths(c, lens, cap);
}

int bpe_read_samples(bpe_ctx *c, const int64_t *idx, int64_t n, int32_t *ids_out, int64_t ids_cap,
                     int64_t *sample_off) {
    if (!c) return fail(BPE_ERR_ARG, "bpe native: null context");
    MULTI(read_samples(c->multi, idx, n, ids_out, ids_cap, sample_off));
    int rc = set_device(c);
    if (rc) return rc;
    return read_samples(c, idx, n, ids_out, ids_cap, sample_off);
}

int bpe_find_next_merge(bpe_ctx *c, int64_t max_length, int64_t min_weight, int32_t *a,
                        int32_t *b, int64_t *w) {
    if (a && b && w) MULTI(find_next_merge(c->multi, max_length, min_weight, a, b, w));
    if (!c || !a || !b || !w) return fail(BPE_ERR_ARG, "bpe native: null argument");
    int rc = set_device(c);
    if (rc) return rc;
    return do_find(c, max_length, min_weight, a, b, w);
}

int bpe_apply_merge(bpe_ctx *c, int32_t a, int32_t b, int32_t cc, int64_t *replaced) {
    MULTI(apply_merge(c->multi, a, b, cc, replaced));
    if (!c) return fail(BPE_ERR_ARG, "bpe native: null context");
    int rc = set_device(c);
    if (rc) return rc;
    return do_apply(c, a, b, cc, replaced);
}

int bpe_rank_loop_begin(bpe_ctx *c, int64_t max_length, int64_t min_weight, uint64_t *xchg,
                        uint64_t *tie, int rank, int world, int64_t *xchg_words) {
    NOT_MULTI;
    if (!c || !xchg || !tie || rank < 0 || world < 1 || rank >= world || !xchg_words)
        return fail(BPE_ERR_ARG, "bpe native: bad rank loop arguments");
    int rc = set_device(c);
    if (rc) return rc;
    rc = rank_loop_begin(c, max_length, min_weight, (unsigned long long *)xchg,
                         (unsigned long long *)tie, rank, world, xchg_words);
    if (rc == BPE_OK) c->rl_words = *xchg_words;
    return rc;
}

int bpe_cold_counts(bpe_ctx *c, uint32_t *keys, uint64_t *counts, int64_t cap, int64_t *n) {
    NOT_MULTI;
    if (!c || !n || cap < 0) return fail(BPE_ERR_ARG, "bpe native: null argument");
    int rc = set_device(c);
    if (rc) return rc;
    return cold_counts(c, keys, (unsigned long long *)counts, cap, n);
}

int bpe_set_global_counts(bpe_ctx *c, const uint64_t *table, const uint32_t *keys,
                          const uint64_t *counts, int64_t n) {
    NOT_MULTI;
    if (!c || !table) return fail(BPE_ERR_ARG, "bpe native: null argument");
    int rc = set_device(c);
    if (rc) return rc;
    return set_global_counts(c, (const unsigned long long *)table, keys,
                             (const unsigned long long *)counts, n);
}

int bpe_rank_loop_select(bpe_ctx *c) {
    NOT_MULTI;
    if (!c) return fail(BPE_ERR_ARG, "bpe native: null context");
    int rc = set_device(c);
    if (rc == BPE_OK && c->stats_on && c->rl_open) {
        // (every iteration's exchange: one all-reduce(SUM) of rl_words words before this call)
        c->stats.xchg_bytes += c->rl_words * 8;
        c->stats.xchg_iters += 1;
    }
    return rc ? rc : rank_loop_select(c);
}

}  // extern "C"

// (internal, bpe_multi.cpp bpe_rank_loop_rccl) the buffers and size of the open batch: the
// all-reduces a caller issues must be over exactly these
int rank_loop_buffers(bpe_ctx *c, unsigned long long **xchg, unsigned long long **tie, int64_t *words) {
    if (!c || !c->rl_open) return fail(BPE_ERR_STATE, "bpe native: rank loop not begun");
    *xchg = c->rl_table;
    *tie = c->rl_tie;
    *words = c->rl_words;
    return BPE_OK;
}

extern "C" {

int bpe_rank_loop_decide(bpe_ctx *c) {
    NOT_MULTI;
    if (!c) return fail(BPE_ERR_ARG, "bpe native: null context");
    int rc = set_device(c);
    return rc ? rc : rank_loop_decide(c);
}

int bpe_rank_loop_count(bpe_ctx *c) {
    NOT_MULTI;
    if (!c) return fail(BPE_ERR_ARG, "bpe native: null context");
    int rc = set_device(c);
    return rc ? rc : rank_loop_count(c);
}

int bpe_rank_loop_end(bpe_ctx *c, int64_t *out_abwr, int64_t cap, int64_t *n_merges, int *status) {
    NOT_MULTI;
    if (!c || !n_merges || !status || (cap > 0 && !out_abwr))
        return fail(BPE_ERR_ARG, "bpe native: null argument");
    int rc = set_device(c);
    return rc ? rc : rank_loop_end(c, out_abwr, cap, n_merges, status);
}

int bpe_apply_merges(bpe_ctx *c, const int32_t *abc, int64_t n, int64_t *replaced, int count_after) {
    if (n >= 0 && (n == 0 || abc)) MULTI(apply_merges(c->multi, abc, n, replaced, count_after));
    if (!c || n < 0 || (n > 0 && !abc)) return fail(BPE_ERR_ARG, "bpe native: bad apply_merges arguments");
    int rc = set_device(c);
    if (rc) return rc;
    return replay(c, abc, n, replaced, count_after != 0);
}

// The streaming mergeUntil: batches on the device-resident loop, host iterations between them.
static int merge_until_stream(bpe_ctx *c, int64_t max_length, int64_t min_weight, int64_t max_iterations,
                       int64_t *out_abw, int64_t cap, int64_t *n_merges) {
    int rc;
    int64_t n = 0;
    const int64_t mw = min_weight == 0 ? 2 : min_weight;                  // core.ts:256
    int64_t abw[3 * LOOP_BATCH];
    // Batch size adapts to how often the host path is needed: a batch that ends early leaves its
    // remaining iterations' launches as no-ops, so after an early end the next batch is sized to
    // about twice the merges that one finished; after a batch that finished none, the device loop
    // rests for a few host iterations (backing off up to 16) before it is tried again.
    int64_t batch = LOOP_BATCH, rest = 0, backoff = 0;
    while (!max_iterations || n < max_iterations) {                      // core.ts:374-378
        // (a maintained cold table: do_find settles the pending merge with its selection, and
        // do_apply compacts)
        if (!(c->pending && c->cold_exact)) {
            if ((rc = settle(c))) return rc;
            if (c->n_live < 2) break;
            if ((rc = maybe_compact(c))) return rc;
        }
        // batches on the device while the vocabulary has room (the host path reports the limit)
        int64_t want = std::min<int64_t>(batch, BPE_MAX_VOCAB - (int64_t)c->h_len16.size());
        if (max_iterations) want = std::min<int64_t>(want, max_iterations - n);
        if (rest > 0) {
            --rest;
            want = 0;
        }
        if (want > 0) {
            int64_t nd = 0;
            int st = LOOP_DONE;
            if ((rc = loop_batch(c, max_length, mw, want, abw, &nd, &st))) return rc;
            for (int64_t i = 0; i < nd; ++i, ++n)
                if (n < cap)
                    for (int q = 0; q < 3; ++q) out_abw[3 * n + q] = abw[3 * i + q];
            if (st == LOOP_DONE) break;
            if (st == LOOP_RUN) {
                batch = std::min<int64_t>(LOOP_BATCH, 2 * batch);
                backoff = 0;
                continue;
            }
            batch = std::max<int64_t>(1, std::min<int64_t>(LOOP_BATCH, 2 * nd));
            if (nd == 0) rest = backoff = std::min<int64_t>(16, 2 * backoff + 1);
            else backoff = 0;
            if (max_iterations && n >= max_iterations) break;
        }
        // LOOP_HOST (heavy sketch buckets, many tied candidates) or no vocabulary room: one
        // host-driven iteration
        int32_t a, b;
        int64_t w;
        rc = do_find(c, max_length, min_weight, &a, &b, &w);
        if (rc == BPE_NO_MERGE) break;
        if (rc) return rc;
        const int32_t cc = (int32_t)c->h_len16.size();
        if ((rc = do_apply(c, a, b, cc, nullptr))) return rc;
        if (c->pending) c->pend_expect = w;    // checked when the count comes back
        if (n < cap) {
            out_abw[3 * n] = a;
            out_abw[3 * n + 1] = b;
            out_abw[3 * n + 2] = w;
        }
        ++n;
    }
    *n_merges = n;
    return settle(c);
}

int bpe_merge_until(bpe_ctx *c, int64_t max_length, int64_t min_weight, int64_t max_iterations,
                    int64_t *out_abw, int64_t cap, int64_t *n_merges) {
    if (n_merges && (cap <= 0 || out_abw)) MULTI(merge_until(c->multi, max_length, min_weight, max_iterations, out_abw, cap, n_merges));
    if (!c || !n_merges || (cap > 0 && !out_abw))
        return fail(BPE_ERR_ARG, "bpe native: null argument");
    int rc = set_device(c);
    if (rc) return rc;
    if (!c->use_pix) return merge_until_stream(c, max_length, min_weight, max_iterations, out_abw, cap, n_merges);
    int64_t n = 0;
    rc = pix_merge_until(c, max_length, min_weight, max_iterations, out_abw, cap, &n);
    *n_merges = n;
    if (rc != PIX_NOT_ELIGIBLE) return rc;
    // the corpus does not fit the index (or keeps failing it): the stream takes the rest
    if (max_iterations && n >= max_iterations) return settle(c);
    int64_t m = 0;
    rc = merge_until_stream(c, max_length, min_weight, max_iterations ? max_iterations - n : 0,
                            cap > n ? out_abw + 3 * n : out_abw, cap - n, &m);
    *n_merges = n + m;
    return rc;
}

int bpe_set_mode(bpe_ctx *c, int mode) {
    if (mode == BPE_MODE_STREAM || mode == BPE_MODE_INCREMENTAL) MULTI(set_mode(c->multi, mode));
    if (!c || (mode != BPE_MODE_STREAM && mode != BPE_MODE_INCREMENTAL))
        return fail(BPE_ERR_ARG, "bpe native: bad mode");
    c->use_pix = mode == BPE_MODE_INCREMENTAL;
    return BPE_OK;
}

int bpe_export_counts(bpe_ctx *c, uint64_t *table) {
    NOT_MULTI;
    if (!c || !table) return fail(BPE_ERR_ARG, "bpe native: null argument");
    int rc = set_device(c);
    if (rc) return rc;
    LEAVE_GLOBAL(c);
    if ((rc = settle(c))) return rc;
    if (!table_ok(c))
        if ((rc = run_pass(c, false, 0, 0, 0, nullptr))) return rc;
    HIP_TRY(hipMemcpyAsync(table, c->d_hot, TABLE_BINS * sizeof(uint64_t), hipMemcpyDeviceToDevice,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return BPE_OK;
}

int bpe_heavy_counts(bpe_ctx *c, const uint64_t *table, int64_t max_length, uint32_t *cold_keys,
                     uint64_t *cold_counts, int64_t cap, int64_t *n_cold) {
    NOT_MULTI;
    if (!c || !table || !n_cold || cap < 0) return fail(BPE_ERR_ARG, "bpe native: null argument");
    int rc = set_device(c);
    if (rc) return rc;
    LEAVE_GLOBAL(c);
    if ((rc = settle(c))) return rc;
    if ((rc = sync_len16(c, max_length))) return rc;
    hipStream_t s = c->stream;
    const auto *t = (const unsigned long long *)table;
    HIP_TRY(hipMemsetAsync(c->d_res, 0, sizeof(Result), s));
    k_argmax_hot<<<HOT_BINS / 256, 256, 0, s>>>(t, c->d_len16, max_length, c->d_res);
    k_heavy<<<SKETCH_BINS / 256, 256, 0, s>>>(t, c->d_res, c->d_heavy);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(c->h_res, c->d_res, sizeof(Result), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *n_cold = -1;   // no heavy bucket: the same on every rank (bpe.h)
    if (!c->h_res->n_heavy) return BPE_OK;
    *n_cold = 0;
    if ((rc = exact_pass(c))) return rc;
    uint32_t nu = 0;
    HIP_TRY(hipMemcpy(&nu, c->cold.n_used, sizeof nu, hipMemcpyDeviceToHost));
    nu = std::min<uint32_t>(nu, c->cold.mask + 1);
    *n_cold = nu;
    if ((int64_t)nu > cap) return fail(BPE_ERR_ARG, "bpe native: export buffer too small");
    if (nu) {
        if (!cold_keys || !cold_counts) return fail(BPE_ERR_ARG, "bpe native: null cold buffers");
        k_export_cold<<<256, 256, 0, s>>>(c->cold, cold_keys, (unsigned long long *)cold_counts);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize(s));
    }
    return BPE_OK;
}

int bpe_select_counts(bpe_ctx *c, const uint64_t *table, const uint32_t *cold_keys,
                      const uint64_t *cold_counts, int64_t n_cold, int64_t max_length,
                      int64_t min_weight, int32_t *cand, int64_t cap, int64_t *n_cand,
                      int64_t *w) {
    NOT_MULTI;
    const uint64_t *hot = table;
    if (!c || !hot || !n_cand || !w || n_cold < 0 || (n_cold && (!cold_keys || !cold_counts)) ||
        (cap > 0 && !cand))
        return fail(BPE_ERR_ARG, "bpe native: bad select arguments");
    int rc = set_device(c);
    if (rc) return rc;
    if (min_weight == 0) min_weight = 2;                               // core.ts:256
    if ((rc = sync_len16(c, max_length))) return rc;
    hipStream_t s = c->stream;
    HIP_TRY(hipMemsetAsync(c->d_res, 0, sizeof(Result), s));
    const auto *h = (const unsigned long long *)hot;
    const auto *cc = (const unsigned long long *)cold_counts;
    k_argmax_hot<<<HOT_BINS / 256, 256, 0, s>>>(h, c->d_len16, max_length, c->d_res);
    if (n_cold)
        k_argmax_list<<<256, 256, 0, s>>>(cold_keys, cc, n_cold, c->d_len16, max_length, c->d_res);
    k_collect_list<<<HOT_BINS / 256, 256, 0, s>>>(h, cold_keys, cc, n_cold, c->d_len16, max_length,
                                                  c->d_res, c->d_cand);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(c->h_res, c->d_res, sizeof(Result), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const Result res = *c->h_res;
    *n_cand = 0;
    if (res.best == 0) return BPE_NO_MERGE;                            // core.ts:312
    const int64_t W = (int64_t)(res.best >> 17);
    if (W < min_weight) return BPE_NO_MERGE;                           // core.ts:313
    const int64_t nc = std::min<int64_t>(res.n_cand, CAND_CAP);
    std::vector<int2> buf(nc);
    HIP_TRY(hipMemcpy(buf.data(), c->d_cand, nc * sizeof(int2), hipMemcpyDeviceToHost));
    std::sort(buf.begin(), buf.end(), [](const int2 &x, const int2 &y) {
        return x.x != y.x ? x.x < y.x : x.y < y.y;
    });
    for (int64_t i = 0; i < std::min(nc, cap); ++i) {
        cand[2 * i] = buf[i].x;
        cand[2 * i + 1] = buf[i].y;
    }
    *n_cand = res.n_cand;
    *w = W;
    return BPE_OK;
}

int bpe_tie_positions(bpe_ctx *c, const int32_t *cand, int64_t n, uint64_t *last) {
    NOT_MULTI;
    if (!c || n < 0 || (n > 0 && (!cand || !last)))
        return fail(BPE_ERR_ARG, "bpe native: bad tie arguments");
    int rc = set_device(c);
    if (rc) return rc;
    if (n > CAND_CAP) return fail(BPE_ERR_ARG, "bpe native: too many tie candidates");
    if (n == 0) return BPE_OK;
    std::vector<int2> cv(n);
    for (int64_t i = 0; i < n; ++i) cv[i] = make_int2(cand[2 * i], cand[2 * i + 1]);
    if ((rc = settle(c))) return rc;
    HIP_TRY(hipMemcpyAsync(c->d_cand, cv.data(), n * sizeof(int2), hipMemcpyHostToDevice, c->stream));
    return tie_positions(c, c->d_cand, (unsigned)n, (unsigned long long *)last);
}

int bpe_stats_enable(bpe_ctx *c, int on) {
    MULTI(stats_enable(c->multi, on));
    if (!c) return fail(BPE_ERR_ARG, "bpe native: null context");
    c->stats_on = on != 0;
    return BPE_OK;
}

int bpe_get_stats(bpe_ctx *c, bpe_stats *out) {
    if (out) MULTI(get_stats(c->multi, out));
    if (!c || !out) return fail(BPE_ERR_ARG, "bpe native: null argument");
    int rc = flush_spans(c);
    if (rc) return rc;
    *out = c->stats;
    return BPE_OK;
}

int bpe_reset_stats(bpe_ctx *c) {
    MULTI(reset_stats(c->multi));
    if (!c) return fail(BPE_ERR_ARG, "bpe native: null context");
    int rc = flush_spans(c);
    if (rc) return rc;
    memset(&c->stats, 0, sizeof c->stats);
    return BPE_OK;
}

int bpe_recount(bpe_ctx *c) {
    NOT_MULTI;
    if (!c) return fail(BPE_ERR_ARG, "bpe native: null context");
    int rc = set_device(c);
    if (rc) return rc;
    LEAVE_GLOBAL(c);
    if ((rc = settle(c))) return rc;
    return run_pass(c, false, 0, 0, 0, nullptr);
}

// (internal, bpe_multi.cpp) the exchange of shards that share one device: the sum (or max) of the
// shards' buffers written back to every one of them, on `stream` (which the caller orders after
// every shard's producer and before every shard's consumer with events).  No host copies.
}  // extern "C"
namespace {
struct ShardBufs {
    unsigned long long *p[BPE_MAX_SHARDS_ONE_DEVICE];
};
__global__ void __launch_bounds__(256) k_sum_shards(ShardBufs b, int n, size_t count, int take_max) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count;
         i += (size_t)gridDim.x * blockDim.x) {
        unsigned long long v = b.p[0][i];
        for (int r = 1; r < n; ++r) {
            const unsigned long long x = b.p[r][i];
            v = take_max ? (x > v ? x : v) : v + x;
        }
        for (int r = 0; r < n; ++r) b.p[r][i] = v;
    }
}
}  // namespace
extern "C" {
int bpe_sum_shards(unsigned long long *const *bufs, int n, size_t count, int take_max, void *stream) {
    if (n < 1 || n > BPE_MAX_SHARDS_ONE_DEVICE) return fail(BPE_ERR_ARG, "bpe native: too many shards on one device");
    ShardBufs b{};
    for (int r = 0; r < n; ++r) b.p[r] = bufs[r];
    const unsigned grid = (unsigned)std::min<size_t>(1024, (count + 255) / 256 + 1);
    k_sum_shards<<<grid, 256, 0, (hipStream_t)stream>>>(b, n, count, take_max);
    HIP_TRY(hipGetLastError());
    return BPE_OK;
}

// (internal, bpe_multi.cpp) the corpus of one shard changed outside the rank loop: every shard
// leaves the replicated global tables, so the next batch starts from the table state on all alike
int bpe_leave_global(bpe_ctx *c) {
    if (!c || c->multi) return fail(BPE_ERR_ARG, "bpe native: bad shard context");
    const int rc = set_device(c);
    if (rc) return rc;
    LEAVE_GLOBAL(c);
    return BPE_OK;
}

// (debug: BPE_DEBUG_GLOBAL, bpe_multi.cpp) this context's maintained tables: the hot bins
// (HOT_BINS u64 into hot) and the cold table's dense entries (up to cap; *n = n_used)
int bpe_debug_tables(bpe_ctx *c, uint64_t *hot, uint32_t *keys, uint64_t *counts, int64_t cap,
                     int64_t *n) {
    int rc = set_device(c);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy(hot, c->d_hot, HOT_BINS * sizeof(uint64_t), hipMemcpyDeviceToHost));
    uint32_t nu = 0;
    HIP_TRY(hipMemcpy(&nu, c->cold.n_used, sizeof nu, hipMemcpyDeviceToHost));
    uint32_t of = 0;
    HIP_TRY(hipMemcpy(&of, c->cold.overflow, sizeof of, hipMemcpyDeviceToHost));
    if (of) fprintf(stderr, "[bpe debug] cold table overflow (n_used %u, capacity %u)\n", nu, c->cold.mask + 1);
    nu = std::min<uint32_t>(nu, c->cold.mask + 1);
    *n = nu;
    const int64_t k = std::min<int64_t>(nu, cap);
    if (k) {
        HIP_TRY(hipMemcpy(keys, c->cold.dkeys, k * sizeof(uint32_t), hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(counts, c->cold.dcounts, k * sizeof(uint64_t), hipMemcpyDeviceToHost));
    }
    return BPE_OK;
}

int bpe_get_stream(bpe_ctx *c, void **stream) {
    if (stream) MULTI(get_stream(c->multi, stream));
    if (!c || !stream) return fail(BPE_ERR_ARG, "bpe native: null argument");
    *stream = (void *)c->stream;
    return BPE_OK;
}

}  // extern "C"
