// bpe_kernels.hip.h — CDNA4 (gfx950) kernels of the BPE merge-training hot path.
//
// Reference semantics: /root/reference/core.ts findNextMerge (247-326) and applyMerge (332-360);
// order-free restatement in SURVEY.md Appendix A (R1-R5).
//
// Corpus layout in HBM: one int32 slot array cut into 256-slot *chunks*.  Every sample (one
// `corpus_in_code` element, core.ts:106) is its token ids followed by one SEP (-1).  Every chunk is
// LEFT-PACKED: its live slots (tokens and SEPs) come first, dead slots (TOMB, -2) fill the tail.
// The logical corpus is the concatenation of the chunks' live prefixes.  A merge therefore never
// moves data between chunks: it rewrites only the chunks that contain a match (1 KiB each).  A
// spare all-SEP chunk follows the last chunk so "first slot of the next chunk" loads stay in range.
//
// Work decomposition: the chunks are cut into R contiguous *regions*; one wave (64 lanes) owns one
// region and streams it chunk by chunk (lane L holds slots 4L..4L+3 as one int4: a 1 KiB fully
// coalesced load per wave-instruction).  Inside a region the state that crosses chunks (the open
// run of equal tokens behind the `X X X` skip rule, core.ts:285-290) lives in wave-uniform
// registers.  Across regions nothing is shared during a pass: each wave writes a RegionSum and
// k_runs stitches the boundaries (the pair straddling each boundary, runs crossing regions, and
// the carries the next pass needs).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace bpe {

constexpr int32_t SEP = -1;                 // sample separator (live slot, never in a pair)
constexpr int32_t TOMB = -2;                // dead slot in a chunk tail
constexpr int32_t NONE = -3;                // "no token" (register sentinel only)
// Tail tag of a partial chunk (every stored value < SEP is a dead slot): slot 255 holds
// LEN_TAG - len - ((last + 3) << 8), i.e. its live length and its last live slot (NONE when empty)
// in one value, read with one v_readlane.
constexpr int32_t LEN_TAG = -16;
// Dead slots alternate TOMB (even slots) and TOMB_ODD (odd slots), so no dead slot equals its
// neighbour: equal-neighbour masks need no liveness masking.
constexpr int32_t TOMB_ODD = -4;

__host__ __device__ __forceinline__ int32_t tail_tag(int len, int32_t last) {
    return LEN_TAG - len - (int32_t)((uint32_t)(last + 3) << 8);
}
constexpr int CHUNK = 256;                  // slots per wave-chunk (64 lanes x int4)
#ifndef BPE_WAVES
#define BPE_WAVES 16
#endif
constexpr int WAVES_PER_WG = BPE_WAVES;
// Register ring of the streaming passes: RING chunks per wave (k_step: loads issued RING - 3
// chunks ahead, k_tie: RING - 2).  Depth 2 already streams at 5.8 TB/s and 12 at 6.06
// (tools/probe/stream_probe.hip).  With the round-end overflow screen, depth 6 times best over
// the full C3 run: k_step 0.760 ms against 0.767 (5), 0.795 (7), 0.83 (8, 9).
#ifndef BPE_RING
#define BPE_RING 6
#endif
constexpr int RING = BPE_RING;
static_assert(RING >= 5, "ring depth");
// (the overflow screen runs once per ring round: 16 waves x RING chunks x 256 adds must stay
// below the 49152 adds of headroom above 0x4000, see lds_sweep)
static_assert(WAVES_PER_WG * RING * 256 < 49152,
              "ring depth vs the LDS overflow screen");
// How far ahead k_step loads: chunk c + LEAD at stage c, into the slot of chunk c + LEAD - RING.
// At stage c the wave holds chunks c - 1 (count), c (apply) and c + 1 (its first token), so every
// slot of a chunk <= c - 2 is free: LEAD <= RING - 2.
#ifndef BPE_LEAD
#define BPE_LEAD (BPE_RING - 3)
#endif
constexpr int LEAD = BPE_LEAD;
static_assert(LEAD >= 2 && LEAD <= RING - 2, "load lead");

// Cache-policy bits of the streaming passes' corpus loads (buffer_load aux: 0 plain, 2 nt).  A
// pass streams 4 GB, far past the caches, so the loads are non-temporal: 6.15 -> 7.0 TB/s for
// this access pattern (tools/probe/stream_probe2.hip), k_step 2.6 % faster.
#ifndef BPE_LOAD_AUX
#define BPE_LOAD_AUX 2
#endif
// f(integral_constant<I>) for I = 0 .. N-1, unrolled in the source (the ring's slot indices must be
// compile-time constants, or the ring is moved to scratch memory)
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}
constexpr int WG = WAVES_PER_WG * 64;       // one workgroup per CU (LDS-bound)
constexpr int MAX_WG = 256;                 // one per CU on MI355X
constexpr int MAX_REGIONS = MAX_WG * WAVES_PER_WG;
constexpr int HOT = 256;                    // ids < HOT form the dense LDS histogram
constexpr int HOT_BINS = HOT * HOT;
constexpr int SKETCH_BINS = 16384;          // count sketch of the cold pairs (an id >= HOT)
constexpr int TABLE_BINS = HOT_BINS + SKETCH_BINS;   // [0, 64K) exact hot pairs, then the sketch
// Hot pair (a, b) sits at table bin b * 256 + a: the order of the LDS table's 16-bit counters
// (dword (b << 7) | (a >> 1), half a & 1), so the reduction writes the table contiguously.
__host__ __device__ constexpr uint32_t hot_bin(uint32_t a, uint32_t b) { return (b << 8) | a; }
__host__ __device__ constexpr int32_t bin_a(uint32_t bin) { return (int32_t)(bin & 255); }
__host__ __device__ constexpr int32_t bin_b(uint32_t bin) { return (int32_t)(bin >> 8); }
constexpr int HIST_WORDS = TABLE_BINS / 2;  // two 16-bit counters per LDS dword: 160 KiB, all of it
constexpr int HEAVY_WORDS = SKETCH_BINS / 32;        // bitmap of sketch buckets needing exact counts
// What a streaming pass does with the pairs it sees: the pair table, exact counts of the cold
// pairs in heavy sketch buckets, or nothing (apply-only replay: restoreMerge, batch encoding).
// MODE_FUSED: a merge pass that also refreshes the maintained cold table (the table counts plus
// MODE_EXACT's refresh of the pairs with a side in {ma, mb, mc}, in one stream of the corpus)
// MODE_INCR: incremental counts.  Both tables are maintained: the merge
// (ma, mb) -> mc changes only the counts of the pairs with a side in {ma, mb, mc} (every other pair
// keeps its occurrences and its run parity), so those are zeroed before the pass and the pass
// counts only them, into dense per-token LDS rows (no 128 KiB histogram of every pair).
enum CountMode { MODE_TABLE = 0, MODE_EXACT = 1, MODE_NONE = 2, MODE_FUSED = 3, MODE_INCR = 4 };
constexpr int MAX_CAND = 16;                // candidates resolved per tie pass
constexpr int CAND_CAP = 65536;             // candidates collected per iteration
constexpr uint32_t EMPTY = 0xFFFFFFFFu;

// What one pass learned about its region of the (post-merge) corpus.  Live slots only.
struct RegionSum {
    int64_t n_live;      // live slots (tokens + SEPs)
    int64_t lead_len;    // length of the first run (the whole region when uniform)
    int32_t first_tok;   // first live slot value (NONE when the region is empty)
    int32_t last_tok;    // last live slot value
    int32_t uniform;     // the region is one single run
    int32_t trail_odd;   // the last run's length is odd (meaningful when not uniform)
};

// Boundary facts k_runs derives for the NEXT pass over the same corpus.
struct RegionCarry {
    int64_t carry_off;   // parity of the run offset of the region's first live token (0 unless
                         // its run began in an earlier region)
    int32_t prev_tok;    // last live slot before the region (SEP at the corpus start)
    int32_t next_tok;    // first live slot after the region (SEP at the corpus end)
};

// Sparse pair table for pairs with an id >= HOT: open addressing on key = a << 16 | b.
struct ColdTable {
    // open-addressing hash of the claimed pairs: slot = (key << 32) | dense index, EMPTY64 = free
    unsigned long long *slots;
    // the dense arrays, entry i = the i-th claimed index (claim order): every scan (argmax,
    // collect, invalidate, export) streams these coalesced, and the counts live here, so a scan
    // never gathers hashed slots.  A claim that loses its slot race leaves a hole (key EMPTY,
    // count 0).  dcounts[i] == 0 for every i >= *n_used (zeroed with the table).  Counts are
    // 64-bit: one pair of a 16 GiB shard can occur more than 2^32 times (JS numbers in the
    // reference's Map are exact to 2^53, core.ts:280-292).
    uint32_t *dkeys;
    unsigned long long *dcounts;
    uint32_t *n_used;
    uint32_t *overflow;  // set when a probe sequence wraps the table or the dense arrays fill up
    uint32_t mask;       // slots - 1 (= dense capacity - 1)
    uint32_t shift;
    // Block maxima of the dense view (the device loop's maintained selection, k_select_maint):
    // per CB entries the best packed key, exact except in the blocks flagged dirty (listed in
    // blist, n_blist entries); sel_n0 = n_used at the last selection, dead = the dead claims
    // found by the last full scan.  n_blist, sel_n0 and dead follow n_used and overflow in the
    // same flags array.
    unsigned long long *bmax;
    uint32_t *bdirty, *blist;
    uint32_t *n_blist, *sel_n0, *dead;
    uint32_t *n_recomputed;   // block maxima recomputed by incremental selections (a statistic)
};
// entries per block of the cold table's block maxima
constexpr uint32_t CB = 1024;

struct Result {
    unsigned long long best;             // packed (W << 17) | (0x1FFFF - c_index), 0 = none
    unsigned int n_cand;                 // pairs sharing the best packed key (list in `cand`)
    unsigned int n_heavy;                // sketch buckets that need exact cold counts
    unsigned long long last[MAX_CAND];   // R3: slot + 1 of the last counted occurrence
    unsigned long long replaced;         // apply: replacement count
    unsigned long long cold_flags;       // k_argmax_cold: (overflow << 32) | n_used of the cold table
    unsigned long long cold_dead;        // k_argmax_cold: claims whose pair is gone (count 0, key set)
    // k_reduce_table: the largest bin of the table it wrote, plus one (0: unknown); consumed and
    // cleared by the next decision (LoopCtl::unscreened)
    unsigned long long bin_max;
};

// Device-resident mergeUntil loop (core.ts:367-384): the decision of each iteration stays in HBM and
// the next pass reads it from there, so a batch of iterations runs without a host round trip.
// Every kernel of the loop returns at once when status != LOOP_RUN (the batch has ended early).
enum LoopStatus { LOOP_RUN = 0, LOOP_DONE = 1, LOOP_HOST = 2, LOOP_ERROR = 3 };

struct LoopCtl {
    int32_t status;
    int32_t tie;          // the candidates wait for the tie pass (rule R3)
    int32_t a, b, c;      // the merge the next pass applies
    int32_t next_id;      // id of the next new token (token_table.length, core.ts:315)
    int64_t w;            // its weight (-1: no merge applied yet in this batch)
    int64_t n_done;       // merges decided in this batch (entries of the log)
    int64_t min_weight;   // after the core.ts:256 default
    int32_t n_tie;        // tie passes run in this batch
    // one rank of a sharded corpus: W is global (this shard's replacement count is logged, not
    // checked), ties take the full pass and their positions come from the all-reduced tie table
    int32_t sharded;
    int32_t max_id;       // ids below it fit the vocabulary (BPE_MAX_VOCAB): at it the batch ends
    int32_t n_tail;       // ties decided from the tail window alone (k_tie tail mode)
    int32_t n_lone;       // ... of which by the lone candidate missing from the window
    int32_t n_host;       // iterations handed to the host path (LOOP_HOST: 0 or 1 per batch)
    // the maintained cold-pair table (skewed corpora): selection reads it instead of the sketch,
    // each merge pass refreshes it (MODE_FUSED); cold_cap = its capacity (for the fill limits)
    int32_t maintained;
    // sharded: this rank holds the corpus tail (the tie pass's tail window scans it alone)
    int32_t last_rank;
    unsigned long long cold_cap;
    // sharded: this rank asks the others to hand the iteration to the host (its copy of the
    // maintained tables is too full, or dead, or the merge's refresh might not fit: facts that
    // differ between ranks, so they travel through the tie all-reduce(MAX) before any decision)
    int32_t vote;
    // sharded: the single candidate chosen before the vote (tie == 3)
    int32_t pend_a, pend_b;
    // LOOP_ERROR: 1 the replacement count (sum) != W, 2 a tie pass found no occurrence
    int32_t err;
    // (err 1: the count found and the W expected)
    unsigned long long err_got, err_want;
    // The pass applying this merge cannot take any LDS counter of any workgroup to 16 bits, so it
    // counts with adds that return nothing and no overflow screen (k_step_loop<MODE_TABLE>).  Set
    // by the decision when (largest bin of the pre-merge table) + 2 W < 2^16: a pair's count never
    // grows by a merge (a b -> c only removes occurrences of pairs next to a or b, and runs of X
    // only shrink), the new pairs (x, c) and (c, y) number W each at most, and a workgroup's LDS
    // count of a bin is at most the bin's count over the whole corpus (pairs across regions go
    // to the spill; a run's segments count at most the run's floor(L / 2)).  A sharded rank bounds
    // its own shard's counts with its own largest bin and the global W (W >= the shard's count of
    // the pair).  0 (screened) in the maintained state and for the first pass of a batch.
    int32_t unscreened;
    int32_t n_unscreened;   // decisions that set it, in this batch
};

// Merge log entry of the device loop: (a, b, W, this corpus's replacement count).
constexpr int LOG_WORDS = 4;

__device__ __forceinline__ bool loop_off(const LoopCtl *ctl) {
    return ctl && ctl->status != LOOP_RUN;
}

__device__ __forceinline__ unsigned long long pack_key(unsigned long long w, int32_t a, int32_t b) {
    return w ? ((w << 17) | (unsigned long long)(0x1FFFF - (a + b))) : 0ull;
}

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        unsigned long long o = __shfl_xor(v, d);
        v = o > v ? o : v;
    }
    return v;
}

__device__ __forceinline__ int wave_incl_sum(int v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        int o = __shfl_up(v, d);
        if (lane >= d) v += o;
    }
    return v;
}

// DPP wavefront shifts by one lane (a VALU modifier: no LDS crossbar round trip, unlike
// __shfl_*).  from_next: lane i gets lane i+1's x, lane 63 gets fill.  from_prev: lane i gets lane
// i-1's x, lane 0 gets fill.
__device__ __forceinline__ int32_t from_next(int32_t x, int32_t fill) {
    return __builtin_amdgcn_update_dpp(fill, x, 0x130, 0xF, 0xF, false);   // wave_shl:1
}

__device__ __forceinline__ int32_t from_prev(int32_t x, int32_t fill) {
    return __builtin_amdgcn_update_dpp(fill, x, 0x138, 0xF, 0xF, false);   // wave_shr:1
}

// A (token, right neighbour) pair as one word: (low 16 bits of x) << 16 | (low 16 bits of y), one
// v_perm.  Token ids are < 55296; SEP, TOMB and TOMB_ODD have low halves >= 0xFFFC, so they never
// alias one.  A tail tag (slot 255 of a partial chunk) can: code comparing packed pairs must not
// trust a match involving slot 255 of a partial chunk.
__device__ __forceinline__ uint32_t pack_pair(int32_t x, int32_t y) {
    return __builtin_amdgcn_perm((uint32_t)x, (uint32_t)y, 0x05040100u);
}

// The same packing on wave-uniform values, as scalar arithmetic.
__device__ __forceinline__ uint32_t pack_pair_s(int32_t x, int32_t y) {
    return ((uint32_t)x << 16) | ((uint32_t)y & 0xFFFFu);
}

constexpr unsigned long long EMPTY64 = ~0ull;

__device__ __forceinline__ void cold_add(const ColdTable &ct, uint32_t key, unsigned long long inc) {
    uint32_t h = (key * 0x9E3779B1u) >> ct.shift;
    uint32_t mine = EMPTY;   // the dense index this call reserved (at its first free slot)
    for (uint32_t probes = 0; probes <= ct.mask; ++probes) {
        unsigned long long v =
            __hip_atomic_load(&ct.slots[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v == EMPTY64) {
            if (mine == EMPTY) {
                mine = atomicAdd(ct.n_used, 1u);
                if (mine > ct.mask) {
                    atomicOr(ct.overflow, 1u);
                    return;
                }
                ct.dkeys[mine] = key;
            }
            v = atomicCAS(&ct.slots[h], EMPTY64, ((unsigned long long)key << 32) | mine);
            if (v == EMPTY64) {
                atomicAdd(&ct.dcounts[mine], inc);
                return;
            }
        }
        if ((uint32_t)(v >> 32) == key) {
            atomicAdd(&ct.dcounts[(uint32_t)v], inc);
            if (mine != EMPTY) ct.dkeys[mine] = EMPTY;   // (lost the race for this key: a hole)
            return;
        }
        h = (h + 1) & ct.mask;
    }
    atomicOr(ct.overflow, 1u);
}

// Claimed dense entries to scan: a claim past the capacity bumps n_used before it sees the
// overflow, so n_used alone can point past the dense arrays.
__device__ __forceinline__ uint32_t cold_used(const ColdTable &ct) {
    const uint32_t n = *ct.n_used;
    return n <= ct.mask ? n : ct.mask + 1;
}

// entries per thread and sweep of the cold-table scans (their loads in flight together)
constexpr int COLD_ILP = 8;

__device__ __forceinline__ uint32_t pair_key(int32_t x, int32_t y) {
    return ((uint32_t)x << 16) | (uint32_t)y;
}

// Sketch hash of a cold pair: h = y * SKETCH_K + (x >> 1) (one v_mad_u32_u24), sketch dword
// h & 0x1FFF = (y * K + x / 2) mod 8192 (K odd), its half x & 1.  Consecutive ids land in
// consecutive bins, so the merged tokens (allocated in sequence) spread evenly.  (Round 5: y
// multiplied, x halved, so that the fast path forms 4 h from the x << 1 its hot address uses and
// the sketch address in one more bit operation, pair_slot.  Round 4's x * K + y; a bucket of the
// ids' low bits alone, with no multiply, collided: profiles/r05_ab_sketch_low.txt.)
constexpr uint32_t SKETCH_K = 0x19B1u;
__device__ __forceinline__ uint32_t sketch_hash(int32_t x, int32_t y) {
    // (written out: left to itself the compiler may widen this to a 64-bit multiply-add)
    uint32_t h;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(h) : "v"(y), "s"(SKETCH_K), "v"((uint32_t)x >> 1));
    return h;
}

// Sketch bucket: the dword from the hash, the half from x (as for hot pairs, see below).
__device__ __forceinline__ uint32_t sketch_bucket(int32_t x, int32_t y) {
    return ((sketch_hash(x, y) & 0x1FFFu) << 1) | ((uint32_t)x & 1u);
}

// Table index of a pair: its exact bin when both ids are hot, else its sketch bucket.
// Branch-free: both forms are computed and selected.
__device__ __forceinline__ int table_index(int32_t x, int32_t y) {
    const uint32_t hot = hot_bin((uint32_t)x, (uint32_t)y);
    const uint32_t cold = HOT_BINS + sketch_bucket(x, y);
    return ((uint32_t)x | (uint32_t)y) < (uint32_t)HOT ? (int)hot : (int)cold;
}

// Where a pass's pair occurrences go.  MODE_TABLE: the per-workgroup LDS table (exact hot bins +
// cold sketch buckets, 16-bit counters) with a global u64 spill.  MODE_EXACT: exact counts of the
// cold pairs whose sketch bucket is marked heavy, into the sparse table; the rest is ignored.
// MODE_FUSED: the hot bins (no sketch: the maintained cold table counts the cold pairs) plus the
// cold pairs with a side in {ma, mb, mc}.
struct Sink {
    uint32_t *hist;                  // LDS table (MODE_TABLE)
    unsigned long long *spill;       // global u64 [TABLE_BINS]
    ColdTable ct;
    const uint32_t *heavy;           // LDS bitmap [HEAVY_WORDS] (MODE_EXACT)
    // MODE_FUSED (ma >= 0): the maintained cold table's refresh after the merge (ma, mb) -> mc,
    // every cold pair with a side in {ma, mb, mc}, whatever its bucket (heavy is then unused)
    int32_t ma, mb, mc;
    // MODE_INCR: the maintained hot table (global u64 [HOT_BINS]) and the rows' spill
    // (global u64 [4 * INCR_RLIM])
    unsigned long long *hot;
    unsigned long long *rspill;
    // MODE_INCR on a rank of a sharded corpus: the touched pairs' counts go to this shard's delta
    // rows (summed over the ranks, then added to every rank's copy of the global tables by
    // k_apply_delta) instead of straight into the tables
    unsigned long long *delta;
    // HOT_BYTES in a VGPR: the third operand of the fast path's sketch address (pair_slot)
    uint32_t hot_bytes_v;
};

// Delta rows of the sharded maintained state (include/bpe.h BPE_XCHG_*): the pairs a merge
// (a, b) -> c can change, at HDR + 6 * other + row, rows in precedence order (a, .) (b, .)
// (., a) (., b) (c, .) (., c).  Every touched pair has a side in {a, b, c}: each maps to one slot.
constexpr int XCHG_HDR = 8;
constexpr int DELTA_ROWS = 6;
constexpr int XCHG_WORDS = XCHG_HDR + DELTA_ROWS * 55296;   // BPE_MAX_VOCAB
static_assert(XCHG_WORDS >= XCHG_HDR + TABLE_BINS, "exchange buffer holds the table too");

__device__ __forceinline__ uint32_t delta_slot(int32_t x, int32_t y, int32_t a, int32_t b,
                                                int32_t c) {
    int row, other;
    if (x == a) { row = 0; other = y; }
    else if (x == b) { row = 1; other = y; }
    else if (y == a) { row = 2; other = x; }
    else if (y == b) { row = 3; other = x; }
    else if (x == c) { row = 4; other = y; }
    else { row = 5; other = x; }
    return (uint32_t)(XCHG_HDR + DELTA_ROWS * other + row);
}

template <int MODE>
__device__ __forceinline__ bool exact_wanted(const Sink &k, int32_t x, int32_t y) {
    const int idx = table_index(x, y);
    if (idx < HOT_BINS) return false;
    if (k.ma >= 0)
        return (x == k.ma) | (x == k.mb) | (x == k.mc) | (y == k.ma) | (y == k.mb) | (y == k.mc);
    const int b = idx - HOT_BINS;
    return (k.heavy[b >> 5] >> (b & 31)) & 1u;
}

// MODE_INCR: is (x, y) a valid pair with a side in {ma, mb, mc}?
__device__ __forceinline__ bool incr_touched(const Sink &k, int32_t x, int32_t y) {
    return ((x | y) >= 0) & ((x == k.ma) | (x == k.mb) | (x == k.mc) | (y == k.ma) | (y == k.mb) |
                             (y == k.mc));
}

// MODE_INCR: n occurrences of a touched pair straight into the maintained tables.
__device__ __forceinline__ void incr_global_add(const Sink &k, int32_t x, int32_t y,
                                                unsigned long long n) {
    if (k.delta) {
        atomicAdd(&k.delta[delta_slot(x, y, k.ma, k.mb, k.mc)], n);
        return;
    }
    if (((uint32_t)x | (uint32_t)y) < (uint32_t)HOT)
        atomicAdd(&k.hot[hot_bin((uint32_t)x, (uint32_t)y)], n);
    else
        cold_add(k.ct, ((uint32_t)x << 16) | (uint32_t)y, n);
}

// Adds n occurrences of (x, y) from outside the LDS table (boundary pairs, resolved runs).
template <int MODE>
__device__ __forceinline__ void add_pairs_global(const Sink &k, int32_t x, int32_t y,
                                                 unsigned long long n) {
    if (n == 0 || MODE == MODE_NONE) return;
    if (MODE == MODE_INCR) {
        if (incr_touched(k, x, y)) incr_global_add(k, x, y, n);
        return;
    }
    if (MODE == MODE_TABLE || MODE == MODE_FUSED) atomicAdd(&k.spill[table_index(x, y)], n);
    if (MODE != MODE_TABLE && exact_wanted<MODE>(k, x, y))
        cold_add(k.ct, pair_key(x, y), n);
}

// The LDS table: 16-bit counters, two per dword.
//  - hot pair (x, y), both < 256: dword (y << 7) | (x >> 1), half x & 1, i.e. byte address
//    ((x << 1) & 0x1FC) | (y << 9) and increment 1 << ((x << 4) & 16): five VALU operations, the
//    half chosen by a bit the shift amount already carries;
//  - sketch bucket b of a cold pair: dword HOT_BINS / 2 + (b >> 1), half b & 1, with
//    b = ((hash & 0x1FFF) << 1) | (x & 1): the dword from the hash, the half from x, so both
//    classes share the increment.
// Overflow: the adds return the dword they found.  Each wave ORs the returns of a ring round
// (RING chunks) together and, at the round's end, when some half it touched stood at >= 0x4000,
// sweeps the table (lds_sweep): every half >= 0x4000 gives its top two bits to the global u64
// spill (indexed by the bin, 2 * dword + half) with one atomic AND, race-free against the other
// waves' adds and sweeps.  No half can pass 0xFFFF: it receives at most 49152 adds between
// reaching 0x4000 and the first sweep, and every one of those adds comes from a wave that saw
// it at >= 0x4000 and sweeps at the end of its round, after at most RING chunks of at most 256
// adds to any one counter: 16 waves x 7 x 256 = 28672.
constexpr uint32_t HOT_BYTES = HOT_BINS * 2;   // 128 KiB

__device__ __forceinline__ uint32_t hot_addr(int32_t x, int32_t y) {
    return (((uint32_t)x << 1) & 0x1FCu) | ((uint32_t)y << 9);
}

// 1 << ((x & 1) * 16): the shift operand's low five bits of x << 4 are exactly that
__device__ __forceinline__ uint32_t hot_inc(int32_t x) {
    return 1u << (((uint32_t)x << 4) & 31u);
}

// byte address of sketch dword HOT_BINS / 2 + (h & 0x1FFF)
__device__ __forceinline__ uint32_t cold_addr(uint32_t h) { return HOT_BYTES | ((h & 0x1FFFu) << 2); }


__device__ __forceinline__ uint32_t *lds_word(const Sink &k, uint32_t addr) {
    return reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(k.hist) + addr);
}

// The halves a sweep moves: bits 14 and 15 of each.
constexpr uint32_t SWEEP_BITS = 0xC000C000u;

__device__ __forceinline__ void sweep_word(uint32_t *hist, unsigned long long *spill, int i,
                                           uint32_t w) {
    if (!(w & SWEEP_BITS)) return;
    const uint32_t old = atomicAnd(&hist[i], ~SWEEP_BITS);
    const uint32_t lo = old & 0xC000u, hi = (old >> 16) & 0xC000u;
    if (lo) atomicAdd(&spill[2 * i], (unsigned long long)lo);
    if (hi) atomicAdd(&spill[2 * i + 1], (unsigned long long)hi);
}

// One wave's sweep of LDS dwords [begin, end) (begin a multiple of 4): each half >= 0x4000 moves
// its top two bits to spill[2 * dword + half].  (Rare: no counter of the uniform C3 corpus ever
// reaches 0x4000 in a workgroup.)
__device__ __attribute__((noinline)) void lds_sweep(uint32_t *hist, unsigned long long *spill,
                                                    int lane, int begin, int end) {
    const int end4 = begin + ((end - begin) & ~3);
    for (int i = begin + 4 * lane; i < end4; i += 4 * 64) {
        const uint4 v = *reinterpret_cast<const uint4 *>(hist + i);
        sweep_word(hist, spill, i, v.x);
        sweep_word(hist, spill, i + 1, v.y);
        sweep_word(hist, spill, i + 2, v.z);
        sweep_word(hist, spill, i + 3, v.w);
    }
    for (int i = end4 + lane; i < end; i += 64) sweep_word(hist, spill, i, hist[i]);
}

// MODE_EXACT: each workgroup first sums its cold-pair counts in an LDS hash (open addressing,
// after the heavy bitmap; the table's LDS is free in that mode) and adds each distinct key to the
// global sparse table once at the end, so a skewed corpus's frequent cold pairs do not serialise
// on one global counter.  A key that finds no slot within LH_PROBES goes to the global table.
constexpr int LH_BITS = 14;
constexpr int LH_SLOTS = 1 << LH_BITS;   // (key, count) dword pairs: 128 KiB
constexpr int LH_PROBES = 8;
static_assert(HEAVY_WORDS + 2 * LH_SLOTS <= HIST_WORDS, "LDS cold hash does not fit");

__device__ __forceinline__ void lds_cold_add(const Sink &k, uint32_t key, uint32_t inc) {
    uint32_t *keys = k.hist + HEAVY_WORDS;
    uint32_t *cnt = keys + LH_SLOTS;
    uint32_t h = (key * 0x9E3779B1u) >> (32 - LH_BITS);
    for (int p = 0; p < LH_PROBES; ++p) {
        uint32_t kk = __hip_atomic_load(&keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (kk == EMPTY) kk = atomicCAS(&keys[h], EMPTY, key);   // (EMPTY: this lane claimed it)
        if (kk == EMPTY || kk == key) {
            atomicAdd(&cnt[h], inc);
            return;
        }
        h = (h + 1) & (LH_SLOTS - 1);
    }
    cold_add(k.ct, key, inc);
}

// MODE_FUSED's LDS hash: all of the sketch dwords (the sketch is not kept while the cold table is
// maintained), (key, count) x 4096.
constexpr int FH_BITS = 12;
constexpr int FH_SLOTS = 1 << FH_BITS;
constexpr int FH_BASE = HOT_BINS / 2;   // dword index of the first key
static_assert(FH_BASE + 2 * FH_SLOTS == HIST_WORDS, "fused LDS hash = the sketch's dwords");

__device__ __forceinline__ void lds_fused_add(const Sink &k, uint32_t key, uint32_t inc) {
    uint32_t *keys = k.hist + FH_BASE;
    uint32_t *cnt = keys + FH_SLOTS;
    uint32_t h = (key * 0x9E3779B1u) >> (32 - FH_BITS);
    for (int p = 0; p < LH_PROBES; ++p) {
        uint32_t kk = __hip_atomic_load(&keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (kk == EMPTY) kk = atomicCAS(&keys[h], EMPTY, key);
        if (kk == EMPTY || kk == key) {
            atomicAdd(&cnt[h], inc);
            return;
        }
        h = (h + 1) & (FH_SLOTS - 1);
    }
    cold_add(k.ct, key, inc);
}

// MODE_INCR's LDS: four rows of 16-bit counters indexed by the pair's other token, for the pairs
// (ma, y), (mb, y), (x, ma), (x, mb) in this order of precedence (each pair counts once), the
// other token below INCR_RLIM; then a hash of (key, count) dwords for everything else touched
// (the pairs of mc, and other tokens >= INCR_RLIM).  Overflow as in the hot table: the round's
// screen and lds_sweep over the rows' used part, to the global rspill rows.
constexpr int INCR_RLIM = 18432;                       // counters per row
constexpr int IH_SLOTS = 2048;
constexpr int IH_BASE = 4 * INCR_RLIM / 2;             // dword index of the hash keys
static_assert(IH_BASE + 2 * IH_SLOTS == HIST_WORDS, "MODE_INCR LDS layout");

// counters of a row in use: other tokens below the vocabulary size after the merge (mc + 1)
static_assert(INCR_RLIM % 2 == 0, "a row's counters pair up in dwords");
__device__ __forceinline__ int incr_vlim(int32_t mc) {
    const int v = (mc + 2) & ~1;
    return v < INCR_RLIM ? v : INCR_RLIM;
}

__device__ __forceinline__ void incr_hash_add(const Sink &k, uint32_t key, uint32_t inc) {
    uint32_t *keys = k.hist + IH_BASE;
    uint32_t *cnt = keys + IH_SLOTS;
    uint32_t h = (key * 0x9E3779B1u) >> (32 - 11);
    for (int p = 0; p < LH_PROBES; ++p) {
        uint32_t kk = __hip_atomic_load(&keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (kk == EMPTY) kk = atomicCAS(&keys[h], EMPTY, key);
        if (kk == EMPTY || kk == key) {
            atomicAdd(&cnt[h], inc);
            return;
        }
        h = (h + 1) & (IH_SLOTS - 1);
    }
    incr_global_add(k, (int32_t)(key >> 16), (int32_t)(key & 0xFFFFu), inc);
}

// One occurrence of a pair touched by the merge (incr_touched) into MODE_INCR's LDS.
__device__ __forceinline__ void incr_add(const Sink &k, int32_t x, int32_t y, uint32_t &seen) {
    int row, idx;
    if (x == k.ma) {
        row = 0;
        idx = y;
    } else if (x == k.mb) {
        row = 1;
        idx = y;
    } else if (y == k.ma) {
        row = 2;
        idx = x;
    } else if (y == k.mb) {
        row = 3;
        idx = x;
    } else {
        row = 4;
        idx = INCR_RLIM;
    }
    if (idx >= INCR_RLIM) {
        incr_hash_add(k, ((uint32_t)x << 16) | (uint32_t)y, 1u);
        return;
    }
    const uint32_t c = (uint32_t)(row * INCR_RLIM + idx);
    const uint32_t sh = (c & 1u) << 4;
    // (the round's overflow screen, as for the hot table: consumed at once, see count_pair)
    uint32_t old = atomicAdd(&k.hist[c >> 1], 1u << sh);
    asm volatile("" : "+v"(old));
    seen |= old;
}

// One counted occurrence of (x, y) (outside the streaming fast paths).
// (MODE_TABLE / MODE_FUSED: the dword the add found is ORed into `seen`, the wave's overflow
// screen; see lds_sweep)
template <int MODE, bool SCREEN = true>
__device__ __forceinline__ void count_pair(const Sink &k, int32_t x, int32_t y, uint32_t &seen) {
    if (MODE == MODE_NONE) return;
    if (MODE == MODE_INCR) {
        if (incr_touched(k, x, y)) incr_add(k, x, y, seen);
        return;
    }
    if (MODE == MODE_TABLE || MODE == MODE_FUSED) {
        const bool hot = ((uint32_t)x | (uint32_t)y) < (uint32_t)HOT;
        const uint32_t addr = hot ? hot_addr(x, y) : cold_addr(sketch_hash(x, y));
        // (MODE_FUSED keeps no sketch: its cold pairs go to the maintained table only)
        if (MODE == MODE_TABLE && !SCREEN) {
            atomicAdd(lds_word(k, addr), hot_inc(x));
        } else if (MODE == MODE_TABLE || hot) {
            // (consumed at once: a `seen` still in flight would make every later join wait for
            // all of the wave's LDS adds, the fast path's deferred ones included)
            uint32_t old = atomicAdd(lds_word(k, addr), hot_inc(x));
            asm volatile("" : "+v"(old));
            seen |= old;
        }
        if (MODE == MODE_FUSED && exact_wanted<MODE>(k, x, y)) lds_fused_add(k, pair_key(x, y), 1u);
    } else if (exact_wanted<MODE>(k, x, y)) {
        lds_cold_add(k, pair_key(x, y), 1u);
    }
}

// ---------------------------------------------------------------------------------------------
// A left-packed chunk as seen by one lane: slots k = 4*lane + e, live iff k < len.
// ---------------------------------------------------------------------------------------------
struct View {
    int32_t t[4];
    int len;
};

__device__ __forceinline__ View make_view(const int4 v) {
    View w;
    w.t[0] = v.x;
    w.t[1] = v.y;
    w.t[2] = v.z;
    w.t[3] = v.w;
    // chunks are left-packed, so len = number of non-TOMB slots (256 iff the last slot is live)
    if (__builtin_amdgcn_readlane(v.w, 63) >= SEP) {
        w.len = CHUNK;
    } else {
        w.len = (LEN_TAG - __builtin_amdgcn_readlane(v.w, 63)) & 255;
    }
    return w;
}

template <typename T>
__device__ __forceinline__ T pick4(const T (&a)[4], int e) {
    const T a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
    return e == 0 ? a0 : e == 1 ? a1 : e == 2 ? a2 : a3;
}

// c ? a : b on values (a conditional over two lvalues compiles to a select of their addresses,
// which pins arrays and structs in registers to scratch)
template <typename T>
__device__ __forceinline__ T sel(bool c, T a, T b) { return c ? a : b; }

// Broadcast of lane `src` (wave-uniform) through v_readlane.
__device__ __forceinline__ int32_t bcast(int32_t v, int src) {
    return __builtin_amdgcn_readlane(v, src);
}

__device__ __forceinline__ int64_t bcast64(int64_t v, int src) {
    const int32_t lo = __builtin_amdgcn_readlane((int32_t)(v & 0xFFFFFFFF), src);
    const int32_t hi = __builtin_amdgcn_readlane((int32_t)(v >> 32), src);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// Token at chunk index k (wave-uniform k), broadcast.
__device__ __forceinline__ int32_t view_at(const View &w, int k) {
    return bcast(pick4(w.t, k & 3), k >> 2);
}

// Neighbourhood of each live slot: partner = next live token (the pair's right side), prev.
struct Nbr {
    int32_t partner[4];
    bool live[4];
    bool eqn[4];   // live, non-SEP, equal to partner  (an X X pair starts here)
    bool eqp[4];   // live, non-SEP, equal to the previous live token (continues a run)
};

__device__ __forceinline__ void neighbours(const View &w, int32_t prev, int32_t nxt, int lane,
                                           Nbr &n) {
    const int32_t dn = from_next(w.t[0], nxt);
    const int32_t pm = from_prev(w.t[3], prev);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int k = 4 * lane + e;
        n.live[e] = k < w.len;
        const int32_t right = sel(e < 3, w.t[e < 3 ? e + 1 : 0], dn);
        n.partner[e] = (k + 1 < w.len) ? right : nxt;
        const int32_t left = sel(e == 0, pm, w.t[e > 0 ? e - 1 : 0]);
        n.eqp[e] = n.live[e] && w.t[e] >= 0 && w.t[e] == left;
        n.eqn[e] = n.live[e] && w.t[e] >= 0 && w.t[e] == n.partner[e];
    }
}

// Run-start scan over the live prefix: rs[e] = chunk index of the start of the run containing
// slot 4*lane+e, or -1 when that run began before the chunk.
__device__ __forceinline__ void run_starts(const Nbr &n, int lane, int rs[4]) {
    int lmax = -1;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        if (n.live[e] && !n.eqp[e]) lmax = 4 * lane + e;
        rs[e] = lmax;
    }
    int incl = lmax;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        int o = __shfl_up(incl, d);
        if (lane >= d) incl = o > incl ? o : incl;
    }
    int excl = __shfl_up(incl, 1);
    if (lane == 0) excl = -1;
#pragma unroll
    for (int e = 0; e < 4; ++e) rs[e] = max(rs[e], excl);
}

// Exact run offsets of the live slots (needed where X X pairs are matched / located exactly).
// prev_off = offset of the live token before the chunk (valid when slot 0 continues its run).
// Returns the offset of the last live slot (the next chunk's prev_off).
__device__ __forceinline__ int64_t run_offsets(const View &w, const Nbr &n, int lane,
                                               int64_t prev_off, int64_t (&off)[4]) {
    bool slow = false;
#pragma unroll
    for (int e = 0; e < 4; ++e) slow |= n.eqn[e] && n.eqp[e];
    if (__ballot(slow) == 0ull) {
        // every X X slot starts its run (offset 0); a run reaching the next chunk starts at the
        // last live slot, so the carried offset is 0 whenever it is used
#pragma unroll
        for (int e = 0; e < 4; ++e) off[e] = 0;
        return 0;
    }
    int rs[4];
    run_starts(n, lane, rs);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int k = 4 * lane + e;
        off[e] = rs[e] >= 0 ? (int64_t)(k - rs[e]) : prev_off + 1 + k;
    }
    const int kl = w.len - 1;
    return bcast64(pick4(off, kl & 3), kl >> 2);
}

// ---------------------------------------------------------------------------------------------
// Chunk re-packing in registers (no LDS: it is all pair table).  Each kept slot moves left by
// D = the number of dropped slots before it, one binary digit of D per step, least significant
// first; that order never lands two slots on one position.  A slot travels as one dword:
// value+1 (17 bits) | D << 17 (8 bits) | kept << 25.  Returns the new live length.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int compact_chunk(int32_t (&val)[4], const bool (&keep)[4], int len,
                                             int lane) {
    const unsigned long long K0 = __ballot(keep[0]), K1 = __ballot(keep[1]),
                             K2 = __ballot(keep[2]), K3 = __ballot(keep[3]);
    const int total = __popcll(K0) + __popcll(K1) + __popcll(K2) + __popcll(K3);
    int kb = (int)(__builtin_amdgcn_mbcnt_hi((uint32_t)(K0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)K0, 0)) +
                   __builtin_amdgcn_mbcnt_hi((uint32_t)(K1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)K1, 0)) +
                   __builtin_amdgcn_mbcnt_hi((uint32_t)(K2 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)K2, 0)) +
                   __builtin_amdgcn_mbcnt_hi((uint32_t)(K3 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)K3, 0)));
    constexpr uint32_t KEPT = 1u << 25;
    uint32_t pk[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const uint32_t d = (uint32_t)(4 * lane + e - kb);
        pk[e] = keep[e] ? ((uint32_t)(val[e] + 1) | (d << 17) | KEPT) : 0u;
        kb += keep[e];
    }
    const int dmax = len - total;   // dropped live slots; dead slots all follow the live ones
    for (int sh = 1; sh <= dmax; sh <<= 1) {
        uint32_t nb[4];   // the slot sh positions to the right
        if (sh == 1) {
            nb[0] = pk[1];
            nb[1] = pk[2];
            nb[2] = pk[3];
            nb[3] = (uint32_t)from_next((int32_t)pk[0], 0);
        } else if (sh == 2) {
            nb[0] = pk[2];
            nb[1] = pk[3];
            nb[2] = (uint32_t)from_next((int32_t)pk[0], 0);
            nb[3] = (uint32_t)from_next((int32_t)pk[1], 0);
        } else {
            const int dl = sh >> 2;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t x = __shfl_down(pk[e], dl);
                nb[e] = sel(lane < 64 - dl, x, 0u);
            }
        }
        const uint32_t bit = (uint32_t)sh << 17;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const bool mv = (nb[e] & KEPT) && (nb[e] & bit);
            const bool stay = (pk[e] & KEPT) && !(pk[e] & bit);
            pk[e] = sel(mv, nb[e], sel(stay, pk[e], 0u));
        }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
        val[e] = sel(4 * lane < total - e, (int32_t)(pk[e] & 0x1FFFFu) - 1, (e & 1) ? TOMB_ODD : TOMB);
    return total;
}

// ---------------------------------------------------------------------------------------------
// K1 (fused with K4): the streaming pass.
//
// One wave streams one region chunk by chunk through a 6-slot register ring (the loop is unrolled
// by 6, so every slot is a fixed set of registers and nothing is ever copied):
//   - the current chunk j is applied in place (merge passes), its right-hand neighbour being the
//     first live token of chunk j+1, already in the ring;
//   - the post-merge chunk before it (the ring slot of j-1) is counted, its right-hand neighbour
//     being the first post-merge token of chunk j;
//   - that slot is then refilled with chunk j+5.
// Empty chunks (rare: every token deleted) hand the pending chunk on to the next slot.
//
// Per-slot tests are vector compares whose results are wave masks (SGPR pairs); everything
// derived from them is scalar work.  Only the pair-table address arithmetic and the compares are
// vector instructions on the common path.
//
// X X pairs follow the reference's skip rule (core.ts:285-290): an X X pair counts iff its left
// slot sits at an even offset of its maximal run of X.  The wave carries the offset parity of the
// last token from chunk to chunk, and measures the region's first run from the region start as if
// nothing preceded it; k_runs adds what that assumption missed for runs that cross regions.  A
// chunk with no slot in the middle of a run of three or more (the common case) needs no parity:
// then every valid pair counts.
// ---------------------------------------------------------------------------------------------

// Registers of one ring slot: the lane's four slots + wave-uniform facts.
struct Chunk {
    int32_t t[4];
    int len;         // live slots (left-packed)
    int32_t first;   // slot 0 (dead when empty)
    int32_t last;    // last live slot (NONE when empty)
};

// Slot k (wave-uniform) broadcast from its lane.
__device__ __forceinline__ int32_t slot_at(const int32_t (&t)[4], int k) {
    const int l = k >> 2;
    switch (k & 3) {
    case 0: return bcast(t[0], l);
    case 1: return bcast(t[1], l);
    case 2: return bcast(t[2], l);
    default: return bcast(t[3], l);
    }
}

__device__ __forceinline__ bool lane_in(unsigned long long m) {
    return __builtin_amdgcn_inverse_ballot_w64(m);
}

// Lanes whose plane-e slot 4*lane + e lies below n.
__device__ __forceinline__ unsigned long long lanes_upto(int n, int e) {
    const int m = (n - e + 3) >> 2;
    return m >= 64 ? ~0ull : m <= 0 ? 0ull : ((1ull << m) - 1ull);
}

// Lanes whose t is one of ma, mb, mc: three compares straight into lane masks, OR'ed on the scalar
// unit.  (A ballot of the OR of the three compares made the compiler materialise the OR as a 0/1
// vector value and compare it again: two more VALU per token.)
__device__ __forceinline__ unsigned long long member3(int32_t t, int32_t ma, int32_t mb, int32_t mc) {
    return __ballot(t == ma) | __ballot(t == mb) | __ballot(t == mc);
}

// Wave-uniform facts of a freshly loaded chunk, from slot 255 (a live token, or the tail tag).
__device__ __forceinline__ void finish_load(Chunk &c, int32_t first) {
    c.first = first;
    const int32_t l3 = bcast(c.t[3], 63);
    const int32_t v = LEN_TAG - l3;
    const int live = l3 >= SEP;
    c.len = live ? CHUNK : (v & 255);
    c.last = live ? l3 : (v >> 8) - 3;
}
__device__ __forceinline__ void finish_load(Chunk &c) { finish_load(c, bcast(c.t[0], 0)); }

// Exact run-offset parity of every live slot (SEPs are runs of their own), and the run starts.
// prev = the live token before slot 0 (NONE: none), prev_par = the parity of its offset.
__device__ __forceinline__ void run_parity(const int32_t (&t)[4], int len, int32_t prev,
                                           int prev_par, int lane, int (&par)[4],
                                           bool (&start)[4]) {
    const int32_t l0 = from_prev(t[3], prev);
    int lmax = -1;
    int rs[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int k = 4 * lane + e;
        const int32_t left = sel(e == 0, l0, t[e > 0 ? e - 1 : 0]);
        start[e] = k < len && !(t[e] >= 0 && t[e] == left);
        if (start[e]) lmax = k;
        rs[e] = lmax;
    }
    int incl = lmax;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(incl, d);
        if (lane >= d) incl = o > incl ? o : incl;
    }
    int excl = __shfl_up(incl, 1);
    if (lane == 0) excl = -1;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int k = 4 * lane + e;
        const int s = max(rs[e], excl);
        par[e] = s >= 0 ? ((k - s) & 1) : ((prev_par + 1 + k) & 1);
    }
}

// Count-side state of one region (wave-uniform).
struct Tally {
    int32_t n_live;      // live slots counted so far
    int32_t lead_len;    // length of the region's first run (once it has ended)
    int32_t prev;        // last live token counted (NONE before the first)
    int32_t par;         // run-offset parity of prev (the first run counts from the region start)
    int32_t first_tok;   // the region's first live token
    int32_t in_lead;     // every live token so far belongs to the region's first run
    uint32_t seen;       // (per lane) OR of the words the exact path's LDS adds returned
};

// LDS adds of one chunk's pairs (x[e], y[e]), then the overflow screen.  Per pair (11 VALU): the
// hot address (three operations: x << 1, y << 9, one bit operation), the sketch address (two:
// a multiply-add on x << 1, one bit operation), u = ~(x | y) (one, opaque to the compiler so both
// uses below read it as is), the class select (two), and the increment (three): hot_inc(x) for a
// valid pair, 0 when a side is negative (SEP, dead), with the validity bit (u's sign) as the value
// shifted.  Pairs with a cold side go to their sketch bucket (its half is also x & 1).
// FUSED (the maintained cold table counts the cold pairs): a cold pair adds 0 to a hot dword (its
// address masked into the hot table) instead of going to the sketch.
template <bool FUSED = false>
__device__ __forceinline__ void pair_slot(const Sink &k, int32_t x, int32_t y, uint32_t &addr,
                                          uint32_t &inc) {
    uint32_t u = ~((uint32_t)x | (uint32_t)y);
    asm("" : "+v"(u));
    if (FUSED) {
        const uint32_t hot = (((uint32_t)x << 1) & 0x1FCu) | ((uint32_t)y << 9);
        addr = hot & (HOT_BYTES - 4);
        inc = (uint32_t)(u >= 0xFFFFFF00u) << (((uint32_t)x << 4) & 31u);   // both ids < 256
    } else {
        // both addresses as (a & b) | c (v_bitop3 table 0xEA): the hot one from x << 1 and
        // y << 9; the sketch one from 4 h = y * 4K + (x << 1) (the sketch hash times 4: its
        // dword's byte offset in bits 2..14) and HOT_BYTES
        const uint32_t x2 = (uint32_t)x << 1;
        uint32_t hot, h4, cold;
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xea"
            : "=v"(hot) : "v"(x2), "s"(0x1FCu), "v"((uint32_t)y << 9));
        asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(h4) : "v"(y), "s"(4u * SKETCH_K), "v"(x2));
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xea" : "=v"(cold) : "v"(h4), "s"(0x7FFCu), "v"(k.hot_bytes_v));
        addr = sel(u >= 0xFFFFFF00u, hot, cold);   // both ids < 256
        inc = (u >> 31) << (((uint32_t)x << 4) & 31u);
    }
}

// The words a fast-path count's LDS adds returned (0 when the chunk took another path), and their
// byte addresses.  Each stage of a ring round keeps its own, and they are all screened together at
// the round's end, so the waves wait on LDS returns once per RING chunks, not once per chunk.
// (Screening each chunk's returns one stage later left the compiler a wait for every add still
// in flight at each stage: 5 % of the pass.)  The addresses let the screen sweep just the words
// its adds saw at >= 0x4000 (round 5; see screen_round).
struct Defer {
    uint32_t o[4];
    uint32_t a[4];
};

// The LDS adds of a fast-path chunk; their returned words and
// addresses go to df, screened at the end of the
// ring round (Returns), so no wave waits on its LDS atomics' return before then.
// SCREEN false (MODE_TABLE, when no LDS counter can reach 16 bits in this pass: see LoopCtl::
// unscreened): the adds return nothing, and no word is kept for a screen.
template <bool FUSED = false, bool SCREEN = true>
__device__ __forceinline__ void add_pairs(const int32_t (&x)[4], const int32_t (&y)[4],
                                          const Sink &k, Defer &df) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        uint32_t addr, inc;
        pair_slot<FUSED>(k, x[e], y[e], addr, inc);
        if (SCREEN) {
            df.o[e] = atomicAdd(lds_word(k, addr), inc);
            df.a[e] = addr;
        } else {
            atomicAdd(lds_word(k, addr), inc);   // (ds_add_u32: no return to wait for)
        }
    }
}


// MODE_TABLE merge passes: a chunk's pair-table slots (pair_slot) made at apply time, from the
// chunk before the merge, and counted by the next stage's count of the same chunk whenever the
// merge left it as it was (no rewrite: nearly every chunk).  The apply test then compares the
// slots with the merge's own slot (4 VALU, where packing the pairs cost 8), and the count makes no
// slot again.  A slot stands for two hot pairs (x, y) and (x ^ 1, y) (the counter's half is in
// inc), and for a sketch dword's cold pairs: such a false hit only sends the chunk to the exact
// apply test, which finds no match.
struct Prep {
    uint32_t addr[4], inc[4];
    int32_t x3, r3;   // plane 3's pair: lane 63 of a partial chunk holds (last live slot, nx)
    int32_t nx;       // the first live token after the chunk that r3 was made with
    int32_t ok;       // the slots hold the chunk's current pairs (0: rewritten, or not made)
};

__device__ __forceinline__ void prep_pairs(const int32_t (&t)[4], int len, int32_t last,
                                           int32_t nxt, const Sink &k, Prep &p) {
    const unsigned long long P63 = (unsigned long long)((int64_t)len - CHUNK) & (1ull << 63);
    p.x3 = sel(lane_in(P63), last, t[3]);
    p.r3 = from_next(t[0], nxt);
    const int32_t x[4] = {t[0], t[1], t[2], p.x3}, y[4] = {t[1], t[2], t[3], p.r3};
#pragma unroll
    for (int e = 0; e < 4; ++e) pair_slot<false>(k, x[e], y[e], p.addr[e], p.inc[e]);
    p.nx = nxt;
    p.ok = 1;
}

// The fast-path pairs (x[e], y[e]) of a chunk with a side in {ma, mb, mc} (MODE_FUSED's refresh
// of the maintained cold table): per-token membership masks (compares into lane masks,
// combined on the scalar unit), one wave-wide test, and the LDS hash only in chunks that hold
// such a cold pair.  (t3 differs from x3 only in lane 63 of a partial chunk, where pair 2's right
// side is the tail tag, negative: that pair is not live either way.)
template <int MODE>
__device__ __forceinline__ void refresh_pairs(const Sink &k, int32_t t0, int32_t t1, int32_t t2,
                                              int32_t x3, int32_t r3, const int32_t (&x)[4],
                                              const int32_t (&y)[4]) {
    const int32_t ma = k.ma, mb = k.mb, mc = k.mc;
    const unsigned long long M0 = member3(t0, ma, mb, mc), M1 = member3(t1, ma, mb, mc),
                             M2 = member3(t2, ma, mb, mc), M3 = member3(x3, ma, mb, mc),
                             M4 = member3(r3, ma, mb, mc);
    const unsigned long long W0 = M0 | M1, W1 = M1 | M2, W2 = M2 | M3, W3 = M3 | M4;
    if ((W0 | W1 | W2 | W3) == 0ull) return;
    const unsigned long long Wm[4] = {W0, W1, W2, W3};
#pragma unroll
    for (int e = 0; e < 4; ++e)
        if (lane_in(Wm[e]) & ((x[e] | y[e]) >= HOT)) {
            lds_fused_add(k, pair_key(x[e], y[e]), 1u);
        }
}

// Counts the pairs of one post-merge chunk (len > 0) whose right side lies inside the region:
// nxt = the first live token of the next non-empty chunk, NONE past the region's end.
//
// Fast path: no slot inside a run of >= 3 and, for a partial chunk, a last token that differs
// from nxt.  A partial chunk's last pair (last, nxt) is moved to lane 63's slot 3 (dead in a
// partial chunk), so no lane-dependent fix-up is needed.  Everything else (runs of >= 3, the
// region's first run, a partial chunk ending in an X X pair) takes the exact path.
//
// Per-slot conditions are wave masks combined with 64-bit bitwise operations and uniform
// conditions are integers: no short-circuit operators on the common path (they become control
// flow whose booleans round-trip through vector registers).
// TAIL: the region's last chunk (nxt = NONE).  It always takes the exact path: the parity of its
// last token's run offset feeds RegionSum::trail_odd, which k_runs needs whenever that run goes on
// in the next region, and the fast path does not work that parity out.
// Fast-path counts of MODE_TABLE / MODE_FUSED leave the words their adds returned in `df`, and the
// other paths OR theirs into s.seen: the overflow screen of the ring round (screen_round).
template <int MODE, bool TAIL = false, bool SCREEN = true, bool PREP = false>
__device__ __forceinline__ void count_chunk(const Chunk &w, int32_t nxt, int lane, Tally &s,
                                            const Sink &k, Defer &df, Prep &pp) {
    const int len = w.len;
    if (MODE == MODE_NONE && !TAIL) {
        // apply-only passes keep only the region sums: the chunk needs work only in the region's
        // first run, or when its last token's run goes on in the next chunk (its parity)
        const uint32_t lead0 = (uint32_t)__builtin_amdgcn_readfirstlane(s.in_lead);
        if ((lead0 | (uint32_t)(w.last == nxt)) == 0u) {
            s.first_tok = s.n_live ? s.first_tok : w.first;
            s.par = 0;
            s.prev = w.last;
            s.n_live += len;
            return;
        }
    }
#ifdef BPE_PROBE_NOCOUNT
    if (MODE == MODE_TABLE) {   // (timing probe only: the ring and its bookkeeping, no counting)
        s.first_tok = s.n_live ? s.first_tok : w.first;
        s.par = 0;
        s.prev = w.last;
        s.n_live += len;
        s.in_lead = 0;
        return;
    }
#endif
    const int32_t t0 = w.t[0], t1 = w.t[1], t2 = w.t[2], t3 = w.t[3];
    // lane 63's bit when the chunk is partial (an integer mask, not a boolean: uniform booleans
    // cost a lane-mask round trip per use)
    const unsigned long long P63 = (unsigned long long)((int64_t)len - CHUNK) & (1ull << 63);
    if (PREP && !TAIL) {
        // the slots made at apply time (Prep): made now if the merge rewrote the chunk, plane 3
        // made again if the first token after it changed (a merge at the next chunk's start)
        if (!pp.ok) {
            prep_pairs(w.t, len, w.last, nxt, k, pp);
        } else if (pp.nx != nxt) {
            pp.r3 = from_next(t0, nxt);
            pair_slot<false>(k, pp.x3, pp.r3, pp.addr[3], pp.inc[3]);
            pp.nx = nxt;
        }
    }
    // slot 3 of lane 63 holds the last live slot (a partial chunk's slot 255 is its tail tag)
    const int32_t x3 = PREP && !TAIL ? pp.x3 : sel(lane_in(P63), w.last, t3);
    const int32_t r3 = PREP && !TAIL ? pp.r3 : from_next(t0, nxt);
    const int32_t l0 = from_prev(t3, s.prev);
    // E*: slot equals its right-hand neighbour (Em1: slot 0 equals the token before it).  No
    // dead slot equals its neighbour and slot 0 is live (an SEP next to an SEP only sends the chunk
    // to the exact path); E3's lane-63 bit compares the last live slot with nxt.
    const unsigned long long Em1 = __ballot(t0 == l0), E0 = __ballot(t0 == t1),
                             E1 = __ballot(t1 == t2), E2 = __ballot(t2 == t3), E3 = __ballot(x3 == r3);
    const unsigned long long trip = (E0 & (Em1 | E1)) | (E2 & (E1 | E3));
    // fast: no run of three, not in the region's first run, and a partial chunk does not end in
    // an X X pair
    // (readfirstlane: the compiler cannot see that in_lead is wave-uniform, and would branch on it
    // per lane)
    const unsigned long long lead = (uint32_t)__builtin_amdgcn_readfirstlane(s.in_lead);
    if (!TAIL && (trip | (E3 & P63) | lead) == 0ull) {
        // every X X pair starts its run, so every valid pair counts
        const int32_t x[4] = {t0, t1, t2, x3}, y[4] = {t1, t2, t3, r3};
        if (MODE == MODE_TABLE || MODE == MODE_FUSED) {
            // one form for every chunk: 11 VALU per pair, both classes (a separate 5-VALU form
            // for chunks of hot tokens only paid off only on a fresh corpus; telling the two
            // apart cost more over a whole run: dropping it timed the C3 run 3 % faster)
            if (PREP) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (SCREEN) {
                        df.o[e] = atomicAdd(lds_word(k, pp.addr[e]), pp.inc[e]);
                        df.a[e] = pp.addr[e];
                    } else {
                        atomicAdd(lds_word(k, pp.addr[e]), pp.inc[e]);
                    }
                }
            } else {
                add_pairs<MODE == MODE_FUSED, SCREEN>(x, y, k, df);
            }
            if (MODE == MODE_FUSED) refresh_pairs<MODE>(k, t0, t1, t2, x3, r3, x, y);
        } else if (MODE == MODE_EXACT) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if ((x[e] | y[e]) >= HOT) count_pair<MODE>(k, x[e], y[e], s.seen);
        } else if (MODE == MODE_INCR) {
            // only the pairs with a side in {ma, mb, mc}: membership masks per slot (compares into
            // lane masks, combined on the scalar unit), the LDS only for chunks that hold one
            const int32_t ma = k.ma, mb = k.mb, mc = k.mc;
            const unsigned long long M0 = member3(t0, ma, mb, mc), M1 = member3(t1, ma, mb, mc),
                                     M2 = member3(t2, ma, mb, mc), M3 = member3(x3, ma, mb, mc),
                                     M4 = member3(r3, ma, mb, mc);
            const unsigned long long Wm[4] = {M0 | M1, M1 | M2, M2 | M3, M3 | M4};
            if ((Wm[0] | Wm[1] | Wm[2] | Wm[3]) != 0ull) {
                // branch-free on the common route (a row counter): every lane adds, 0 when its
                // pair is not touched (to a counter of its own: no two lanes on one address);
                // pairs of mc, and other tokens past the rows, take the hash (rare)
                unsigned long long hsh = 0;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    // a plane with no touched pair adds nothing (its df.o[e] stays 0): 3 % of
                    // the skewed corpus's pass (profiles/r05_ab_zipf_plane_skip.txt)
                    if (Wm[e] == 0ull) continue;
                    const int32_t xx = x[e], yy = y[e];
                    const bool act = lane_in(Wm[e]);
                    const bool xa = xx == ma, xb = xx == mb, ya = yy == ma, yb = yy == mb;
                    const int row = xa ? 0 : xb ? 1 : ya ? 2 : 3;
                    const int idx = (xa | xb) ? yy : xx;
                    // (an unsigned bound: a pair with a negative side (SEP, dead) never has both a
                    // member side and idx >= 0, so it never lands in a row; the rare branch below
                    // drops such pairs from the hash)
                    const bool inrow = act & (xa | xb | ya | yb) & ((uint32_t)idx < (uint32_t)INCR_RLIM);
                    // counter cc = row * INCR_RLIM + idx: byte address of its dword (cc >> 1) * 4,
                    // made as (2 cc) & ~3; its half (cc & 1) = (idx & 1) (INCR_RLIM is even)
                    const uint32_t cc2 = (uint32_t)(row * (2 * INCR_RLIM)) + 2u * (uint32_t)idx;
                    const uint32_t ba = inrow ? (cc2 & ~3u) : 4u * (uint32_t)lane;
                    // (the returns wait for the round's overflow screen; a lane's own dword
                    // `lane` is a row 0 counter, so its return can only raise a false alarm)
                    df.o[e] = atomicAdd(reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(k.hist) + ba),
                                        (uint32_t)inrow << (((uint32_t)idx & 1u) << 4));
                    df.a[e] = ba;
                    hsh |= (unsigned long long)(act & !inrow) << e;
                }
                if (__ballot(hsh != 0ull) != 0ull) {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (((hsh >> e) & 1ull) && (x[e] | y[e]) >= 0)
                            incr_hash_add(k, ((uint32_t)x[e] << 16) | (uint32_t)y[e], 1u);
                }
            }
        }
        // the last token starts its run here (a run continuing into the next chunk would be a run
        // of three, or a partial chunk's X X end), so its offset parity is 0
        s.first_tok = s.n_live ? s.first_tok : w.first;
        s.par = 0;
        s.prev = w.last;
        s.n_live += len;
        return;
    }
    const int full = len == CHUNK;
    // exact path
#ifdef BPE_PROBE_COMMON
    s.in_lead = 0;   // (static instruction-count probe only: drop the exact path)
    return;
#endif
    const int kl = len - 1, ll = kl >> 2, el = kl & 3;
    int32_t rr[4] = {t1, t2, t3, r3};
    if (!full) {
        const bool me = lane_in(1ull << ll);
        switch (el) {
        case 0: rr[0] = sel(me, nxt, rr[0]); break;
        case 1: rr[1] = sel(me, nxt, rr[1]); break;
        case 2: rr[2] = sel(me, nxt, rr[2]); break;
        default: rr[3] = sel(me, nxt, rr[3]); break;
        }
    }
    int par[4];
    bool start[4];
    run_parity(w.t, len, s.prev, s.par, lane, par, start);
    bool cnt[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const bool valid = ((w.t[e] | rr[e]) >= 0) & (4 * lane + e < len);
        cnt[e] = valid & !((w.t[e] == rr[e]) & (par[e] != 0));
    }
    const int par_last = bcast(pick4(par, el), ll);
    if (s.in_lead) {
        // the first run ends at the first run start at region position >= 1
        int f = len;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const unsigned long long m = __ballot(start[e] & ((s.n_live + 4 * lane + e) > 0));
            if (m) {
                const int q = 4 * __builtin_ctzll(m) + e;
                f = q < f ? q : f;
            }
        }
        if (f < len) {
            s.lead_len = s.n_live + f;
            s.in_lead = 0;
        }
        // (MODE_TABLE: kept a scalar; as a select the compiler made it a vector value, read back
        // with a readfirstlane in every chunk's fast-path test: C3 pass 0.7249 -> 0.7207 ms.  The
        // maintained state's pass timed 4 % slower with it; profiles/r05_ab_in_lead.txt)
        if (MODE == MODE_TABLE) s.in_lead = __builtin_amdgcn_readfirstlane(s.in_lead);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
        if (cnt[e]) count_pair<MODE, SCREEN>(k, w.t[e], rr[e], s.seen);
    s.first_tok = s.n_live ? s.first_tok : w.first;
    s.prev = w.last;
    s.par = par_last;
    s.n_live += len;
}

// Apply-side state of one region (wave-uniform).
struct Apply {
    int32_t prev;        // last pre-merge live token before the chunk
    int32_t par;         // its run-offset parity (X X merges only)
    int32_t match;       // it is an `a` matched with the chunk's first live token
    uint32_t n_match;
};

// What a k_step pass does before counting: nothing, a merge of two distinct ids, or an X X merge
// (the only kind whose matches depend on run parity, so the only one carrying that code).
enum MergeKind { NO_MERGE = 0, MERGE_XY = 1, MERGE_XX = 2 };

// Writes the tail tag of a re-packed chunk (slot 255 lives on lane 63).
__device__ __forceinline__ void tag_tail(int32_t (&y)[4], int total, int32_t last) {
    if (total < CHUNK) y[3] = sel(lane_in(1ull << 63), tail_tag(total, last), y[3]);
}

// Applies the merge (a, b) -> c to one pre-merge chunk (w.len > 0) at chunk index c of the region,
// in place: nxt = the first pre-merge live token after it (the next region's first for the last
// chunk).  A touched chunk is re-packed and written back.
template <int MERGE, bool PREP = false>
__device__ __forceinline__ void apply_chunk(Chunk &w, int32_t nxt, int32_t ma, int32_t mb,
                                            int32_t mc,
                                            const __amdgpu_buffer_rsrc_t rs, int c, int lane,
                                            Apply &ap, Prep &pp, uint32_t akey) {
#ifdef BPE_PROBE_NOAPPLY
    if (lane >= 0) {   // (timing probe only: no merge detection or rewrite)
        ap.prev = w.last;
        ap.par = 0;
        ap.match = 0;
        return;
    }
#endif
    // The common case, no (a, b) in the chunk: four packed (slot, right neighbour) compares.  In a
    // partial chunk lane 63's slot 3 (dead) stands in for the last live slot, paired with nxt.
    // (A tail tag can alias a token in its low half; such a false hit only takes the exact path.)
    // (Testing for `a` alone, four compares instead of eight VALU, timed 2 % slower on C3 and zipf
    // C3: a chunk holding `a` without (a, b) then pays the full test; profiles/r05_ab_acheck.txt.)
    {
        unsigned long long H;
        if (PREP) {
            // (the chunk's pair-table slots, made by prep_pairs: a slot equal to the merge's own)
            H = __ballot(pp.addr[0] == akey) | __ballot(pp.addr[1] == akey) |
                __ballot(pp.addr[2] == akey) | __ballot(pp.addr[3] == akey);
        } else {
            const int32_t r3 = from_next(w.t[0], nxt);
            const unsigned long long P63 = (unsigned long long)((int64_t)w.len - CHUNK) & (1ull << 63);
            const int32_t x3 = sel(lane_in(P63), w.last, w.t[3]);
            const uint32_t key = pack_pair_s(ma, mb);
            H = __ballot(pack_pair(w.t[0], w.t[1]) == key) | __ballot(pack_pair(w.t[1], w.t[2]) == key) |
                __ballot(pack_pair(w.t[2], w.t[3]) == key) | __ballot(pack_pair(x3, r3) == key);
        }
        unsigned long long T = H | (unsigned long long)(uint32_t)ap.match;
        // (X X merges also carry the run parity while the chunk ends in `a`)
        if (MERGE == MERGE_XX) T |= (unsigned long long)(uint32_t)(w.last == ma);
        if (T == 0ull) {
            ap.prev = w.last;
            ap.par = 0;
            ap.match = 0;
            return;
        }
    }
    // M[e]: slot e is `a` and its in-register right-hand neighbour is `b`
    const unsigned long long A0 = __ballot(w.t[0] == ma), A1 = __ballot(w.t[1] == ma),
                             A2 = __ballot(w.t[2] == ma), A3 = __ballot(w.t[3] == ma);
    const unsigned long long B0 = __ballot(w.t[0] == mb), B1 = __ballot(w.t[1] == mb),
                             B2 = __ballot(w.t[2] == mb), B3 = __ballot(w.t[3] == mb);
    unsigned long long M0 = A0 & B1, M1 = A1 & B2, M2 = A2 & B3, M3 = A3 & (B0 >> 1);
    // the last live slot's neighbour is nxt
    int m_last = ((uint32_t)(w.last ^ ma) | (uint32_t)(nxt ^ mb)) == 0u;
    int par_last = 0;
    if (MERGE == MERGE_XX) {
        // only even run offsets match (core.ts:285-290 == replaceAll's leftmost rule); the
        // parity is carried only while the chunk ends in `a`
        if (((M0 | M1 | M2 | M3) != 0ull) | (w.last == ma)) {
            const int kl = w.len - 1;
            int par[4];
            bool start[4];
            run_parity(w.t, w.len, ap.prev, ap.par, lane, par, start);
            M0 &= __ballot(par[0] == 0);
            M1 &= __ballot(par[1] == 0);
            M2 &= __ballot(par[2] == 0);
            M3 &= __ballot(par[3] == 0);
            par_last = bcast(pick4(par, kl & 3), kl >> 2);
            m_last &= par_last == 0;
        }
    }
    const int32_t t_last = w.last;
    if (((M0 | M1 | M2 | M3) != 0ull) | ((ap.match | m_last) != 0)) {
#ifdef BPE_PROBE_COMMON
        if (lane < 0) {   // (static instruction-count probe only: drop the rewrite)
#endif
        const int kl = w.len - 1;
        if (m_last) {
            const unsigned long long bit = 1ull << (kl >> 2);
            switch (kl & 3) {
            case 0: M0 |= bit; break;
            case 1: M1 |= bit; break;
            case 2: M2 |= bit; break;
            default: M3 |= bit; break;
            }
        }
        const bool m[4] = {lane_in(M0), lane_in(M1), lane_in(M2), lane_in(M3)};
        const bool up = lane_in((M3 << 1) | (unsigned long long)(ap.match != 0));
        const int l4 = 4 * lane;
        bool keep[4];
        keep[0] = (l4 < w.len) & !up;
        keep[1] = (l4 < w.len - 1) & !m[0];
        keep[2] = (l4 < w.len - 2) & !m[1];
        keep[3] = (l4 < w.len - 3) & !m[2];
        int32_t y[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) y[e] = sel(m[e], mc, w.t[e]);
        const int total = compact_chunk(y, keep, w.len, lane);
        const int32_t last = total ? slot_at(y, total - 1) : NONE;
        w.first = total ? bcast(y[0], 0) : TOMB;
#pragma unroll
        for (int e = 0; e < 4; ++e) w.t[e] = y[e];
        tag_tail(y, total, last);
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(__attribute__((__vector_size__(4 * sizeof(unsigned)))) unsigned,
                               make_uint4((unsigned)y[0], (unsigned)y[1], (unsigned)y[2], (unsigned)y[3])),
            rs, lane * 16, c * (CHUNK * 4), 0);
        ap.n_match += (uint32_t)(__popcll(M0) + __popcll(M1) + __popcll(M2) + __popcll(M3));
        w.len = total;
        w.last = last;
        pp.ok = 0;   // (the count makes the rewritten chunk's slots)
#ifdef BPE_PROBE_COMMON
        }
#endif
    }
    ap.prev = t_last;
    ap.par = par_last;
    ap.match = m_last;
}

// hist: the kernel's static LDS table (so, once inlined, LDS addresses are plain constants with no
// symbol base to add per access)
template <int MERGE, int MODE, bool SCREEN = true, bool SLOTS = true>
__device__ __forceinline__ void step_body(uint32_t *hist, int32_t *__restrict__ ids,
                                          int64_t n_chunks, int64_t cpr, int R,
                                          const RegionCarry *__restrict__ carry, int32_t ma,
                                          int32_t mb, int32_t mc, uint32_t *__restrict__ partials,
                                          unsigned long long *__restrict__ spill, ColdTable ct,
                                          const uint32_t *__restrict__ heavy_g,
                                          RegionSum *__restrict__ sums,
                                          unsigned long long *__restrict__ replaced,
                                          unsigned long long *__restrict__ hot_g = nullptr,
                                          unsigned long long *__restrict__ delta = nullptr) {
    // (MODE_INCR: `spill` holds the rows' spill, 4 * INCR_RLIM u64; hot_g the maintained table;
    // delta: a sharded rank's delta rows, which then take the touched pairs instead of the tables)
    unsigned long long *rspill = spill;
    if (MODE == MODE_TABLE || MODE == MODE_FUSED) {
        // (MODE_FUSED: the LDS hash's keys start EMPTY; one store per dword, so no two threads
        // write the same dword before the barrier)
        uint4 *h4 = reinterpret_cast<uint4 *>(hist);
        for (int i = threadIdx.x; i < HIST_WORDS / 4; i += WG) {
            const bool key = MODE == MODE_FUSED && i >= FH_BASE / 4 && i < (FH_BASE + FH_SLOTS) / 4;
            const uint32_t v = key ? EMPTY : 0u;
            h4[i] = make_uint4(v, v, v, v);
        }
    } else if (MODE == MODE_EXACT) {
        for (int i = threadIdx.x; i < HEAVY_WORDS; i += WG) hist[i] = heavy_g[i];
        for (int i = threadIdx.x; i < LH_SLOTS; i += WG) {
            hist[HEAVY_WORDS + i] = EMPTY;
            hist[HEAVY_WORDS + LH_SLOTS + i] = 0;
        }
    } else if (MODE == MODE_INCR) {
        // the rows' used part (other tokens < min(vocabulary, INCR_RLIM)) and the hash
        const int vl = incr_vlim(mc);
        for (int r = 0; r < 4; ++r)
            for (int i = threadIdx.x; i < vl / 2; i += WG) hist[r * (INCR_RLIM / 2) + i] = 0;
        for (int i = threadIdx.x; i < IH_SLOTS; i += WG) {
            hist[IH_BASE + i] = EMPTY;
            hist[IH_BASE + IH_SLOTS + i] = 0;
        }
    }
    if (MODE != MODE_NONE) __syncthreads();
    Sink k;
    k.hist = hist;
    k.spill = spill;
    k.ct = ct;
    k.heavy = hist;
    k.ma = MODE == MODE_FUSED || MODE == MODE_INCR ? ma : -1;
    k.mb = mb;
    k.mc = mc;
    k.hot = hot_g;
    k.rspill = rspill;
    k.delta = delta;
    k.hot_bytes_v = HOT_BYTES;
    asm volatile("" : "+v"(k.hot_bytes_v));   // (kept in a VGPR for the whole pass)
    const int lane = threadIdx.x & 63;
    const int r = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * WAVES_PER_WG + (threadIdx.x >> 6)));
    if (r < R) {
        const int64_t c0 = (int64_t)r * cpr;
        const int64_t c1 = min(c0 + cpr, n_chunks);
        const int nc = (int)(c1 > c0 ? c1 - c0 : 0);
        const RegionCarry rc = carry[r];
        Tally s;
        s.n_live = 0;
        s.lead_len = 0;
        s.prev = NONE;
        s.par = 0;
        s.first_tok = NONE;
        s.in_lead = 1;
        s.seen = 0;
        Apply ap;
        ap.prev = rc.prev_tok;
        ap.par = (int32_t)(rc.carry_off & 1) ^ 1;   // the token before the region (if linked)
        ap.match = 0;
        ap.n_match = 0;
        // the region through a range-checked buffer descriptor (loads past its end return 0 and
        // are never consumed)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            ids + c0 * CHUNK, 0, nc * CHUNK * 4, 0x00020000);
        const int lo = lane * 16;
        auto load = [&](Chunk &q, int c) __attribute__((always_inline)) {
            const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, lo, c * (CHUNK * 4), BPE_LOAD_AUX);
            q.t[0] = (int)x[0];
            q.t[1] = (int)x[1];
            q.t[2] = (int)x[2];
            q.t[3] = (int)x[3];
        };
        // first pre-merge live token at or after chunk c (whose slot 0 is f0)
        auto live_from = [&](int c, int32_t f0) -> int32_t {
            int32_t v = c < nc ? f0 : rc.next_tok;
            if (__builtin_expect(v < SEP, 0)) {
                // rare: empty chunks; scan their slot 0s
                int q = c + 1;
                for (; q < nc; ++q) {
                    v = __builtin_amdgcn_readfirstlane(
                        (int)__builtin_amdgcn_raw_buffer_load_b32(rs, 0, q * (CHUNK * 4), 0));
                    if (v >= SEP) break;
                }
                if (q >= nc) v = rc.next_tok;
            }
            return v;
        };
        // Ring of RING slots: stage c applies chunk c (cur), counts chunk c-1 (prv) and loads chunk
        // c+RING-3 into the slot of chunk c-3 (fre), which the previous stage freed, so the load
        // can issue at once without its registers overlapping a chunk still in use.  Stage i of a
        // round keeps its count's LDS returns in D[i] until the round's overflow screen.
        Defer D[RING];
        static_for<0, RING>([&](auto i) __attribute__((always_inline)) {
            D[i].o[0] = D[i].o[1] = D[i].o[2] = D[i].o[3] = 0u;
            D[i].a[0] = D[i].a[1] = D[i].a[2] = D[i].a[3] = 0u;
        });
        // The overflow screen of a round (MODE_TABLE / MODE_FUSED / MODE_INCR): every word the
        // wave's adds returned since the last screen; where a half stood at >= 0x4000, a sweep.
        // The fast path's adds kept their addresses: each lane sweeps just the words its adds saw
        // high (sweep_word: an atomic AND, so lanes and waves sweeping one word take its bits
        // once).  The next add to a half that crossed 0x4000 sees it high, and its wave sweeps it
        // at the end of that round: the bound of the whole-table sweep, 0x4000 + the adds of one
        // round of every wave (the static_assert on RING).  The exact path's adds (s.seen) kept
        // no address: the whole table then, as before round 5.  (Early on a skewed corpus a few
        // pairs hold most of a workgroup's counts: every round swept all 40960 words, and a pass
        // took 4 ms instead of 0.6.)
        auto screen_round = [&]() __attribute__((always_inline)) {
            if (MODE != MODE_TABLE && MODE != MODE_FUSED && MODE != MODE_INCR) return;
            if (!SCREEN) return;
            const bool whole = __ballot((s.seen & SWEEP_BITS) != 0u) != 0ull;
            s.seen = 0;
            uint32_t acc = 0;
            static_for<0, RING>([&](auto i) __attribute__((always_inline)) {
                acc |= D[i].o[0] | D[i].o[1] | D[i].o[2] | D[i].o[3];
            });
            if (!whole && __ballot((acc & SWEEP_BITS) != 0u) != 0ull) {
                unsigned long long *sp = MODE == MODE_INCR ? rspill : spill;
                static_for<0, RING>([&](auto i) __attribute__((always_inline)) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) sweep_word(hist, sp, (int)(D[i].a[e] >> 2), D[i].o[e]);
                });
            }
            static_for<0, RING>([&](auto i) __attribute__((always_inline)) {
                D[i].o[0] = D[i].o[1] = D[i].o[2] = D[i].o[3] = 0u;
            });
            if (whole) {
                if (MODE == MODE_INCR) {
                    const int vl = incr_vlim(mc);
                    for (int rw = 0; rw < 4; ++rw)
                        lds_sweep(hist, rspill, lane, rw * (INCR_RLIM / 2),
                                  rw * (INCR_RLIM / 2) + vl / 2);
                } else {
                    lds_sweep(hist, spill, lane, 0, MODE == MODE_FUSED ? HOT_BINS / 2 : HIST_WORDS);
                }
            }
        };
        // pf (MODE_TABLE): slot 0 of the chunk the next stage takes up, read (a lane read, one
        // VALU) by the stage before it for its merge test's right-hand neighbour, and handed on
        // rather than read again when that chunk's own stage begins: C3 pass -0.2 %; the other
        // modes read it again (the maintained state's pass timed 2.6 % slower with the hand-on;
        // profiles/r05_ab_first_handon.txt)
        int32_t pf = 0;
        // MODE_TABLE merge passes: each chunk's pair-table slots made at apply time (Prep), and the
        // merge's own slot, to test against them
        constexpr bool PREP = MODE == MODE_TABLE && MERGE != NO_MERGE && SLOTS;
        uint32_t akey = 0;
        if (PREP) {
            uint32_t a0, i0;
            pair_slot<false>(k, ma, mb, a0, i0);
            akey = (uint32_t)__builtin_amdgcn_readfirstlane((int)a0);
        }
        // (the stage waits for chunk c + 1's load at its start: chunk c's merge test needs its
        // first token.  Loading slot 0 of every chunk on its own a stage earlier, so that a stage
        // waits only for loads issued two stages back, timed the same: profiles/r06_ab_early.txt)
        auto stage = [&](Chunk &cur, const Chunk &nxt_slot, Chunk &prv, Chunk &fre, int c,
                         Defer &df, Prep &pcur, Prep &pprv) __attribute__((always_inline)) {
            load(fre, c + LEAD);
            const int32_t f_next = bcast(nxt_slot.t[0], 0);
            if (c < nc) {
                finish_load(cur, MODE == MODE_TABLE ? pf : bcast(cur.t[0], 0));
            } else {
                // past the region: an empty chunk hands the pending one on (every field stored on
                // both sides, so the stores merge as values, not as a select of addresses)
                cur.first = TOMB;
                cur.len = 0;
                cur.last = NONE;
            }
            if (MERGE && cur.len) {
                const int32_t nx = live_from(c + 1, MODE == MODE_TABLE ? f_next : bcast(nxt_slot.t[0], 0));
                if (PREP) prep_pairs(cur.t, cur.len, cur.last, nx, k, pcur);
                apply_chunk<MERGE, PREP>(cur, nx, ma, mb, mc, rs, c, lane, ap, pcur, akey);
            }
            if (cur.len) {
                if (prv.len) count_chunk<MODE, false, SCREEN, PREP>(prv, cur.first, lane, s, k, df, pprv);
            } else {
                cur = prv;   // rare: hand the pending chunk on
                if (PREP) pcur = pprv;
            }
            // (prv kept live past the hand-on's merge of two register sets, so the register
            // allocator gives the merged chunk cur's registers and puts the copies on the rare
            // path: 7 -> 2 register moves per stage, C3 pass -0.9 %; in the other modes it timed
            // 2 % slower on the skewed corpus; profiles/r05_ab_handon_live.txt)
            if (MODE == MODE_TABLE)
                asm volatile("" ::"v"(prv.t[0]), "v"(prv.t[1]), "v"(prv.t[2]), "v"(prv.t[3]),
                             "s"(prv.last), "s"(prv.first), "s"(prv.len));
            pf = f_next;
        };
        if (nc > 0) {
            Chunk S[RING];   // (constant indices only: the ring stays in registers)
            Prep P[RING];
            static_for<0, RING>([&](auto i) __attribute__((always_inline)) { P[i].ok = 0; });
            static_for<0, LEAD>([&](auto i) __attribute__((always_inline)) { load(S[i], i); });
            S[RING - 1].len = 0;
            pf = bcast(S[0].t[0], 0);
            if (MERGE) {
                // does the token before the region match the region's first live token?
                const int32_t f = live_from(0, pf);
                // (integer arithmetic: a short-circuit && here makes the flag a vector value)
                ap.match = (((uint32_t)(ap.prev ^ ma) | (uint32_t)(f ^ mb)) == 0u) &
                           ((MERGE == MERGE_XY) | (ap.par == 0));
            }
            // whole rounds of RING stages; stages past the region see empty chunks, so the
            // pending chunk always ends in the last slot
            for (int c = 0; c < nc; c += RING) {
                static_for<0, RING>([&](auto I) __attribute__((always_inline)) {
                    constexpr int i = decltype(I)::value;
                    stage(S[i], S[(i + 1) % RING], S[(i + RING - 1) % RING],
                          S[(i + LEAD) % RING], c + i, D[i], P[i], P[(i + RING - 1) % RING]);
                });
                screen_round();
            }
            Defer dt;   // (the region's last chunk takes the exact path: s.seen)
            if (S[RING - 1].len)
                count_chunk<MODE, true, SCREEN>(S[RING - 1], NONE, lane, s, k, dt, P[RING - 1]);
            screen_round();
        }
        if (lane == 0) {
            RegionSum o;
            o.n_live = s.n_live;
            o.first_tok = s.n_live ? s.first_tok : NONE;
            o.last_tok = s.n_live ? s.prev : NONE;
            o.uniform = s.n_live && s.in_lead ? 1 : 0;
            o.lead_len = s.in_lead ? s.n_live : s.lead_len;
            o.trail_odd = s.par ^ 1;   // trail run length = offset of the last token + 1
            sums[r] = o;
            if (MERGE && ap.n_match) atomicAdd(replaced, (unsigned long long)ap.n_match);
        }
    }
    if (MODE == MODE_TABLE || MODE == MODE_FUSED) {
        __syncthreads();
        uint4 *out = reinterpret_cast<uint4 *>(partials + (size_t)blockIdx.x * HIST_WORDS);
        const uint4 *h4 = reinterpret_cast<const uint4 *>(hist);
        for (int i = threadIdx.x; i < HIST_WORDS / 4; i += WG) out[i] = h4[i];
        if (MODE == MODE_FUSED)   // (the slab's sketch dwords are then garbage: unused)
            for (int j = threadIdx.x; j < FH_SLOTS; j += WG) {
                // (each workgroup starts its flush elsewhere: workgroups adding one new key at
                // the same moment each reserve a dense index, and all but one become holes)
                const int i = (j + (int)blockIdx.x * 97 * 64) & (FH_SLOTS - 1);
                const uint32_t key = hist[FH_BASE + i];
                if (key != EMPTY) cold_add(ct, key, hist[FH_BASE + FH_SLOTS + i]);
            }
    } else if (MODE == MODE_INCR) {
        // the rows' used part to this workgroup's slab (k_reduce_rows sums the slabs), the hash's
        // keys straight into the maintained tables
        __syncthreads();
        const int vl = incr_vlim(mc);
        uint32_t *out = partials + (size_t)blockIdx.x * HIST_WORDS;
        for (int r = 0; r < 4; ++r)
            for (int i = threadIdx.x; i < vl / 2; i += WG)
                out[r * (INCR_RLIM / 2) + i] = hist[r * (INCR_RLIM / 2) + i];
        for (int j = threadIdx.x; j < IH_SLOTS; j += WG) {
            const int i = (j + (int)blockIdx.x * 97 * 64) & (IH_SLOTS - 1);
            const uint32_t key = hist[IH_BASE + i];
            if (key != EMPTY)
                incr_global_add(k, (int32_t)(key >> 16), (int32_t)(key & 0xFFFFu),
                                hist[IH_BASE + IH_SLOTS + i]);
        }
    } else if (MODE == MODE_EXACT) {
        __syncthreads();
        for (int j = threadIdx.x; j < LH_SLOTS; j += WG) {
            const int i = (j + (int)blockIdx.x * 97 * 64) & (LH_SLOTS - 1);   // (as above)
            const uint32_t key = hist[HEAVY_WORDS + i];
            if (key != EMPTY) cold_add(ct, key, hist[HEAVY_WORDS + LH_SLOTS + i]);
        }
    }
}

template <int MERGE, int MODE>
__global__ void __launch_bounds__(WG)
k_step(int32_t *__restrict__ ids, int64_t n_chunks, int64_t cpr, int R,
       const RegionCarry *__restrict__ carry, int32_t ma, int32_t mb, int32_t mc,
       uint32_t *__restrict__ partials, unsigned long long *__restrict__ spill, ColdTable ct,
       const uint32_t *__restrict__ heavy_g, RegionSum *__restrict__ sums,
       unsigned long long *__restrict__ replaced, unsigned long long *__restrict__ hot_g = nullptr) {
    __shared__ __attribute__((aligned(16))) uint32_t hist[HIST_WORDS];
    step_body<MERGE, MODE>(hist, ids, n_chunks, cpr, R, carry, ma, mb, mc, partials, spill, ct,
                           heavy_g, sums, replaced, hot_g);
}

// Apply-only pass (restoreMerge replay, batch encoding, core.ts:477-494 / 392-409): the merge is
// applied exactly as by k_step, and the region sums are kept (k_runs<MODE_NONE> turns them into the
// carries of the next pass), but no pair is counted: no LDS table, no slab.
template <int MERGE>
__global__ void __launch_bounds__(WG)
k_apply(int32_t *__restrict__ ids, int64_t n_chunks, int64_t cpr, int R,
        const RegionCarry *__restrict__ carry, int32_t ma, int32_t mb, int32_t mc,
        RegionSum *__restrict__ sums, unsigned long long *__restrict__ replaced) {
    step_body<MERGE, MODE_NONE>(nullptr, ids, n_chunks, cpr, R, carry, ma, mb, mc, nullptr, nullptr,
                                ColdTable{}, nullptr, sums, replaced);
}

// The device loop's pass: the merge to apply is the one k_decide left in the LoopCtl.
// MODE_FUSED: the maintained cold table's refresh rides along (k_cold_invalidate ran before).
template <int MODE = MODE_TABLE>
__global__ void __launch_bounds__(WG)
k_step_loop(int32_t *__restrict__ ids, int64_t n_chunks, int64_t cpr, int R,
            const RegionCarry *__restrict__ carry, const LoopCtl *__restrict__ ctl,
            uint32_t *__restrict__ partials, unsigned long long *__restrict__ spill, ColdTable ct,
            RegionSum *__restrict__ sums, unsigned long long *__restrict__ replaced,
            unsigned long long *__restrict__ hot_g = nullptr,
            unsigned long long *__restrict__ delta = nullptr) {
    __shared__ __attribute__((aligned(16))) uint32_t hist[HIST_WORDS];
    if (ctl->status != LOOP_RUN) return;
    const int32_t ma = ctl->a, mb = ctl->b, mc = ctl->c;
    if (ma == mb)
        step_body<MERGE_XX, MODE>(hist, ids, n_chunks, cpr, R, carry, ma, mb, mc, partials, spill,
                                  ct, nullptr, sums, replaced, hot_g, delta);
    else if (MODE == MODE_TABLE && ctl->unscreened)
        step_body<MERGE_XY, MODE, false>(hist, ids, n_chunks, cpr, R, carry, ma, mb, mc, partials,
                                         spill, ct, nullptr, sums, replaced, hot_g, delta);
    else if (MODE == MODE_TABLE && (int64_t)ctl->w * 16 >= n_chunks)
        // a heavy merge (a skewed corpus's first merges: W in the millions, always screened)
        // rewrites too many chunks for the apply-time slots to pay: the packed-pair test
        step_body<MERGE_XY, MODE, true, false>(hist, ids, n_chunks, cpr, R, carry, ma, mb, mc,
                                               partials, spill, ct, nullptr, sums, replaced, hot_g,
                                               delta);
    else
        step_body<MERGE_XY, MODE>(hist, ids, n_chunks, cpr, R, carry, ma, mb, mc, partials, spill,
                                  ct, nullptr, sums, replaced, hot_g, delta);
}

__device__ __forceinline__ int prev_nonempty(const RegionSum *s, int q) {
    while (q >= 0 && s[q].n_live == 0) --q;
    return q;
}

__device__ __forceinline__ int next_nonempty(const RegionSum *s, int q, int R) {
    while (q < R && s[q].n_live == 0) ++q;
    return q;
}

// Stitches the regions after a pass.  The waves counted every pair inside their region, with the
// X X pairs of each region's first run counted from the region start; here, per region:
//  - the pair straddling its left boundary (unless both sides belong to one run);
//  - for the run that starts in the region and continues into later regions (segments of lengths
//    L_1..L_n, the waves having counted sum floor(L_i / 2)): floor(sum L_i / 2) - sum floor(L_i / 2)
//    = floor(#odd segments / 2) more X X pairs;
//  - the RegionCarry the next pass needs (neighbour tokens, run-offset parity of the first token).
template <int MODE>
__global__ void k_runs(const RegionSum *__restrict__ s, int R, RegionCarry *__restrict__ carry,
                       unsigned long long *__restrict__ spill, ColdTable ct,
                       const uint32_t *__restrict__ heavy, const LoopCtl *ctl, int32_t ma = -1,
                       int32_t mb = -1, int32_t mc = -1, unsigned long long *hot = nullptr,
                       unsigned long long *delta = nullptr) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    // the region and its two neighbours, loaded together before anything else (the loop's state
    // included): one memory latency for the common case, where both neighbours are non-empty and
    // no run crosses a boundary.  (Walking to the neighbours first made a chain of four dependent
    // loads, each a round trip to memory for sums another XCD's L2 wrote: 4.9 us per launch.)
    RegionSum empty;
    empty.n_live = 0;
    empty.lead_len = 0;
    empty.first_tok = NONE;
    empty.last_tok = NONE;
    empty.uniform = 0;
    empty.trail_odd = 0;
    const RegionSum me = s[r];
    const RegionSum sl = r > 0 ? s[r - 1] : empty;
    const RegionSum sr = r + 1 < R ? s[r + 1] : empty;
    if (loop_off(ctl)) return;
    if ((MODE == MODE_FUSED || MODE == MODE_INCR) && ctl) {   // (device loop: the merge applied)
        ma = ctl->a;
        mb = ctl->b;
        mc = ctl->c;
    }
    Sink k;
    k.hist = nullptr;
    k.spill = spill;
    k.ct = ct;
    k.heavy = heavy;
    k.ma = MODE == MODE_FUSED || MODE == MODE_INCR ? ma : -1;
    k.mb = mb;
    k.mc = mc;
    k.hot = hot;
    k.rspill = nullptr;
    k.delta = delta;
    // the nearest non-empty regions before and after (rarely past the immediate neighbours)
    int p = r - 1;
    RegionSum P = sl;
    if (p >= 0 && P.n_live == 0) {
        p = prev_nonempty(s, p - 1);
        P = p >= 0 ? s[p] : empty;
    }
    int nx = r + 1;
    RegionSum N = sr;
    if (nx < R && N.n_live == 0) {
        nx = next_nonempty(s, nx + 1, R);
        N = nx < R ? s[nx] : empty;
    }
    RegionCarry rc;
    rc.prev_tok = p >= 0 ? P.last_tok : SEP;
    rc.next_tok = nx < R ? N.first_tok : SEP;
    rc.carry_off = 0;
    if (me.n_live == 0) {
        carry[r] = rc;
        return;
    }
    const int32_t x0 = me.first_tok;
    const bool linked = p >= 0 && x0 >= 0 && P.last_tok == x0;
    if (linked) {
        // parity of the number of x0 tokens of the run before this region
        int64_t par = 0;
        for (int q = p; q >= 0;) {
            const RegionSum Q = q == p ? P : s[q];
            if (Q.uniform) {
                par ^= Q.n_live & 1;
                const int q2 = prev_nonempty(s, q - 1);
                if (q2 >= 0 && s[q2].last_tok == x0) q = q2;
                else break;
            } else {
                par ^= Q.trail_odd;
                break;
            }
        }
        rc.carry_off = par;
    } else if (p >= 0 && x0 >= 0 && P.last_tok >= 0) {
        add_pairs_global<MODE>(k, P.last_tok, x0, 1);            // the boundary pair
    }
    carry[r] = rc;
    // the run that starts in this region and reaches its end
    if (me.uniform && linked) return;
    const int32_t x = me.uniform ? x0 : me.last_tok;
    if (x < 0) return;
    int64_t odd = me.uniform ? (me.n_live & 1) : me.trail_odd;
    int segs = 1;
    for (int q = nx; q < R;) {
        const RegionSum Q = q == nx ? N : s[q];
        if (Q.first_tok != x) break;
        ++segs;
        if (Q.uniform) {
            odd += Q.n_live & 1;
            q = next_nonempty(s, q + 1, R);
        } else {
            odd += Q.lead_len & 1;
            break;
        }
    }
    if (segs > 1 && odd >= 2) add_pairs_global<MODE>(k, x, x, (unsigned long long)(odd >> 1));
}

// Sums the per-workgroup 16-bit LDS partials and the spill table into the u64 table (hot bins
// [0, 64K), sketch buckets [64K, TABLE_BINS)), zeroes the spill for the next pass, and leaves the
// best hot key (max_length filter applied) in res->best.  A block owns 128 words (256 bins):
// 32 lanes x 4 words, each of its 8 lane groups sums every 8th slab, so each thread keeps 32
// independent uint4 loads in flight instead of walking all G slabs.
constexpr int REDUCE_WORDS_PER_BLOCK = 128;
static_assert(HIST_WORDS % REDUCE_WORDS_PER_BLOCK == 0, "reduce tiling");

__device__ __forceinline__ bool pair_ok(int32_t a, int32_t b, const int32_t *len16,
                                        int64_t max_length);

// A block owns 128 dwords (256 bins): 32 lanes x 4 dwords (512 contiguous bytes of a slab per
// lane group), each of its REDUCE_GROUPS lane groups summing every REDUCE_GROUPS-th slab with up to
// 16 16-B loads in flight.  (Narrower column tiles, reading many slabs per wave-instruction, ran
// 2-3x slower.)  The slabs were just written (MALL-resident): the kernel is latency-bound, so the
// lane groups are many (more waves per CU hiding the loads' latency) rather than few with deep
// chains of loads.
#ifndef BPE_REDUCE_GROUPS
#define BPE_REDUCE_GROUPS 8
#endif
constexpr int REDUCE_GROUPS = BPE_REDUCE_GROUPS;
constexpr int REDUCE_THREADS = 32 * REDUCE_GROUPS;
static_assert(REDUCE_THREADS >= 256 && REDUCE_THREADS <= 1024, "reduce block");
__global__ void __launch_bounds__(REDUCE_THREADS)
k_reduce_table(const uint32_t *__restrict__ partials, int G, unsigned long long *__restrict__ spill,
               unsigned long long *__restrict__ table, const int32_t *__restrict__ len16,
               int64_t max_length, Result *res, const LoopCtl *ctl,
               unsigned long long *__restrict__ hdr = nullptr,
               const unsigned long long *__restrict__ rep = nullptr,
               unsigned long long *__restrict__ bin_max = nullptr) {
    __shared__ uint32_t s_sum[REDUCE_GROUPS][32][8];
    if (loop_off(ctl)) return;
    const int t = threadIdx.x;
    // (sharded: the exchange header carries this shard's replacement count, summed with the table)
    if (hdr && rep && blockIdx.x == 0 && t == 0) hdr[0] = *rep;
    const int wl = t & 31, grp = t >> 5;
    const int w0 = blockIdx.x * REDUCE_WORDS_PER_BLOCK + 4 * wl;   // first of my 4 words
    uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // < 2^24 each: G <= 256 slabs x halves < 2^16
    const uint4 *p4 = reinterpret_cast<const uint4 *>(partials + w0);
    auto add = [&](const uint4 p) {
        acc[0] += p.x & 0xFFFFu;
        acc[1] += p.x >> 16;
        acc[2] += p.y & 0xFFFFu;
        acc[3] += p.y >> 16;
        acc[4] += p.z & 0xFFFFu;
        acc[5] += p.z >> 16;
        acc[6] += p.w & 0xFFFFu;
        acc[7] += p.w >> 16;
    };
    constexpr int RG = REDUCE_GROUPS;
    int g = grp;
    for (; g + 15 * RG < G; g += 16 * RG) {
        uint4 p[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) p[q] = p4[(size_t)(g + RG * q) * (HIST_WORDS / 4)];
#pragma unroll
        for (int q = 0; q < 16; ++q) add(p[q]);
    }
    for (; g + 7 * RG < G; g += 8 * RG) {
        uint4 p[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) p[q] = p4[(size_t)(g + RG * q) * (HIST_WORDS / 4)];
#pragma unroll
        for (int q = 0; q < 8; ++q) add(p[q]);
    }
    for (; g < G; g += RG) add(p4[(size_t)g * (HIST_WORDS / 4)]);
#pragma unroll
    for (int i = 0; i < 8; ++i) s_sum[grp][wl][i] = acc[i];
    __syncthreads();
    // thread t < 256 finalises bin 2*w0' + i for one (word-lane, i) pair: 256 bins
    unsigned long long k = 0, vm = 0;
    if (t < 256) {
        const int bl = t >> 3, bi = t & 7;
        uint32_t sum = 0;
#pragma unroll
        for (int q = 0; q < RG; ++q) sum += s_sum[q][bl][bi];
        // dword w holds bins 2w and 2w + 1 (hot pairs and sketch buckets alike): contiguous writes
        const int bin = blockIdx.x * (2 * REDUCE_WORDS_PER_BLOCK) + t;
        const unsigned long long v = (unsigned long long)sum + spill[bin];
        table[bin] = v;
        spill[bin] = 0;
        if (bin < HOT_BINS && v && pair_ok(bin_a(bin), bin_b(bin), len16, max_length))
            k = pack_key(v, bin_a(bin), bin_b(bin));
        vm = v;
    }
    // one atomic per workgroup (a wave each would queue over a thousand on one address); and the
    // largest bin of all, hot and sketch alike: the next decision's bound, LoopCtl::unscreened
    k = wave_max_u64(k);
    vm = wave_max_u64(vm);
    __shared__ unsigned long long s_best[4], s_vmax[4];
    if ((t & 63) == 0 && t < 256) {
        s_best[t >> 6] = k;
        s_vmax[t >> 6] = vm;
    }
    __syncthreads();
    // (bin_max: where the largest bin goes, res->bin_max by default; a sharded rank's reduce has no
    // Result to select from, but its own largest bin bounds its own next pass alike)
    if (!bin_max && res) bin_max = &res->bin_max;
    if (t == 0 && (res || bin_max)) {
        for (int w = 1; w < 4; ++w) {
            k = s_best[w] > k ? s_best[w] : k;
            vm = s_vmax[w] > vm ? s_vmax[w] : vm;
        }
        if (k && res) atomicMax(&res->best, k);
        if (bin_max) atomicMax(bin_max, vm + 1);
    }
}

// Marks the sketch buckets whose (global) sum reaches the best hot count: only cold pairs there
// can still reach W, so only they need exact counts.  T = max(W_hot, 1).
__global__ void k_heavy(const unsigned long long *__restrict__ table, Result *res,
                        uint32_t *__restrict__ heavy) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;   // one thread per bucket
    const unsigned long long w_hot = res->best >> 17;
    const unsigned long long T = w_hot ? w_hot : 1;
    const bool h = b < SKETCH_BINS && table[HOT_BINS + b] >= T;
    const unsigned long long m = __ballot(h);
    if ((threadIdx.x & 31) == 0 && b < SKETCH_BINS) {
        const uint32_t word = (uint32_t)(m >> (threadIdx.x & 32));
        heavy[b >> 5] = word;
        if (word) atomicAdd(&res->n_heavy, (unsigned)__popc(word));
    }
}

// max_length filter (core.ts:270-273) applied at selection time: it depends only on the pair,
// so excluding a pair here is equivalent to never counting it.
__device__ __forceinline__ bool pair_ok(int32_t a, int32_t b, const int32_t *len16,
                                        int64_t max_length) {
    return !max_length || (int64_t)len16[a] + len16[b] <= max_length;
}

// argmax over the dense hot table: best = max packed key.  One atomic per block of 256 (an atomic
// per wave queued a thousand on one address: 12 us per launch).
__global__ void __launch_bounds__(256)
k_argmax_hot(const unsigned long long *__restrict__ hot_counts, const int32_t *__restrict__ len16,
             int64_t max_length, Result *res, const LoopCtl *ctl = nullptr) {
    __shared__ unsigned long long s_best[4];
    if (loop_off(ctl)) return;
    unsigned long long k = 0;
    for (int bin = blockIdx.x * blockDim.x + threadIdx.x; bin < HOT_BINS;
         bin += gridDim.x * blockDim.x)
        if (pair_ok(bin_a(bin), bin_b(bin), len16, max_length)) {
            const unsigned long long v = pack_key(hot_counts[bin], bin_a(bin), bin_b(bin));
            k = v > k ? v : k;
        }
    k = wave_max_u64(k);
    if ((threadIdx.x & 63) == 0) s_best[threadIdx.x >> 6] = k;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) k = s_best[w] > k ? s_best[w] : k;
        if (k) atomicMax(&res->best, k);
    }
}

// argmax over the claimed cold slots (dense view, coalesced).
// Also counts the claims whose pair is gone (res->cold_dead, zero on entry: a real key whose count a
// merge zeroed and no pass counted again): they stay in the dense view, and every scan streams
// them, until the table is rebuilt.  (Holes, key EMPTY, are claims that lost a race.)
__global__ void k_argmax_cold(ColdTable ct, const int32_t *__restrict__ len16, int64_t max_length,
                              Result *res, const LoopCtl *ctl = nullptr) {
    __shared__ unsigned long long s_best[4];
    __shared__ unsigned s_live;
    if (loop_off(ctl)) return;
    const uint32_t n = cold_used(ct);
    if (blockIdx.x == 0 && threadIdx.x == 0)   // (rides along with the Result's copy to the host)
        res->cold_flags = ((unsigned long long)*ct.overflow << 32) | n;
    if (threadIdx.x == 0) s_live = 0;
    __syncthreads();
    unsigned long long best = 0;
    unsigned dead = 0;
    // COLD_ILP entries per thread and sweep, their loads issued together (one dependent load per
    // thread at a time left the scan latency-bound at about a third of the stream rate)
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += COLD_ILP * stride) {
        unsigned long long v[COLD_ILP];
        uint32_t kk[COLD_ILP];
#pragma unroll
        for (int q = 0; q < COLD_ILP; ++q) {
            const uint32_t i = i0 + q * stride;
            v[q] = i < n ? ct.dcounts[i] : 0ull;
            kk[q] = i < n ? ct.dkeys[i] : EMPTY;
        }
#pragma unroll
        for (int q = 0; q < COLD_ILP; ++q) {
            const unsigned long long n_ab = v[q];
            dead += (n_ab == 0) & (kk[q] != EMPTY);
            const int32_t a = (int32_t)(kk[q] >> 16), b = (int32_t)(kk[q] & 0xFFFFu);
            if (n_ab && pair_ok(a, b, len16, max_length)) {
                const unsigned long long k = pack_key(n_ab, a, b);
                best = k > best ? k : best;
            }
        }
    }
    // one atomic per workgroup (a wave each would queue thousands on one address)
    best = wave_max_u64(best);
    if ((threadIdx.x & 63) == 0) s_best[threadIdx.x >> 6] = best;
    if (dead) atomicAdd(&s_live, dead);
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) best = s_best[w] > best ? s_best[w] : best;
        if (best) atomicMax(&res->best, best);
        if (s_live) atomicAdd(&res->cold_dead, (unsigned long long)s_live);
    }
}

// Last-block detection over a whole grid.  Thread 0 of each block calls it after its block's
// writes and a __threadfence; it returns true in the one block that finishes last.  Same-address
// atomics are serialised by the memory side (a device-wide ticket of 1024 blocks took ~60 us), so
// blocks count in groups of TK_GROUP, one counter per group on its own 128-byte line, and only
// each group's last block takes the top ticket.  Counters are zero between launches (each last
// block resets the counter it completed).
constexpr int TK_STRIDE = 32, TK_GROUP = 32, TK_MAX_GROUPS = 64;
constexpr int TICKET_WORDS = TK_STRIDE * (1 + TK_MAX_GROUPS);
__device__ bool grid_last(unsigned int *ticket) {
    const unsigned G = gridDim.x, g = blockIdx.x / TK_GROUP;
    const unsigned ng = (G + TK_GROUP - 1) / TK_GROUP;
    const unsigned size = min((unsigned)TK_GROUP, G - g * TK_GROUP);
    unsigned int *gc = ticket + TK_STRIDE * (1 + g);
    if (atomicAdd(gc, 1u) != size - 1) return false;
    *gc = 0;
    __threadfence();
    if (atomicAdd(ticket, 1u) != ng - 1) return false;
    *ticket = 0;
    return true;
}

// The maintained state's selection in one launch (the single-corpus device loop; was k_argmax_hot
// + k_argmax_cold + k_collect): the best key over the hot bins and the cold table's dense entries,
// and every pair holding it.  res->best and res->n_cand are zero on entry (k_decide / k_tie_fused
// clear them).  Two forms, the same for every block of the launch:
//  - full (full_req: the first selection of a batch, every SEL_FULL_EVERY-th, and always in
//    MODE_FUSED; launched on the full grid): every dense entry.  Workgroup w takes the CB-entry blocks w, w + G, ...; each
//    thread keeps its best key, its first entry holding it and how many of its entries hold it;
//    each workgroup its best and the entries holding it (a rescan only by the threads with
//    several).  Every block's max is written (ct.bmax), the dirty flags cleared, and the dead
//    claims (count 0, key set) counted: they decide when the table is rebuilt.
//  - incremental: a merge (a, b) -> c changes only the pairs with a side in {a, b, c}.  Those with
//    a or b were zeroed (k_incr_invalidate flagged the blocks whose max they may have been) and
//    recounted to at most their old count; those with c are new claims, at the end of the dense
//    view.  So only the flagged blocks and the blocks of claims made since the last selection are
//    recomputed; the other blocks' maxima are still exact.  The hot bins are scanned in full.
//    (Launched on HOT_BINS / 256 workgroups: zipf C3 recomputes ~24 of ~7700 blocks per merge,
//    so the grid's tickets and the last workgroup's record scan were most of the cost.)
// A ticket picks the last workgroup, which settles the global best from the workgroups' records
// (and, incremental, from the block maxima: the entries of the blocks holding it are the cold
// candidates).  The dead-claim count of the last full scan stands for the incremental ones.
constexpr int SEL_MAX = MAX_CAND + 1;   // (more than MAX_CAND candidates: the host path)
constexpr int SEL_FULL_EVERY = 16;
constexpr uint32_t SEL_MAX_BLOCKS = 1u << 16;   // (more blocks: always the full scan)
struct BlockBest {
    unsigned long long key;
    uint32_t n;
    uint32_t dead;   // the block's dead claims
    int2 cand[SEL_MAX];
};

__device__ __forceinline__ unsigned long long cold_entry_key(const ColdTable &ct, uint32_t i,
                                                             uint32_t n, const int32_t *len16,
                                                             int64_t max_length, int2 &ab,
                                                             unsigned &dead) {
    if (i >= n) return 0;
    const unsigned long long v = ct.dcounts[i];
    const uint32_t kk = ct.dkeys[i];
    dead += (v == 0) & (kk != EMPTY);
    ab = make_int2((int32_t)(kk >> 16), (int32_t)(kk & 0xFFFFu));
    return v && pair_ok(ab.x, ab.y, len16, max_length) ? pack_key(v, ab.x, ab.y) : 0ull;
}

// max over a 256-thread workgroup (s: 4 words of LDS); every thread gets it
__device__ __forceinline__ unsigned long long wg_max_u64(unsigned long long v, unsigned long long *s) {
    v = wave_max_u64(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
    __syncthreads();
    return max(max(s[0], s[1]), max(s[2], s[3]));
}

__global__ void __launch_bounds__(256) k_select_maint(const unsigned long long *__restrict__ hot,
                                                      ColdTable ct, const int32_t *__restrict__ len16,
                                                      int64_t max_length, Result *res, int2 *cand,
                                                      BlockBest *rec, unsigned int *ticket,
                                                      const LoopCtl *ctl, int full_req) {
    __shared__ unsigned long long s_best[4], s_red[4];
    __shared__ unsigned s_dead, s_n;
    __shared__ int2 s_c[SEL_MAX];
    __shared__ bool s_last;
    __shared__ int s_full;
    __shared__ uint32_t s_nl, s_b0, s_b1, s_ncb;
    __shared__ uint32_t s_cb[64];
    if (loop_off(ctl)) return;
    const uint32_t n_cold = cold_used(ct);
    const uint32_t nblk = (n_cold + CB - 1) / CB;
    if (threadIdx.x == 0) {
        // (read once and broadcast: every branch around a barrier below is uniform)
        const uint32_t n0 = *ct.sel_n0;
        s_full = full_req || nblk > SEL_MAX_BLOCKS || n0 > n_cold;
        s_nl = min(*ct.n_blist, ct.mask / CB + 1);
        s_b0 = n0 / CB;              // blocks holding claims made since the last selection
        s_b1 = nblk;
        s_dead = s_n = 0;
    }
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
    if (tid == 0) res->cold_flags = ((unsigned long long)*ct.overflow << 32) | n_cold;
    __syncthreads();
    const bool full = s_full;
    unsigned long long best = 0;
    int2 first = make_int2(-1, -1);
    uint32_t cnt = 0;
    unsigned dead = 0;
    auto see = [&](unsigned long long k, int2 ab) {
        if (k > best) {
            best = k;
            first = ab;
            cnt = 1;
        } else if (k && k == best) {
            ++cnt;
        }
    };
    for (uint32_t bin = tid; bin < (uint32_t)HOT_BINS; bin += stride) {
        const int32_t a = bin_a(bin), b = bin_b(bin);
        if (pair_ok(a, b, len16, max_length)) see(pack_key(hot[bin], a, b), make_int2(a, b));
    }
    // one CB-entry block: every thread its 4 entries (coalesced); the block's max to ct.bmax
    auto block = [&](uint32_t blk, bool keep) {
        unsigned long long m = 0;
#pragma unroll
        for (int q = 0; q < (int)(CB / 256); ++q) {
            int2 ab;
            const unsigned long long k =
                cold_entry_key(ct, blk * CB + threadIdx.x + 256 * q, n_cold, len16, max_length, ab, dead);
            if (keep) see(k, ab);
            m = max(m, k);
        }
        m = wg_max_u64(m, s_red);
        if (threadIdx.x == 0) {
            ct.bmax[blk] = m;
            ct.bdirty[blk] = 0;
        }
    };
    if (full) {
        for (uint32_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) block(blk, true);
    } else {
        // the flagged blocks, then the blocks of the new claims
        const uint32_t nl = s_nl, nn = s_b1 - min(s_b0, s_b1);
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(ct.n_recomputed, nl + nn);
        for (uint32_t j = blockIdx.x; j < nl + nn; j += gridDim.x) {
            // (blist holds blocks of entries below n_used: always < nblk, so every thread of
            // the workgroup calls block() with the same blk)
            block(j < nl ? ct.blist[j] : s_b0 + (j - nl), false);
        }
        dead = 0;
    }
    unsigned long long bb = wave_max_u64(best);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s_best[threadIdx.x >> 6] = bb;
    if (dead) atomicAdd(&s_dead, dead);
    __syncthreads();
    bb = max(max(s_best[0], s_best[1]), max(s_best[2], s_best[3]));
    if (bb && best == bb) {
        if (cnt == 1) {
            const unsigned k = atomicAdd(&s_n, 1u);
            if (k < SEL_MAX) s_c[k] = first;
        } else {
            // (rare: several entries of this thread hold the block's best) the thread's elements again
            for (uint32_t bin = tid; bin < (uint32_t)HOT_BINS; bin += stride) {
                const int32_t a = bin_a(bin), b = bin_b(bin);
                if (pair_ok(a, b, len16, max_length) && pack_key(hot[bin], a, b) == bb) {
                    const unsigned k = atomicAdd(&s_n, 1u);
                    if (k < SEL_MAX) s_c[k] = make_int2(a, b);
                }
            }
            if (full)
                for (uint32_t blk = blockIdx.x; blk < nblk; blk += gridDim.x)
                    for (int q = 0; q < (int)(CB / 256); ++q) {
                        int2 ab;
                        unsigned dd = 0;
                        if (cold_entry_key(ct, blk * CB + threadIdx.x + 256 * q, n_cold, len16,
                                           max_length, ab, dd) == bb) {
                            const unsigned k = atomicAdd(&s_n, 1u);
                            if (k < SEL_MAX) s_c[k] = ab;
                        }
                    }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        BlockBest &r = rec[blockIdx.x];
        r.key = bb;
        r.n = s_n;
        r.dead = s_dead;
        for (unsigned k = 0; k < min(s_n, (unsigned)SEL_MAX); ++k) r.cand[k] = s_c[k];
        __threadfence();
        s_last = grid_last(ticket);
    }
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    // the last block: the global best, the dead claims and the candidates from every block's
    // record, read by all its threads (one thread alone waited on ~1000 dependent loads)
    unsigned long long g = 0, dsum = 0;
    for (unsigned q = threadIdx.x; q < gridDim.x; q += blockDim.x) {
        g = max(g, rec[q].key);
        dsum += rec[q].dead;
    }
    // incremental: the best block max; per thread its best, its first block holding it and how
    // many (16 loads in flight per thread: one at a time left this scan latency-bound)
    unsigned long long gc = 0;
    uint32_t gfirst = 0, gcnt = 0;
    if (!full)
        for (uint32_t b0 = threadIdx.x; b0 < nblk; b0 += 16 * 256) {
            unsigned long long v[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = b0 + 256 * q < nblk ? ct.bmax[b0 + 256 * q] : 0ull;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                if (v[q] > gc) {
                    gc = v[q];
                    gfirst = b0 + 256 * q;
                    gcnt = 1;
                } else if (v[q] && v[q] == gc) {
                    ++gcnt;
                }
            }
        }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) dsum += __shfl_xor(dsum, d);
    __shared__ unsigned long long s_dsum[4];
    if ((threadIdx.x & 63) == 0) s_dsum[threadIdx.x >> 6] = dsum;
    g = wg_max_u64(max(g, gc), s_best);
    if (threadIdx.x == 0) {
        s_n = 0;
        s_ncb = 0;
    }
    __syncthreads();
    if (g)
        for (unsigned q = threadIdx.x; q < gridDim.x; q += blockDim.x) {
            const BlockBest &r = rec[q];
            if (r.key != g) continue;
            const unsigned k0 = atomicAdd(&s_n, r.n);
            for (unsigned k = 0; k < min(r.n, (unsigned)SEL_MAX) && k0 + k < (unsigned)SEL_MAX; ++k)
                cand[k0 + k] = r.cand[k];
        }
    if (!full && g) {
        // the cold blocks holding the best key, then their entries holding it
        if (gc == g && gcnt == 1) {
            const unsigned k = atomicAdd(&s_ncb, 1u);
            if (k < 64) s_cb[k] = gfirst;
        } else if (gc == g) {
            // (rare: several of this thread's blocks hold it) its blocks again
            for (uint32_t blk = threadIdx.x; blk < nblk; blk += blockDim.x)
                if (ct.bmax[blk] == g) {
                    const unsigned k = atomicAdd(&s_ncb, 1u);
                    if (k < 64) s_cb[k] = blk;
                }
        }
        __syncthreads();
        const uint32_t ncb = s_ncb;
        if (ncb > 64) {
            if (threadIdx.x == 0) s_n = SEL_MAX;   // (too many: the host path)
        } else {
            for (uint32_t j = 0; j < ncb; ++j)
#pragma unroll
                for (int q = 0; q < (int)(CB / 256); ++q) {
                    int2 ab;
                    unsigned dd = 0;
                    if (cold_entry_key(ct, s_cb[j] * CB + threadIdx.x + 256 * q, n_cold, len16,
                                       max_length, ab, dd) == g) {
                        const unsigned k = atomicAdd(&s_n, 1u);
                        if (k < SEL_MAX) cand[k] = ab;
                    }
                }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        res->best = g;
        res->n_cand = s_n;
        if (full) *ct.dead = (uint32_t)(s_dsum[0] + s_dsum[1] + s_dsum[2] + s_dsum[3]);
        res->cold_dead = *ct.dead;
        *ct.n_blist = 0;
        *ct.sel_n0 = n_cold;
    }
}

// One workgroup: best hot key (wave + LDS max), the hot pairs sharing it, and the heavy sketch
// buckets (sum >= max(W_hot, 1)).  Replaces three launches and their atomics on the fast path.
__global__ void __launch_bounds__(1024) k_select(const unsigned long long *__restrict__ table,
                                                 const int32_t *__restrict__ len16,
                                                 int64_t max_length, Result *res, int2 *cand,
                                                 uint32_t *__restrict__ heavy) {
    __shared__ unsigned long long s_best[16];
    __shared__ unsigned int s_n, s_heavy;
    const int t = threadIdx.x;
    unsigned long long best = 0;
    for (int bin = t; bin < HOT_BINS; bin += 1024) {
        const int32_t a = bin_a(bin), b = bin_b(bin);
        if (!pair_ok(a, b, len16, max_length)) continue;
        const unsigned long long k = pack_key(table[bin], a, b);
        best = k > best ? k : best;
    }
    best = wave_max_u64(best);
    if ((t & 63) == 0) s_best[t >> 6] = best;
    if (t == 0) s_n = s_heavy = 0;
    __syncthreads();
    best = 0;
    for (int i = 0; i < 16; ++i) best = s_best[i] > best ? s_best[i] : best;
    if (best)
        for (int bin = t; bin < HOT_BINS; bin += 1024) {
            const int32_t a = bin_a(bin), b = bin_b(bin);
            if (pair_ok(a, b, len16, max_length) && pack_key(table[bin], a, b) == best) {
                const unsigned i = atomicAdd(&s_n, 1u);
                if (i < CAND_CAP) cand[i] = make_int2(a, b);
            }
        }
    const unsigned long long w_hot = best >> 17;
    const unsigned long long T = w_hot ? w_hot : 1;
    for (int b0 = 0; b0 < SKETCH_BINS; b0 += 1024) {
        const int b = b0 + t;
        const unsigned long long m = __ballot(table[HOT_BINS + b] >= T);
        if ((t & 31) == 0) {
            const uint32_t word = (uint32_t)(m >> (t & 32));
            heavy[b >> 5] = word;
            if (word) atomicAdd(&s_heavy, (unsigned)__popc(word));
        }
    }
    __syncthreads();
    if (t == 0) {
        res->best = best;
        res->n_cand = s_n;
        res->n_heavy = s_heavy;
    }
}

// Multi-workgroup selection once res->best holds the best hot key (k_reduce_table): every hot
// pair sharing it (unordered: the tie rule does not depend on the order) and the heavy sketch
// buckets (sum >= max(W_hot, 1)).  res->n_cand / n_heavy must be zero on entry.
__global__ void __launch_bounds__(256) k_select_multi(const unsigned long long *__restrict__ table,
                                                      const int32_t *__restrict__ len16,
                                                      int64_t max_length, Result *res, int2 *cand,
                                                      uint32_t *__restrict__ heavy,
                                                      const LoopCtl *ctl) {
    if (loop_off(ctl)) return;
    const int idx = blockIdx.x * 256 + threadIdx.x;   // grid covers TABLE_BINS exactly
    const unsigned long long best = res->best;
    if (idx < HOT_BINS) {
        const int32_t a = bin_a(idx), b = bin_b(idx);
        if (best && pack_key(table[idx], a, b) == best && pair_ok(a, b, len16, max_length)) {
            const unsigned i = atomicAdd(&res->n_cand, 1u);
            if (i < CAND_CAP) cand[i] = make_int2(a, b);
        }
    } else {
        const unsigned long long w_hot = best >> 17;
        const unsigned long long T = w_hot ? w_hot : 1;
        const int bk = idx - HOT_BINS;
        const unsigned long long m = __ballot(table[idx] >= T);
        if ((threadIdx.x & 31) == 0) {
            const uint32_t word = (uint32_t)(m >> (threadIdx.x & 32));
            heavy[bk >> 5] = word;
            if (word) atomicAdd(&res->n_heavy, (unsigned)__popc(word));
        }
    }
}

// The device loop's decision: do_find's selection tail (core.ts:294-318) without leaving the GPU.
// phase 0, after the selection kernels: checks the previous merge's replacement count against its
// W, then ends the batch (no pair or W < min_weight: LOOP_DONE; heavy sketch buckets or more than
// MAX_CAND candidates: LOOP_HOST, the host path takes that iteration), waits for the tie pass
// (several candidates), or decides.  phase 1, after k_tie: the candidate whose last counted
// occurrence is earliest (rule R3).  A decision logs (a, b, W), registers the new token's UTF-16
// length (core.ts:318) and clears the Result for the next pass.  One thread.
//
// With a maintained cold table (ctl->maintained) the selection read that table, not the sketch:
// the batch hands over to the host when the table overflowed, is 3/4 full, is more than half dead
// claims (it is then rebuilt), or when the refresh of the chosen merge might not fit (2 claims
// per replacement at most).
//
// One rank of a sharded corpus (ctl->sharded): the replacement count checked is the SUM over the
// ranks (the exchange header `hdr`, all-reduced with the table or the delta rows).  Phase 0 only
// proposes (ctl->tie: 1 / 2 tie pass in the tail window / over the whole shard, 3 one candidate,
// 4 no merge, 5 the host path) and votes: the reasons above that depend on this rank's copy of the
// maintained tables (fill, dead claims, room) differ between ranks, so they ride in the tie
// all-reduce(MAX) (tie_pos[MAX_CAND]) and phase 1 decides on every rank alike.
// ---- the decision's parts (k_decide, and k_tie_fused's last block) ----
// Room in the maintained table for the refresh of the merge: every pair the merge creates has
// the new token c as a side, and c occurs W times, so it claims at most 2 W new slots.
__device__ __forceinline__ bool decide_room(const LoopCtl &C, const Result &R) {
    if (!C.maintained) return true;
    const long long W = (long long)(R.best >> 17);
    const unsigned long long V = (unsigned long long)C.next_id + 1;
    const unsigned long long claims = 2 * (unsigned long long)W < V * V ? 2 * W : V * V;
    return (R.cold_flags & 0xFFFFFFFFull) + claims + 64 <= C.cold_cap / 4 * 3;
}

// Phase 0's proposal from the snapshots: 4 no merge (LOOP_DONE), 5 the host path, 1 / 2 a tie
// pass over the corpus tail window / the whole corpus, 3 one candidate.  *vote: this corpus's
// own reasons for the host path (a sharded rank votes; one corpus proposes 5).  Sorts
// cand[0 .. n) by (a, b) when tied (the same order on every rank).
__device__ int decide_propose(const LoopCtl &C, const Result &R, int2 *cand, int &vote) {
    const unsigned long long best = R.best;
    const long long W = (long long)(best >> 17);
    const unsigned n = R.n_cand;
    vote = 0;
    if (C.maintained) {
        const unsigned long long used = R.cold_flags & 0xFFFFFFFFull;
        if ((R.cold_flags >> 32) || used * 4 > C.cold_cap * 3 || 2 * R.cold_dead > used + 65536)
            vote = 1;
    }
    if (!decide_room(C, R)) vote = 1;
    if (vote && !C.sharded) return 5;
    // a heavy sketch bucket may hold a cold pair above the best hot one (even when no hot pair
    // exists at all): only the host path's exact counts can tell
    if (!C.maintained && R.n_heavy) return 5;
    if (best == 0 || W < C.min_weight) return 4;                     // core.ts:312-313
    if (n == 0 || n > (unsigned)MAX_CAND || C.next_id >= C.max_id) return 5;
    if (n == 1) return 3;
    for (unsigned j = 1; j < n; ++j) {
        const int2 v = cand[j];
        unsigned i = j;
        for (; i > 0 && (cand[i - 1].x > v.x || (cand[i - 1].x == v.x && cand[i - 1].y > v.y)); --i)
            cand[i] = cand[i - 1];
        cand[i] = v;
    }
    // X Y candidates only: the corpus tail window first (a sharded corpus's tail is the last
    // rank's); else the full pass
    int all_xy = 1;
    for (unsigned j = 0; j < n; ++j) all_xy &= cand[j].x != cand[j].y;
    return all_xy ? 1 : 2;
}

// Rule R3 from the last positions (0: none): the candidate whose last counted occurrence comes
// first.  Tail window (tie == 1): one candidate missing there occurs only earlier, so it wins;
// two or more missing need the host path's full pass.  Returns 0 (a, b set), 1 (host), 2 (no
// occurrence at all: an error).
__device__ int decide_r3(int tie, unsigned n, const unsigned long long *pos, const int2 *cand,
                         int32_t &a, int32_t &b, int &lone) {
    unsigned long long bp = ~0ull;
    unsigned missing = 0;
    a = b = -1;
    lone = 0;
    for (unsigned j = 0; j < n; ++j) {
        const unsigned long long p = pos[j];
        if (p && p < bp) {
            bp = p;
            a = cand[j].x;
            b = cand[j].y;
        }
        missing += p == 0;
    }
    if (tie == 1 && missing) {
        if (missing > 1) return 1;
        for (unsigned j = 0; j < n; ++j)
            if (pos[j] == 0) {
                a = cand[j].x;
                b = cand[j].y;
            }
        lone = 1;
    }
    return a < 0 ? 2 : 0;
}

// The decision's writes: the log entry (a, b, W), the new token's UTF-16 length (core.ts:318),
// the merge the next pass applies, and a Result cleared for the next selection.
__device__ void decide_commit(LoopCtl *ctl, Result *res, const LoopCtl &C, long long W, int32_t a,
                              int32_t b, int32_t *len16, long long *log) {
    const int32_t c = C.next_id;
    len16[c] = len16[a] + len16[b];
    const long long i = C.n_done;
    log[LOG_WORDS * i] = a;
    log[LOG_WORDS * i + 1] = b;
    log[LOG_WORDS * i + 2] = W;
    log[LOG_WORDS * i + 3] = -1;   // (filled in by the next decision or at the batch end)
    ctl->a = a;
    ctl->b = b;
    ctl->c = c;
    ctl->w = W;
    ctl->next_id = c + 1;
    ctl->n_done = i + 1;
    const unsigned long long bm = res->bin_max;
    const int32_t uns = !C.maintained && bm &&
                        (bm - 1) + 2 * (unsigned long long)W < 0x10000ull;
    ctl->unscreened = uns;
    ctl->n_unscreened = C.n_unscreened + uns;
    res->bin_max = 0;
    res->best = 0;
    res->n_cand = 0;
    res->n_heavy = 0;
    res->replaced = 0;
    res->cold_dead = 0;
}

// Phase 0's check of the previous merge's replacement count: == W on the whole corpus (sharded:
// summed over the ranks in the exchange header); this corpus's own count is logged.
__device__ bool decide_check_replaced(LoopCtl *ctl, const LoopCtl &C, const Result &R,
                                      const unsigned long long *hdr, long long *log) {
    if (C.w < 0) return true;
    const unsigned long long total = C.sharded && hdr ? hdr[0] : R.replaced;
    if ((C.sharded && !hdr) || total != (unsigned long long)C.w) {
        ctl->status = LOOP_ERROR;
        ctl->err = 1;
        ctl->err_got = total;
        ctl->err_want = (unsigned long long)C.w;
        return false;
    }
    // (a sharded batch may open on the last batch's last merge: not in this log)
    if (C.n_done > 0) log[LOG_WORDS * (C.n_done - 1) + 3] = (long long)R.replaced;
    return true;
}

__global__ void k_decide(LoopCtl *ctl, Result *res, int2 *__restrict__ cand, int32_t *len16,
                         long long *log, int phase, const unsigned long long *__restrict__ tie_pos,
                         const unsigned long long *__restrict__ hdr = nullptr) {
    if (threadIdx.x != 0) return;
    // Snapshots of the control block and the Result (their loads issue together: one memory
    // latency instead of a chain of dependent ones); the fields are written back one by one.
    const LoopCtl C = *ctl;
    const Result R = *res;
    if (C.status != LOOP_RUN) return;
    const long long W = (long long)(R.best >> 17);
    const unsigned n = R.n_cand;
    auto to_host = [&]() {
        ctl->status = LOOP_HOST;
        ctl->n_host = C.n_host + 1;
    };
    int32_t a = -1, b = -1;
    if (phase == 0) {
        if (!decide_check_replaced(ctl, C, R, hdr, log)) return;
        ctl->w = -1;
        int vote = 0;
        const int prop = decide_propose(C, R, cand, vote);
        if (prop == 1 || prop == 2) {
            for (int j = 0; j < MAX_CAND; ++j) res->last[j] = 0;
            ctl->n_tie = C.n_tie + 1;
        }
        if (C.sharded) {
            ctl->tie = prop;
            ctl->vote = vote;
            ctl->pend_a = cand[0].x;
            ctl->pend_b = cand[0].y;
            return;
        }
        if (prop == 4) {
            ctl->status = LOOP_DONE;
            return;
        }
        if (prop == 5) {
            to_host();
            return;
        }
        if (prop != 3) {
            ctl->tie = prop;
            return;
        }
        a = cand[0].x;
        b = cand[0].y;
    } else {
        if (!C.tie) return;
        if (C.sharded) {
            ctl->tie = 0;
            if (tie_pos[MAX_CAND] || C.tie == 5) {   // some rank voted for the host path
                to_host();
                return;
            }
            if (C.tie == 4) {
                ctl->status = LOOP_DONE;
                return;
            }
        }
        if (C.tie == 3) {
            a = C.pend_a;
            b = C.pend_b;
        } else {
            unsigned long long pos[MAX_CAND];
            for (unsigned j = 0; j < n && j < (unsigned)MAX_CAND; ++j) pos[j] = tie_pos ? tie_pos[j] : R.last[j];
            int lone = 0;
            const int r3 = decide_r3(C.tie, n, pos, cand, a, b, lone);
            if (r3 == 1) {
                to_host();
                return;
            }
            if (lone) ctl->n_lone = C.n_lone + 1;
            if (C.tie == 1) ctl->n_tail = C.n_tail + 1;
            if (r3 == 2) {
                ctl->status = LOOP_ERROR;
                ctl->err = 2;
                return;
            }
            if (!C.sharded && !decide_room(C, R)) {
                to_host();
                return;
            }
        }
        ctl->tie = 0;
    }
    decide_commit(ctl, res, C, W, a, b, len16, log);
}

__device__ __forceinline__ void push_cand(Result *res, int2 *cand, int32_t a, int32_t b) {
    const unsigned int i = atomicAdd(&res->n_cand, 1u);
    if (i < CAND_CAP) cand[i] = make_int2(a, b);
}

// Collects every pair whose packed key equals the best (same W and same a+b).
__global__ void k_collect(const unsigned long long *__restrict__ hot_counts, ColdTable ct,
                          const int32_t *__restrict__ len16, int64_t max_length, Result *res,
                          int2 *cand, const LoopCtl *ctl = nullptr) {
    if (loop_off(ctl)) return;
    const unsigned long long best = res->best;
    if (best == 0) return;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    if (tid < HOT_BINS) {
        const int32_t a = bin_a(tid), b = bin_b(tid);
        if (pair_ok(a, b, len16, max_length) && pack_key(hot_counts[tid], a, b) == best)
            push_cand(res, cand, a, b);
    }
    const uint32_t n = cold_used(ct);
    const unsigned long long w = best >> 17;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i0 = tid; i0 < n; i0 += COLD_ILP * stride) {
        unsigned long long v[COLD_ILP];   // (loads issued together, as in k_argmax_cold)
#pragma unroll
        for (int q = 0; q < COLD_ILP; ++q) {
            const uint32_t i = i0 + q * stride;
            v[q] = i < n ? ct.dcounts[i] : 0ull;
        }
#pragma unroll
        for (int q = 0; q < COLD_ILP; ++q) {
            if (v[q] != w) continue;   // (dense view; the key only for count matches)
            const uint32_t key = ct.dkeys[i0 + q * stride];
            const int32_t a = (int32_t)(key >> 16), b = (int32_t)(key & 0xFFFFu);
            if (pair_ok(a, b, len16, max_length) && pack_key(w, a, b) == best)
                push_cand(res, cand, a, b);
        }
    }
}

// ---- sharded selection over caller-provided (global) tables ----------------------------------
__global__ void k_export_cold(ColdTable ct, uint32_t *keys, unsigned long long *counts) {
    const uint32_t n = cold_used(ct);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        keys[i] = ct.dkeys[i];
        counts[i] = ct.dcounts[i];   // (a hole exports count 0)
    }
}

__global__ void k_argmax_list(const uint32_t *__restrict__ keys,
                              const unsigned long long *__restrict__ counts, int64_t n,
                              const int32_t *__restrict__ len16, int64_t max_length, Result *res) {
    unsigned long long best = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (!counts[i]) continue;   // (holes: count 0, key EMPTY)
        const int32_t a = (int32_t)(keys[i] >> 16), b = (int32_t)(keys[i] & 0xFFFFu);
        if (!pair_ok(a, b, len16, max_length)) continue;
        const unsigned long long k = pack_key(counts[i], a, b);
        best = k > best ? k : best;
    }
    best = wave_max_u64(best);
    if ((threadIdx.x & 63) == 0 && best) atomicMax(&res->best, best);
}

__global__ void k_collect_list(const unsigned long long *__restrict__ hot,
                               const uint32_t *__restrict__ keys,
                               const unsigned long long *__restrict__ counts, int64_t n,
                               const int32_t *__restrict__ len16, int64_t max_length, Result *res,
                               int2 *cand) {
    const unsigned long long best = res->best;
    if (best == 0) return;
    const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (tid < HOT_BINS) {
        const int32_t a = bin_a((uint32_t)tid), b = bin_b((uint32_t)tid);
        if (pair_ok(a, b, len16, max_length) && pack_key(hot[tid], a, b) == best)
            push_cand(res, cand, a, b);
    }
    for (int64_t i = tid; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (counts[i] != (best >> 17)) continue;   // (holes: count 0)
        const int32_t a = (int32_t)(keys[i] >> 16), b = (int32_t)(keys[i] & 0xFFFFu);
        if (pair_ok(a, b, len16, max_length) && pack_key(counts[i], a, b) == best)
            push_cand(res, cand, a, b);
    }
}

// The maintained cold table before its refresh after the merge (a, b) -> c: the pairs with a side
// a or b lose their count (the refresh pass counts them again on the merged corpus; every other
// pair's count is unchanged by the merge).
// (device loop: the merge the next pass applies, from the LoopCtl)
__global__ void k_cold_invalidate(ColdTable ct, int32_t a, int32_t b, const LoopCtl *ctl = nullptr) {
    if (loop_off(ctl)) return;
    if (ctl) {
        a = ctl->a;
        b = ctl->b;
    }
    const uint32_t n = cold_used(ct);
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += COLD_ILP * stride) {
        uint32_t kk[COLD_ILP];   // (loads issued together, as in k_argmax_cold)
#pragma unroll
        for (int q = 0; q < COLD_ILP; ++q) {
            const uint32_t i = i0 + q * stride;
            kk[q] = i < n ? ct.dkeys[i] : EMPTY;
        }
#pragma unroll
        for (int q = 0; q < COLD_ILP; ++q) {
            const int32_t x = (int32_t)(kk[q] >> 16), y = (int32_t)(kk[q] & 0xFFFFu);
            if ((kk[q] != EMPTY) & ((x == a) | (x == b) | (y == a) | (y == b)))
                ct.dcounts[i0 + q * stride] = 0;   // (MODE_FUSED: its selections are full scans)
        }
    }
}


// MODE_INCR before the pass of the merge (a, b) -> c: every pair with a side a or b loses its
// count, in the maintained hot table (rows and columns a, b) and in the cold table.
__global__ void k_incr_invalidate(ColdTable ct, unsigned long long *__restrict__ hot, int32_t a,
                                  int32_t b, const LoopCtl *ctl = nullptr,
                                  const int32_t *__restrict__ len16 = nullptr,
                                  int64_t max_length = 0) {
    if (loop_off(ctl)) return;
    if (ctl) {
        a = ctl->a;
        b = ctl->b;
    }
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < 4 * HOT) {   // hot bin (x, y) = y * 256 + x: column x = a / b, row y = a / b
        const int32_t m = (t >> 8) & 1 ? b : a, o = t & 255;
        if (m < HOT) hot[(t >> 9) ? hot_bin((uint32_t)m, (uint32_t)o) : hot_bin((uint32_t)o, (uint32_t)m)] = 0;
    }
    const uint32_t n = cold_used(ct);
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i0 = t; i0 < n; i0 += COLD_ILP * stride) {
        uint32_t kk[COLD_ILP];
#pragma unroll
        for (int q = 0; q < COLD_ILP; ++q) {
            const uint32_t i = i0 + q * stride;
            kk[q] = i < n ? ct.dkeys[i] : EMPTY;
        }
#pragma unroll
        for (int q = 0; q < COLD_ILP; ++q) {
            const int32_t x = (int32_t)(kk[q] >> 16), y = (int32_t)(kk[q] & 0xFFFFu);
            if ((kk[q] != EMPTY) & ((x == a) | (x == b) | (y == a) | (y == b))) {
                const uint32_t i = i0 + q * stride;
                const unsigned long long old = ct.dcounts[i];
                ct.dcounts[i] = 0;
                // a fall matters to the block maxima only where the entry may have been its
                // block's max (W at least the max's): that block is recomputed before the next
                // selection (the recount after this merge can only give it back less)
                const uint32_t blk = i / CB;
                const unsigned long long ko =
                    old && pair_ok(x, y, len16, max_length) ? pack_key(old, x, y) : 0ull;
                if (ko && ko >= ct.bmax[blk] && atomicExch(&ct.bdirty[blk], 1u) == 0u) {
                    const uint32_t k = atomicAdd(ct.n_blist, 1u);
                    if (k <= ct.mask / CB) ct.blist[k] = blk;
                }
            }
        }
    }
}

// Sharded maintained state, at the start of the next selection: the delta rows summed over the
// ranks (the recount of every pair the last merge (a, b) -> c touched, which k_incr_invalidate
// zeroed before the pass) into this rank's copy of the global tables, and the rows zeroed for the
// next merge.  Each touched pair has exactly one slot (delta_slot), so a hot bin gets one add.
__global__ void __launch_bounds__(256) k_apply_delta(unsigned long long *__restrict__ xchg,
                                                     unsigned long long *__restrict__ hot,
                                                     ColdTable ct, const LoopCtl *ctl) {
    if (loop_off(ctl) || ctl->w < 0) return;   // (w < 0: no merge applied yet in this batch)
    const int32_t a = ctl->a, b = ctl->b, c = ctl->c;
    const uint32_t n = (uint32_t)DELTA_ROWS * (uint32_t)(c + 1);   // other tokens <= c
    unsigned long long *d = xchg + XCHG_HDR;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const unsigned long long v = d[i];
        if (!v) continue;
        d[i] = 0;
        const uint32_t row = i % DELTA_ROWS;
        const int32_t o = (int32_t)(i / DELTA_ROWS);
        const int32_t m = row == 0 || row == 2 ? a : row == 1 || row == 3 ? b : c;
        const bool left = row == 0 || row == 1 || row == 4;   // (m, o), else (o, m)
        const int32_t x = left ? m : o, y = left ? o : m;
        if (((uint32_t)x | (uint32_t)y) < (uint32_t)HOT) hot[hot_bin((uint32_t)x, (uint32_t)y)] += v;
        else cold_add(ct, pair_key(x, y), v);
    }
}

// bpe_set_global_counts: (key, count) entries of every shard, duplicates summed, into the cleared
// cold table (holes, key EMPTY or count 0, skipped).
// The live claims of the cold table (a key, a count > 0) into dense arrays, in any order: the
// maintained table rebuilt from itself (bpe_engine.hip cold_rebuild) instead of from the corpus.
// (A wave-uniform loop: one atomic per wave for the output slots.)
__global__ void __launch_bounds__(256) k_cold_gather(ColdTable ct, uint32_t *__restrict__ keys,
                                                     unsigned long long *__restrict__ counts,
                                                     uint32_t *__restrict__ n_out) {
    const uint32_t n = cold_used(ct), lane = threadIdx.x & 63;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i0 = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); i0 < n; i0 += stride) {
        const uint32_t i = i0 + lane;
        uint32_t k = EMPTY;
        unsigned long long v = 0;
        if (i < n) {
            k = ct.dkeys[i];
            v = ct.dcounts[i];
        }
        const bool live = k != EMPTY && v != 0ull;
        const unsigned long long m = __ballot(live);
        if (!m) continue;
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(n_out, (uint32_t)__popcll(m));
        b = __shfl(b, 0);
        if (live) {
            const uint32_t j = b + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            keys[j] = k;
            counts[j] = v;
        }
    }
}

__global__ void k_load_cold(ColdTable ct, const uint32_t *__restrict__ keys,
                            const unsigned long long *__restrict__ counts, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        if (counts[i] && keys[i] != EMPTY) cold_add(ct, keys[i], counts[i]);
}

// MODE_INCR after the pass: sums the G slabs' rows (+ their spill, zeroed here) and adds each
// nonzero count to its pair in the maintained tables.  A block owns 32 row dwords (64 counters):
// its 8 lane groups each sum every 8th slab, eight loads in flight, then combine in LDS.
constexpr int RR_COLS = 32;
__global__ void __launch_bounds__(256)
k_reduce_rows(const uint32_t *__restrict__ partials, int G, unsigned long long *__restrict__ rspill,
              unsigned long long *__restrict__ hot, ColdTable ct, int32_t a, int32_t b, int32_t c,
              const LoopCtl *ctl = nullptr, unsigned long long *__restrict__ delta = nullptr,
              const unsigned long long *__restrict__ rep = nullptr) {
    __shared__ uint32_t s_lo[8][RR_COLS], s_hi[8][RR_COLS];
    if (loop_off(ctl)) return;
    if (ctl) {
        a = ctl->a;
        b = ctl->b;
        c = ctl->c;
    }
    // (sharded: the exchange header carries this shard's replacement count, summed with the rows)
    if (delta && rep && blockIdx.x == 0 && threadIdx.x == 0) delta[0] = *rep;
    const int vl = incr_vlim(c);
    const int d0 = blockIdx.x * RR_COLS;   // first of the block's dwords (4 rows x INCR_RLIM / 2)
    const int row = d0 / (INCR_RLIM / 2);
    if (row >= 4 || 2 * (d0 % (INCR_RLIM / 2)) >= vl || (a == b && (row & 1))) return;
    const int col = threadIdx.x & (RR_COLS - 1), grp = threadIdx.x / RR_COLS;
    uint32_t lo = 0, hi = 0;
    const uint32_t *p = partials + d0 + col;
    int g = grp;
    for (; g + 56 < G; g += 64) {
        uint32_t v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = p[(size_t)(g + 8 * q) * HIST_WORDS];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            lo += v[q] & 0xFFFFu;
            hi += v[q] >> 16;
        }
    }
    for (; g < G; g += 8) {
        const uint32_t v = p[(size_t)g * HIST_WORDS];
        lo += v & 0xFFFFu;
        hi += v >> 16;
    }
    s_lo[grp][col] = lo;
    s_hi[grp][col] = hi;
    __syncthreads();
    if (grp != 0) return;
    for (int q = 1; q < 8; ++q) {
        lo += s_lo[q][col];
        hi += s_hi[q][col];
    }
    const int wi = (d0 + col) % (INCR_RLIM / 2);
    if (2 * wi >= vl) return;
    const int32_t m = (row & 1) ? b : a;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int idx = 2 * wi + h;
        const uint32_t ci = (uint32_t)(row * INCR_RLIM + idx);
        const unsigned long long n = (unsigned long long)(h ? hi : lo) + rspill[ci];
        rspill[ci] = 0;
        if (!n) continue;
        const int32_t x = row < 2 ? m : idx, y = row < 2 ? idx : m;
        Sink k;
        k.hot = hot;
        k.ct = ct;
        k.delta = delta;
        k.ma = a;
        k.mb = b;
        k.mc = c;
        incr_global_add(k, x, y, n);
    }
}

// ---------------------------------------------------------------------------------------------
// K3 tie pass (rule R3): last counted occurrence (slot + 1) of up to MAX_CAND tied pairs on the
// current corpus, with exact X X parity (carry from k_runs).  Same streaming structure as k_step:
// a 6-slot register ring, each chunk checked once the next chunk's first token (its last slot's
// right-hand neighbour) has arrived.  Per chunk and candidate: four compares of a packed
// (token, right neighbour) word; the positions are worked out only in chunks that match.
// ---------------------------------------------------------------------------------------------
struct TieArgs {
    const int32_t *ids;
    int64_t n_chunks, cpr;
    int R;
    int n_cand;                  // host-driven passes (the device loop reads res->n_cand)
    const RegionCarry *carry;
    const int2 *cand;            // the candidates (a, b), at most MAX_CAND
    Result *res;
    const LoopCtl *ctl;          // device loop: run only when ctl->tie is set
};

struct TieState {
    int32_t prev;     // last live token before the chunk
    int32_t par;      // its run-offset parity (valid when it is an X X candidate's token)
    int32_t n;        // candidates
    uint32_t xx;      // bit j: candidate j is an X X pair
    uint32_t key[MAX_CAND];   // candidate j as a packed (a, b) word (wave-uniform registers)
    int32_t pos[MAX_CAND];    // region slot + 1 of the last counted occurrence (0: none)
};

// Checks one chunk (w.len > 0) at chunk index c of the region; nxt = the first live token after it.
// Every candidate costs four compares per chunk (the loops are unrolled, so keys and positions
// stay in registers); only chunks that hold a candidate work out positions.
__device__ __forceinline__ void tie_chunk(const Chunk &w, int32_t nxt, int c, int lane,
                                          TieState &ts) {
    const int32_t r3 = from_next(w.t[0], nxt);
    const uint32_t k0 = pack_pair(w.t[0], w.t[1]), k1 = pack_pair(w.t[1], w.t[2]),
                   k2 = pack_pair(w.t[2], w.t[3]), k3 = pack_pair(w.t[3], r3);
    const uint32_t kl_key = pack_pair_s(w.last, nxt);   // the last live slot's pair
    const int kl = w.len - 1;
    uint32_t hit = 0;
#pragma unroll
    for (int j = 0; j < MAX_CAND; ++j) {
        if (j < ts.n) {
            const uint32_t key = ts.key[j];
            const unsigned long long m = __ballot(k0 == key) | __ballot(k1 == key) |
                                         __ballot(k2 == key) | __ballot(k3 == key);
            hit |= (uint32_t)((m != 0ull) | (kl_key == key)) << j;
        }
    }
    int par[4] = {0, 0, 0, 0};
    int have_par = 0;
    if (hit) {
        // rare: the chunk holds a candidate.  Partial chunks keep the pairs whose right-hand slot
        // is live (slot < kl) and add the last slot's pair; X X candidates keep even run offsets.
        const int part = w.len < CHUNK;
        const unsigned long long L0 = part ? lanes_upto(kl, 0) : ~0ull,
                                 L1 = part ? lanes_upto(kl, 1) : ~0ull,
                                 L2 = part ? lanes_upto(kl, 2) : ~0ull,
                                 L3 = part ? lanes_upto(kl, 3) : ~0ull;
        unsigned long long Q0 = ~0ull, Q1 = ~0ull, Q2 = ~0ull, Q3 = ~0ull;
        if (hit & ts.xx) {
            bool start[4];
            run_parity(w.t, w.len, ts.prev, ts.par, lane, par, start);
            have_par = 1;
            Q0 = __ballot(par[0] == 0);
            Q1 = __ballot(par[1] == 0);
            Q2 = __ballot(par[2] == 0);
            Q3 = __ballot(par[3] == 0);
        }
        const unsigned long long bit = 1ull << (kl >> 2);
#pragma unroll
        for (int j = 0; j < MAX_CAND; ++j) {
            if ((hit >> j) & 1u) {
                const uint32_t key = ts.key[j];
                unsigned long long M0 = __ballot(k0 == key) & L0, M1 = __ballot(k1 == key) & L1,
                                   M2 = __ballot(k2 == key) & L2, M3 = __ballot(k3 == key) & L3;
                if (part & (kl_key == key)) {
                    switch (kl & 3) {
                    case 0: M0 |= bit; break;
                    case 1: M1 |= bit; break;
                    case 2: M2 |= bit; break;
                    default: M3 |= bit; break;
                    }
                }
                if ((ts.xx >> j) & 1u) {
                    // X X: only even run offsets count (core.ts:285-290)
                    M0 &= Q0;
                    M1 &= Q1;
                    M2 &= Q2;
                    M3 &= Q3;
                }
                // highest matching slot of the chunk
                int best = -1;
                if (M0) best = max(best, 4 * (63 - __builtin_clzll(M0)) + 0);
                if (M1) best = max(best, 4 * (63 - __builtin_clzll(M1)) + 1);
                if (M2) best = max(best, 4 * (63 - __builtin_clzll(M2)) + 2);
                if (M3) best = max(best, 4 * (63 - __builtin_clzll(M3)) + 3);
                ts.pos[j] = best >= 0 ? c * CHUNK + best + 1 : ts.pos[j];
            }
        }
    }
    // the parity of the last token matters only while it continues an X X candidate's run
    int par_last = 0;
    if (ts.xx) {
        uint32_t need = 0;
#pragma unroll
        for (int j = 0; j < MAX_CAND; ++j)
            need |= (uint32_t)((ts.key[j] >> 16) == (uint32_t)w.last) << j;
        if (need & ts.xx) {
            if (!have_par) {
                bool start[4];
                run_parity(w.t, w.len, ts.prev, ts.par, lane, par, start);
            }
            par_last = bcast(pick4(par, kl & 3), kl >> 2);
        }
    }
    ts.prev = w.last;
    ts.par = par_last;
}

// Tail mode of the tie pass (device loop, no X X candidate): the last TIE_TAIL_CHUNKS chunks, two
// per wave, each chunk on its own (an X Y pair needs no run context, only the next live token).
// The last occurrence of a candidate found there is its last occurrence in the corpus; a candidate
// not found there occurs only earlier, so it wins if it is the only one missing (k_decide).
constexpr int TIE_TAIL_PER_WAVE = 2;

// One wave's share of the tie pass: n candidates cand[0 .. n) (any memory), over the corpus tail
// window (tail) or the wave's region; the last positions go to A.res->last[j] (atomicMax).
__device__ __forceinline__ void tie_body(const TieArgs &A, int n, int tail, const int2 *cand) {
    const int lane = threadIdx.x & 63;
    const int r = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    TieState ts;
    ts.n = min(n, MAX_CAND);
    ts.xx = 0;
#pragma unroll
    for (int j = 0; j < MAX_CAND; ++j) {
        ts.pos[j] = 0;
        // unused slots get a key no chunk word has (slot values >= 0xFF01 in both halves)
        const int2 cj = j < ts.n ? cand[j] : make_int2(-1, -1);
        ts.key[j] = __builtin_amdgcn_readfirstlane(pack_pair_s(cj.x, cj.y));
        ts.xx |= (uint32_t)((j < ts.n) & (cj.x == cj.y)) << j;
    }
    ts.xx = __builtin_amdgcn_readfirstlane(ts.xx);
    if (tail) {
        const int64_t win = (int64_t)gridDim.x * 4 * TIE_TAIL_PER_WAVE;
        const int64_t cw = max((int64_t)0, A.n_chunks - win) + (int64_t)r * TIE_TAIL_PER_WAVE;
        if (cw >= A.n_chunks) return;
        ts.prev = NONE;
        ts.par = 0;
        const int4 *v4 = reinterpret_cast<const int4 *>(A.ids);
        for (int q = 0; q < TIE_TAIL_PER_WAVE; ++q) {
            const int64_t c = cw + q;
            if (c >= A.n_chunks) break;
            const int4 v = v4[c * 64 + lane];
            Chunk w;
            w.t[0] = v.x;
            w.t[1] = v.y;
            w.t[2] = v.z;
            w.t[3] = v.w;
            finish_load(w);
            if (w.len == 0) continue;
            // the first live token after the chunk (SEP past the corpus end)
            int32_t nxt = SEP;
            for (int64_t q2 = c + 1; q2 < A.n_chunks; ++q2) {
                const int32_t f = __builtin_amdgcn_readfirstlane(A.ids[q2 * CHUNK]);
                if (f >= SEP) {
                    nxt = f;
                    break;
                }
            }
            tie_chunk(w, nxt, q, lane, ts);
        }
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < MAX_CAND; ++j)
                if (j < ts.n && ts.pos[j])
                    atomicMax(&A.res->last[j], (unsigned long long)(cw * CHUNK + ts.pos[j]));
        }
        return;
    }
    if (r >= A.R) return;
    const int64_t c0 = (int64_t)r * A.cpr;
    const int64_t c1 = min(c0 + A.cpr, A.n_chunks);
    const int nc = (int)(c1 > c0 ? c1 - c0 : 0);
    if (nc == 0) return;
    const RegionCarry rc = A.carry[r];
    ts.prev = rc.prev_tok;
    ts.par = (int32_t)(rc.carry_off & 1) ^ 1;   // the token before the region (if linked)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int32_t *>(A.ids) + c0 * CHUNK, 0, nc * CHUNK * 4, 0x00020000);
    const int lo = lane * 16;
    auto load = [&](Chunk &q, int c) __attribute__((always_inline)) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, lo, c * (CHUNK * 4), BPE_LOAD_AUX);
        q.t[0] = (int)x[0];
        q.t[1] = (int)x[1];
        q.t[2] = (int)x[2];
        q.t[3] = (int)x[3];
    };
    int pc = 0;   // chunk index of the pending chunk
    // the ring of k_step: chunk c+RING-2 loads into the slot chunk c-2 freed
    auto stage = [&](Chunk &cur, Chunk &prv, Chunk &fre, int c) __attribute__((always_inline)) {
        load(fre, c + RING - 2);
        if (c < nc) {
            finish_load(cur);
        } else {
            cur.first = TOMB;
            cur.len = 0;
            cur.last = NONE;
        }
        if (cur.len) {
            if (prv.len) tie_chunk(prv, cur.first, pc, lane, ts);
            pc = c;
        } else {
            cur = prv;   // rare: hand the pending chunk on
        }
    };
    Chunk S[RING];
    static_for<0, RING - 2>([&](auto i) __attribute__((always_inline)) { load(S[i], i); });
    S[RING - 1].len = 0;
    for (int c = 0; c < nc; c += RING) {
        static_for<0, RING>([&](auto I) __attribute__((always_inline)) {
            constexpr int i = decltype(I)::value;
            stage(S[i], S[(i + RING - 1) % RING], S[(i + RING - 2) % RING], c + i);
        });
    }
    if (S[RING - 1].len) tie_chunk(S[RING - 1], rc.next_tok, pc, lane, ts);
    if (lane == 0) {
#pragma unroll
        for (int j = 0; j < MAX_CAND; ++j)
            if (j < ts.n && ts.pos[j])
                atomicMax(&A.res->last[j], (unsigned long long)(c0 * CHUNK + ts.pos[j]));
    }
}

__global__ void __launch_bounds__(256) k_tie(TieArgs A) {
    int n = A.n_cand;
    int tail = 0;
    if (A.ctl) {
        const int tie = A.ctl->tie;
        if (A.ctl->status != LOOP_RUN || (tie != 1 && tie != 2)) return;
        n = (int)A.res->n_cand;
        tail = tie == 1;
        // (a sharded corpus's tail window lies on the last rank: the others find nothing there)
        if (tail && A.ctl->sharded && !A.ctl->last_rank) return;
    }
    tie_body(A, n, tail, A.cand);
}

// The single-corpus device loop's selection tail in one launch (k_decide phase 0, k_tie, k_decide
// phase 1).  Without a tie, block 0 decides alone and the other blocks return at once: a
// device-wide ticket costs one same-address atomic per block, which the memory side serialises
// (1024 of them took 62 us, an iteration's whole selection budget).  With a tie (2 to MAX_CAND
// candidates and an R3 proposal), every block takes the same proposal from the same snapshot of
// the control block, the Result and the candidates (nothing writes them until every block has
// taken its ticket), scans for rule R3, and the last block to finish (the ticket) commits the
// decision with the positions every block left.  `ticket` is zero between launches.
__device__ void fused_commit(const TieArgs &A, const LoopCtl &C, const Result &R, const int2 *sc,
                             int prop, int32_t *len16, long long *log) {
    LoopCtl *ctl = const_cast<LoopCtl *>(A.ctl);
    Result *res = A.res;
    if (!decide_check_replaced(ctl, C, R, nullptr, log)) return;
    ctl->w = -1;
    if (prop == 4) {
        ctl->status = LOOP_DONE;
        return;
    }
    if (prop == 5) {
        ctl->status = LOOP_HOST;
        ctl->n_host = C.n_host + 1;
        return;
    }
    int32_t a = sc[0].x, b = sc[0].y;
    if (prop != 3) {
        const unsigned n = R.n_cand;
        unsigned long long pos[MAX_CAND];
        for (unsigned j = 0; j < n; ++j) {
            pos[j] = __hip_atomic_load(&res->last[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            res->last[j] = 0;   // (for the next tie)
        }
        ctl->n_tie = C.n_tie + 1;
        int lone = 0;
        const int r3 = decide_r3(prop, n, pos, sc, a, b, lone);
        if (r3 == 1) {
            ctl->status = LOOP_HOST;
            ctl->n_host = C.n_host + 1;
            return;
        }
        if (lone) ctl->n_lone = C.n_lone + 1;
        if (prop == 1) ctl->n_tail = C.n_tail + 1;
        if (r3 == 2) {
            ctl->status = LOOP_ERROR;
            ctl->err = 2;
            return;
        }
    }
    decide_commit(ctl, res, C, (long long)(R.best >> 17), a, b, len16, log);
}

__global__ void __launch_bounds__(256) k_tie_fused(TieArgs A, int32_t *len16, long long *log,
                                                   unsigned int *ticket) {
    __shared__ LoopCtl sC;
    __shared__ Result sR;
    __shared__ int2 sc[MAX_CAND];
    __shared__ int s_prop;
    __shared__ bool s_last;
    if (threadIdx.x == 0) {
        int prop = 0;
        // (blocks other than 0 look further only when a tie pass is possible; a late block that
        // finds block 0's decision already made returns here too: the status or n_cand changed)
        const unsigned nc = blockIdx.x ? __hip_atomic_load(&A.res->n_cand, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT) : 2u;
        if (nc >= 2 && nc <= (unsigned)MAX_CAND) {
            sC = *A.ctl;
            sR = *A.res;
            const unsigned n = min(sR.n_cand, (unsigned)MAX_CAND);
            for (unsigned j = 0; j < n; ++j) sc[j] = A.cand[j];
            int vote = 0;
            prop = sC.status == LOOP_RUN ? decide_propose(sC, sR, sc, vote) : 0;
            if (blockIdx.x && prop != 1 && prop != 2) prop = 0;
        }
        s_prop = prop;
    }
    __syncthreads();
    const int prop = s_prop;
    if (prop == 0) return;   // (the batch has ended, or block 0 decides alone)
    if (prop != 1 && prop != 2) {
        if (threadIdx.x == 0) fused_commit(A, sC, sR, sc, prop, len16, log);   // (block 0 only)
        return;
    }
    tie_body(A, (int)sR.n_cand, prop == 1, sc);
    // (every wave's position atomics complete at agent scope before the block takes its ticket)
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) s_last = grid_last(ticket);
    __syncthreads();
    if (!s_last || threadIdx.x != 0) return;
    __threadfence();
    fused_commit(A, sC, sR, sc, prop, len16, log);
}

// Sharded loop: this shard's last tie positions as corpus-wide ones (rank << 40 | position; 0:
// none), and this rank's vote for the host path at [MAX_CAND], for the all-reduce(MAX) that
// follows.  One thread per slot.
constexpr int RANK_SHIFT = 40;
constexpr int TIE_WORDS = 32;   // include/bpe.h BPE_TIE_WORDS
static_assert(TIE_WORDS > MAX_CAND, "tie exchange: positions + vote");
__global__ void k_tie_export(const LoopCtl *ctl, const Result *res, unsigned long long *tie_pos,
                             int rank) {
    const int j = threadIdx.x;
    if (j >= TIE_WORDS) return;
    const bool run = ctl->status == LOOP_RUN;
    const int tie = ctl->tie;
    unsigned long long v = 0;
    if (j < MAX_CAND) {
        if (run && (tie == 1 || tie == 2) && res->last[j])
            v = ((unsigned long long)rank << RANK_SHIFT) | res->last[j];
    } else if (j == MAX_CAND) {
        v = run && ctl->vote ? 1 : 0;
    }
    tie_pos[j] = v;
}

// ---------------------------------------------------------------------------------------------
// Compaction (rare): moves every region's live slots to a dense prefix of a fresh buffer.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) k_scan_live(const RegionSum *__restrict__ s, int R,
                                                    int64_t *__restrict__ out_off,
                                                    unsigned long long *total) {
    __shared__ int64_t part[1024];
    const int per = (R + 1023) / 1024;
    const int t = threadIdx.x;
    int64_t acc = 0;
    for (int i = 0; i < per; ++i) {
        const int r = t * per + i;
        if (r < R) acc += s[r].n_live;
    }
    part[t] = acc;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        int64_t o = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += o;
        __syncthreads();
    }
    int64_t run = part[t] - acc;
    for (int i = 0; i < per; ++i) {
        const int r = t * per + i;
        if (r < R) {
            out_off[r] = run;
            run += s[r].n_live;
        }
    }
    if (t == 1023) *total = (unsigned long long)part[1023];
}

__global__ void __launch_bounds__(256) k_compact(const int32_t *__restrict__ ids, int64_t n_chunks,
                                                 int64_t cpr, int R,
                                                 const int64_t *__restrict__ out_off,
                                                 int32_t *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    const int64_t c0 = (int64_t)r * cpr;
    const int64_t c1 = min(c0 + cpr, n_chunks);
    const int4 *v4 = reinterpret_cast<const int4 *>(ids);
    int64_t o = out_off[r];
    for (int64_t c = c0; c < c1; ++c) {
        const View w = make_view(v4[c * 64 + lane]);
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (4 * lane + e < w.len) out[o + 4 * lane + e] = w.t[e];
        o += w.len;
    }
}

// ---------------------------------------------------------------------------------------------
// Sample index: where every sample ends, for reading back single samples (the rows a merge
// changed, db/core.ts:399-417).  One wave per region, as k_compact.  k_census counts a region's
// live tokens and sample terminators, k_scan_pair turns both into region offsets, and k_sep_emit
// writes, per terminator in corpus order, its slot and the live tokens before it.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t wave_sum64(int64_t v) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) v += __shfl_xor(v, d);
    return v;
}

__global__ void __launch_bounds__(256) k_census(const int32_t *__restrict__ ids, int64_t n_chunks,
                                                int64_t cpr, int R, int64_t *__restrict__ live,
                                                int64_t *__restrict__ seps) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    const int64_t c0 = (int64_t)r * cpr;
    const int64_t c1 = min(c0 + cpr, n_chunks);
    const int4 *v4 = reinterpret_cast<const int4 *>(ids);
    int64_t nl = 0, ns = 0;
    for (int64_t c = c0; c < c1; ++c) {
        const View w = make_view(v4[c * 64 + lane]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const bool in = 4 * lane + e < w.len;
            nl += in && w.t[e] >= 0;
            ns += in && w.t[e] == SEP;
        }
    }
    nl = wave_sum64(nl);
    ns = wave_sum64(ns);
    if (lane == 0) {
        live[r] = nl;
        seps[r] = ns;
    }
}

// Exclusive prefix sums of two arrays of R <= 1024 * k entries, in place.  One block of 1024.
__global__ void __launch_bounds__(1024) k_scan_pair(int R, int64_t *__restrict__ a,
                                                    int64_t *__restrict__ b) {
    __shared__ int64_t pa[1024], pb[1024];
    const int per = (R + 1023) / 1024;
    const int t = threadIdx.x;
    int64_t sa = 0, sb = 0;
    for (int i = 0; i < per; ++i) {
        const int r = t * per + i;
        if (r < R) {
            sa += a[r];
            sb += b[r];
        }
    }
    pa[t] = sa;
    pb[t] = sb;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const int64_t oa = t >= d ? pa[t - d] : 0, ob = t >= d ? pb[t - d] : 0;
        __syncthreads();
        pa[t] += oa;
        pb[t] += ob;
        __syncthreads();
    }
    int64_t ra = pa[t] - sa, rb = pb[t] - sb;
    for (int i = 0; i < per; ++i) {
        const int r = t * per + i;
        if (r < R) {
            const int64_t va = a[r], vb = b[r];
            a[r] = ra;
            b[r] = rb;
            ra += va;
            rb += vb;
        }
    }
}

__global__ void __launch_bounds__(256) k_sep_emit(const int32_t *__restrict__ ids, int64_t n_chunks,
                                                  int64_t cpr, int R,
                                                  const int64_t *__restrict__ live_pre,
                                                  const int64_t *__restrict__ sep_pre,
                                                  int64_t n_samples,
                                                  int64_t *__restrict__ slot_end,
                                                  int64_t *__restrict__ live_end) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    const int64_t c0 = (int64_t)r * cpr;
    const int64_t c1 = min(c0 + cpr, n_chunks);
    const int4 *v4 = reinterpret_cast<const int4 *>(ids);
    const unsigned long long below = (1ull << lane) - 1;
    int64_t ol = live_pre[r], os = sep_pre[r];
    for (int64_t c = c0; c < c1; ++c) {
        const View w = make_view(v4[c * 64 + lane]);
        bool L[4], S[4];
        int bl = 0, bs = 0, tl = 0, ts = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const bool in = 4 * lane + e < w.len;
            L[e] = in && w.t[e] >= 0;
            S[e] = in && w.t[e] == SEP;
            const unsigned long long ml = __ballot(L[e]), ms = __ballot(S[e]);
            bl += __popcll(ml & below);
            bs += __popcll(ms & below);
            tl += __popcll(ml);
            ts += __popcll(ms);
        }
        // slots of lane l precede those of lane l+1: live tokens / terminators before (lane, e)
        // are those of the lanes below plus this lane's slots 0..e-1
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (S[e]) {
                const int64_t k = os + bs;
                if (k < n_samples) {
                    slot_end[k] = c * CHUNK + 4 * lane + e;
                    live_end[k] = ol + bl;
                }
            }
            bl += L[e];
            bs += S[e];
        }
        ol += tl;
        os += ts;
    }
}

// Packs slot ranges [src[k], src[k] + len[k]) to dst + dst_off[k], for reading chosen samples
// back in one copy.  One block per range.
__global__ void __launch_bounds__(256) k_gather_ranges(const int32_t *__restrict__ ids,
                                                       const int64_t *__restrict__ src,
                                                       const int64_t *__restrict__ len,
                                                       const int64_t *__restrict__ dst_off,
                                                       int64_t n, int32_t *__restrict__ dst) {
    for (int64_t k = blockIdx.x; k < n; k += gridDim.x) {
        const int32_t *s = ids + src[k];
        int32_t *d = dst + dst_off[k];
        for (int64_t i = threadIdx.x; i < len[k]; i += 256) d[i] = s[i];
    }
}

// Dead tail + tail tags of the last chunk after a dense write of live_slots slots.  One block of
// CHUNK threads.
__global__ void __launch_bounds__(CHUNK) k_seal(int32_t *__restrict__ ids, int64_t live_slots) {
    const int len = (int)(live_slots % CHUNK);
    if (len == 0) return;
    int32_t *p = ids + (live_slots / CHUNK) * CHUNK;
    const int t = threadIdx.x;
    const int32_t last = p[len - 1];
    if (t >= len) p[t] = (t & 1) ? TOMB_ODD : TOMB;
    __syncthreads();
    if (t == 0) p[CHUNK - 1] = tail_tag(len, last);
}

// ---------------------------------------------------------------------------------------------
// K5 ingest: latin1 bytes -> first-appearance positions + histogram, then expansion to slots.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_byte_stats(const uint8_t *__restrict__ bytes, int64_t n,
                                                    unsigned long long *__restrict__ first,
                                                    unsigned long long *__restrict__ hist) {
    __shared__ unsigned long long s_first[256];
    __shared__ unsigned int s_hist[256];
    s_first[threadIdx.x] = ~0ull;
    s_hist[threadIdx.x] = 0;
    __syncthreads();
    const int64_t per_block = 1 << 16;
    for (int64_t base = (int64_t)blockIdx.x * per_block; base < n;
         base += (int64_t)gridDim.x * per_block) {
        const int64_t end = min(base + per_block, n);
        for (int64_t i = base + threadIdx.x; i < end; i += 256) {
            const uint8_t b = bytes[i];
            atomicAdd(&s_hist[b], 1u);
            if ((unsigned long long)i < s_first[b]) atomicMin(&s_first[b], (unsigned long long)i);
        }
        __syncthreads();
        if (s_hist[threadIdx.x]) {
            atomicAdd(&hist[threadIdx.x], (unsigned long long)s_hist[threadIdx.x]);
            s_hist[threadIdx.x] = 0;
        }
        __syncthreads();
    }
    if (s_first[threadIdx.x] != ~0ull) atomicMin(&first[threadIdx.x], s_first[threadIdx.x]);
}

__global__ void k_expand_latin1(const uint8_t *__restrict__ bytes, int64_t n, int64_t sample_bytes,
                                const int32_t *__restrict__ map, int32_t *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = i / sample_bytes;
        out[i + s] = map[bytes[i]];
        if ((i + 1) % sample_bytes == 0 || i + 1 == n) out[i + s + 1] = SEP;
    }
}

}  // namespace bpe
