// bpe_pix.hip.h — the incremental mergeUntil: a position index, so
// that a merge costs O(W) work instead of a pass over the corpus.
//
// The corpus is one dense slot array (tokens, SEP = -1 between samples, TOMB for merged-away
// slots) with next / prev links over the live slots.  Slots never move, so a slot index is a
// stable position.  Every adjacent pair (u, v) has
//   - its exact count under the reference's rule (core.ts:265-293: each adjacency once, except
//     that a run of L equal tokens x counts floor(L / 2) pairs (x, x)),
//   - a list of the slots where it occurs (a segment of one pool).  A list is written once: the
//     adjacencies of a pair are all born together, either in the initial index or in the merge
//     that creates the newer of its two tokens (a merge makes new adjacencies only with the token
//     it creates).  Entries go stale as merges consume them and are filtered on use.
// in one open-addressing table keyed (u << 16 | v).  A two-level max (per 256-slot block, per 256
// blocks) over the packed selection keys (W << 17 | 0x1FFFF - (u + v), core.ts:294-305) finds the
// best pair; ties on the packed key go to the earliest last counted occurrence (rule R3), taken
// from the candidates' lists.
//
// One merge (a, b) -> c, every kernel reading the decision from PixCtl (no host round trip):
//   k_pix_select   the superblock maxima the previous merge lowered, then the best key, the
//                  candidates, R3 over their lists when tied, W, min_weight / vocabulary checks
//   k_pix_sites    the merge sites from the (a, b) list and the count changes around them (for
//                  a == b the runs, walked from their heads: sites at even offsets, replaceAll's
//                  left-to-right rule); the new adjacencies, all of which contain c
//   k_pix_alloc    segments for the new pairs, the maxima of the blocks whose max entry fell
//   k_pix_apply    tokens and links (the only kernel that changes the corpus), the new pairs'
//                  slots into their segments
// Anything the index cannot do in bounded work (a run or chain longer than PIX_WALK, a full
// buffer, more than MAX_CAND tied pairs) sets PIX_HOST before k_pix_apply: the corpus is still
// that of the last completed merge, and the host takes the iteration on the streaming path.
#pragma once
#include "bpe_kernels.hip.h"

namespace bpe {

constexpr uint32_t PIX_NONE = 0xFFFFFFFFu;    // no slot (links), empty table key
constexpr int PIX_B = 256;                    // table slots per block (block max)
constexpr int PIX_SB = 256;                   // blocks per superblock
constexpr int PIX_WALK = 1 << 16;             // longest run / chain one thread walks
constexpr int PIX_PROBE = 4096;               // longest probe sequence in the table
constexpr int PIX_GRID = 1024;                // blocks of the grid-stride kernels
constexpr uint32_t PIX_MAX_SLOTS = 0xFFFF0000u;  // largest slot array (u32 positions, PIX_NONE free)

constexpr int PIX_LOG = 4;                    // log words per merge: a, b, W, this shard's sites

// PIX_PAUSE: the batch's merges are done (the next batch goes on)
enum PixStatus { PIX_RUN = 0, PIX_DONE = 1, PIX_HOST = 2, PIX_ERROR = 3, PIX_PAUSE = 4 };

struct PixCorpus {
    int32_t *tok;
    uint32_t *nxt, *prv;
    uint32_t n;
};

struct PixTable {
    // A shard of a sharded corpus (the rank loop): cnt holds the GLOBAL counts, kept merge by merge
    // from the summed delta rows (include/bpe.h BPE_XCHG_*); this shard's count changes go to its
    // delta rows (delta != nullptr) instead of cnt.  The lists stay this shard's own.
    unsigned long long *delta;
    // ... in the lane layout (round 5, lane_w != 0): lane_w-bit lanes, lane_q to a u64 word, the
    // right side's lanes from word lane_base on (pix_delta)
    uint32_t lane_w, lane_q, lane_base;
    int32_t *len16;          // UTF-16 lengths (max_length filter)
    long long ml;            // max_length of this index's selections
    uint32_t *keys;
    unsigned long long *cnt;
    uint32_t *off, *len, *fill;
    unsigned long long *bmax, *sbmax;
    uint32_t *bdirty, *sbdirty;
    uint32_t mask;
    uint32_t nblocks, nsuper;
};

struct PixBufs {
    uint32_t *pool;      // list segments
    uint32_t *sites;     // this merge's sites
    uint2 *ent;          // this merge's new adjacencies: (table slot, position)
    uint32_t *dblocks, *dsuper;   // touched blocks / superblocks
    uint32_t site_cap, ent_cap;
};

struct PixCtl {
    int status;
    int tie;
    int32_t a, b, c;
    int32_t next_id, max_id;
    int err;
    unsigned long long W, best;
    long long min_weight, max_length;
    long long n_done, n_want;          // merges done / allowed in this batch
    uint32_t pair_slot, n_cand, tie_done, pad0;
    uint32_t n_sites, n_ent, n_dblocks, n_dsuper;
    unsigned long long n_check;        // merges made (== W when the index is consistent)
    unsigned long long pool_top, pool_cap;
    unsigned long long used, used_cap; // table claims / the claims it may hold
    uint32_t cand_slot[MAX_CAND];
    unsigned long long last[MAX_CAND];
    // sharded (delta rows): the last merge's rows are still to be added (k_pix_apply_delta); this
    // shard's sites of the merge being made (the header word the shards' sum must equal W in)
    uint32_t merged, pad1;
    // sharded, lane layout: a selected count past the batch's lanes paused the batch (the next
    // one takes wider lanes)
    uint32_t lane_over, pad2;

};

__device__ __forceinline__ uint32_t pix_key(int32_t u, int32_t v) {
    return ((uint32_t)u << 16) | (uint32_t)v;
}

__device__ __forceinline__ uint32_t pix_hash(uint32_t key) {
    uint32_t h = key * 0x9E3779B1u;
    return h ^ (h >> 15);
}

// the packed selection key of pair `k` with count w (0: no pair, or filtered by max_length)
__device__ __forceinline__ unsigned long long pix_sel_of(const PixTable &t, uint32_t k,
                                                         unsigned long long w) {
    if (k == PIX_NONE || w == 0 || (long long)w < 0 || t.ml < 0) return 0;
    const int32_t u = (int32_t)(k >> 16), v = (int32_t)(k & 0xFFFF);
    if (t.ml > 0 && (long long)t.len16[u] + t.len16[v] > t.ml) return 0;   // core.ts:270-273
    return (w << 17) | (unsigned long long)(0x1FFFF - (u + v));             // core.ts:294-305
}

__device__ __forceinline__ unsigned long long pix_sel(const PixTable &t, uint32_t s) {
    return pix_sel_of(t, t.keys[s], t.cnt[s]);
}

__device__ __forceinline__ void pix_mark(const PixTable &t, const PixBufs &B, PixCtl *ctl,
                                         uint32_t s) {
    const uint32_t blk = s / PIX_B;
    if (atomicExch(&t.bdirty[blk], 1u) == 0u) {
        const uint32_t i = atomicAdd(&ctl->n_dblocks, 1u);
        if (i < t.nblocks) B.dblocks[i] = blk;
    }
}

__device__ __forceinline__ void pix_fail(PixCtl *ctl, int why) {
    if (atomicCAS(&ctl->status, PIX_RUN, PIX_HOST) == PIX_RUN) ctl->err = why;
}

// A pair's first probe: its home slot and the key found there, loaded ahead (a site issues the
// first probes of both pairs it touches together).  Keys are only claimed during a merge, never
// removed, so a key loaded ahead stays; an empty slot loaded ahead is re-checked by the claim.
struct PixProbe {
    uint32_t s, k;
};

__device__ __forceinline__ PixProbe pix_probe(const PixTable &t, uint32_t key) {
    const uint32_t s = pix_hash(key) & t.mask;
    return {s, t.keys[s]};
}

// find-or-claim the slot of a pair; PIX_NONE when the probe sequence is exhausted
__device__ __forceinline__ uint32_t pix_slot(const PixTable &t, PixCtl *ctl, uint32_t key,
                                             bool claim, bool count_claim, PixProbe pr) {
    uint32_t s = pr.s, k = pr.k;
    for (int i = 0; i < PIX_PROBE; ++i) {
        if (i) {
            s = (s + 1) & t.mask;
            k = t.keys[s];
        }
        if (k == key) return s;
        if (k == PIX_NONE) {
            if (!claim) return PIX_NONE;
            const uint32_t old = atomicCAS(&t.keys[s], PIX_NONE, key);
            if (old == PIX_NONE) {
                if (count_claim) atomicAdd(&ctl->used, 1ull);
                return s;
            }
            if (old == key) return s;
        }
    }
    return PIX_NONE;
}

__device__ __forceinline__ uint32_t pix_slot(const PixTable &t, PixCtl *ctl, uint32_t key,
                                             bool claim, bool count_claim = false) {
    return pix_slot(t, ctl, key, claim, count_claim, pix_probe(t, key));
}

// Count change of an existing or new pair, keeping the block maxima exact.  Only new pairs (they
// all contain c) rise: k_pix_alloc lifts their block's and superblock's max once per pair.  A fall
// only matters to the entry that was its block's max, whose block is then recomputed after the
// merge's count changes (k_pix_alloc).  (The block max is read beside the add: no block max
// changes while k_pix_sites runs.)
// A shard of a sharded corpus: the change goes to this shard's delta row of the pair (every pair a
// merge (a, b) -> c changes has a side in {a, b, c}: delta_slot), summed over the shards and added
// to every shard's global counts by k_pix_apply_delta.
// The lane layout of the exchange (round 5): HDR, then PIX_XCHG_SPECIAL words for the pairs of two
// of {a, b, c}, then one count per token id and side.  Every pair a merge (a, b) -> c changes is
// one of these: a site's left neighbour l loses (l, a) and gains (l, c); its right
// neighbour r loses (b, r) and gains (c, r) (a == b: (a, r)); chains, runs and the new (c, c) pair
// only ids of {a, b, c}.  So one number per neighbour carries both changes: n_l, the sites with
// left neighbour l (the loss of (l, a), the gain of (l, c)), and n_r likewise.  No count is
// negative and n_l <= W, the merge's count, which never exceeds the last merge's (a pair counts at
// most the selected max, and the pairs a merge makes at most its W): so a batch whose first merge
// follows one of count W_0 packs lanes of bits(W_0) bits, floor(64 / bits) to a u64 word, and the
// u64 all-reduce(SUM) adds the lanes without carries.  Lanes: left side at word j / q of the
// lanes, right side from word lane_base on.
constexpr uint32_t PIX_XCHG_SPECIAL = 16;

// exchange word (after the specials) and lane shift of token o on side (0: left, 1: right)
__device__ __forceinline__ uint32_t lane_word(const PixTable &t, int side, uint32_t o, uint32_t &shift) {
    const uint32_t q = o / t.lane_q;
    shift = (o - q * t.lane_q) * t.lane_w;
    return (side ? t.lane_base : 0u) + q;
}

__device__ __forceinline__ void pix_delta(const PixTable &t, PixCtl *ctl, uint32_t key, long long d) {
    if (!d) return;
    const int32_t x = (int32_t)(key >> 16), y = (int32_t)(key & 0xFFFFu);
    if (!t.lane_w) {
        const uint32_t slot = delta_slot(x, y, ctl->a, ctl->b, ctl->c);
        if (slot == PIX_NONE) {
            pix_fail(ctl, 41);   // (cannot happen: every changed pair has its word)
            return;
        }
        atomicAdd(&t.delta[slot], (unsigned long long)d);
        return;
    }
    const int32_t a = ctl->a, b = ctl->b, c = ctl->c;
    const int sx = x == a ? 0 : x == b ? 1 : x == c ? 2 : 3;
    const int sy = y == a ? 0 : y == b ? 1 : y == c ? 2 : 3;
    if (sx < 3 && sy < 3) {
        atomicAdd(&t.delta[XCHG_HDR + 3 * sx + sy], (unsigned long long)d);
        return;
    }
    int side;
    bool gain;
    uint32_t o;
    if (sx == 3 && (sy == 0 || sy == 2)) {             // (x, a) lost, (x, c) gained
        side = 0;
        gain = sy == 2;
        o = (uint32_t)x;
    } else if (sy == 3 && (x == b || sx == 2)) {        // (b, y) lost, (c, y) gained
        side = 1;
        gain = sx == 2;
        o = (uint32_t)y;
    } else {
        pix_fail(ctl, 41);   // (cannot happen: every changed pair is one of these)
        return;
    }
    // a gain mirrors the loss at the same site (k_pix_apply_delta makes both from the count); a
    // loss that rises or a gain that falls would break that: never, checked
    if (gain != (d > 0)) {
        pix_fail(ctl, 42);
        return;
    }
    if (gain) return;
    uint32_t shift;
    const uint32_t w = lane_word(t, side, o, shift);
    atomicAdd(&t.delta[XCHG_HDR + PIX_XCHG_SPECIAL + w], (unsigned long long)(-d) << shift);
}

__device__ __forceinline__ uint32_t pix_add(const PixTable &t, const PixBufs &B, PixCtl *ctl,
                                            uint32_t key, long long d, PixProbe pr) {
    if (t.delta) {   // (sharded: no slot needed, the count is global)
        pix_delta(t, ctl, key, d);
        return PIX_NONE;
    }
    const uint32_t s = pix_slot(t, ctl, key, true, false, pr);
    if (s == PIX_NONE) {
        pix_fail(ctl, 1);
        return s;
    }
    if (d == 0) return s;
    if (d < 0) {
        const unsigned long long bm = t.bmax[s / PIX_B];
        const unsigned long long old = atomicAdd(&t.cnt[s], (unsigned long long)d);
        const unsigned long long sel = pix_sel_of(t, key, old);
        if (sel && sel >= bm) pix_mark(t, B, ctl, s);
    } else {
        atomicAdd(&t.cnt[s], (unsigned long long)d);
    }
    return s;
}

__device__ __forceinline__ uint32_t pix_add(const PixTable &t, const PixBufs &B, PixCtl *ctl,
                                            int32_t u, int32_t v, long long d) {
    const uint32_t key = pix_key(u, v);
    return pix_add(t, B, ctl, key, d, pix_probe(t, key));
}

// A new adjacency (u, v) at slot pos (u or v is c): its count, one more slot in its segment, the
// entry at index e of this merge's entry list (e = ~0u: the next free one), (table slot, pos).
// The entry that opened the pair's segment carries PIX_OWNER in its table slot (the table holds
// fewer than 2^31 slots, so that bit is free; positions use all 32 bits): k_pix_alloc places the
// segment from it.
constexpr uint32_t PIX_OWNER = 0x80000000u;
__device__ __forceinline__ void pix_entry(const PixTable &t, const PixBufs &B, PixCtl *ctl,
                                          uint32_t key, uint32_t pos, long long d, uint32_t e,
                                          PixProbe pr) {
    uint32_t s;
    if (t.delta) {   // sharded: the list entry needs this shard's slot, the count a delta row
        s = pix_slot(t, ctl, key, true, false, pr);
        if (s == PIX_NONE) {
            pix_fail(ctl, 1);
            return;
        }
        pix_delta(t, ctl, key, d);
    } else {
        s = pix_add(t, B, ctl, key, d, pr);
        if (s == PIX_NONE) return;
    }
    const uint32_t owner = atomicAdd(&t.len[s], 1u) == 0u ? PIX_OWNER : 0u;
    if (e == ~0u) e = atomicAdd(&ctl->n_ent, 1u);
    if (e < B.ent_cap) B.ent[e] = make_uint2(s | owner, pos);
    else pix_fail(ctl, 3);
}

__device__ __forceinline__ void pix_entry(const PixTable &t, const PixBufs &B, PixCtl *ctl,
                                          int32_t u, int32_t v, uint32_t pos, long long d,
                                          uint32_t e = ~0u) {
    const uint32_t key = pix_key(u, v);
    pix_entry(t, B, ctl, key, pos, d, e, pix_probe(t, key));
}

__device__ __forceinline__ bool pix_tok_is(const PixCorpus &C, uint32_t p, int32_t x) {
    return p != PIX_NONE && C.tok[p] == x;
}

// ---- index build: a counting scatter of every pair's positions into its segment -------------
// (no sort: the pair table itself is the histogram)
//   k_pix_build_links  links i -> i +- 1, and per block of PB positions its last run start
//   k_pix_scan_max     the run start each block's first position continues (exclusive max-scan)
//   k_pix_hot_count    per valid pair position: list length + 1 and, for (x, x) at an odd offset
//                      of its run, one uncounted occurrence (core.ts:285-290).  Hot pairs (both
//                      ids < 256) go to 65536 16-bit LDS counters per workgroup (one pass),
//                      dumped as the workgroup's slab; other pairs claim their table slot and
//                      count there (global atomics)
//   k_pix_hot_scan     per hot pair: its total, and each workgroup's exclusive offset (in place)
//   k_pix_hot_claim    a table slot per hot pair that occurs, with its length and count
//   k_pix_build_alloc  a pool segment per pair (one pool atomic per wave)
//   (k_pix_hot_seg, k_pix_hot_xoff, k_pix_fill_x, k_pix_fill_y: the two-level fill, below)
//   k_pix_hot_fill     every position into its pair's segment: hot pairs through per-workgroup
//                      LDS cursors (segment + the workgroup's offset), the others through the
//                      pair's global fill counter
// Round 2 sorted the keys with rocPRIM, and round 3's first version claimed and counted every
// position with global atomics (65536 hot addresses, 2 atomics per position: 150 ms at C3).
constexpr int PB = 4096;          // positions per build block

// (run starts are u32 positions; 0 is the identity of their max: position 0 always starts a run)
__device__ __forceinline__ uint32_t block_max_u32(uint32_t v, uint32_t *red) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    v = max(max(red[0], red[1]), max(red[2], red[3]));
    __syncthreads();
    return v;
}

__global__ void __launch_bounds__(256) k_pix_build_links(PixCorpus C, uint32_t *__restrict__ blast) {
    __shared__ uint32_t red[4];
    const uint32_t nblk = (C.n + PB - 1) / PB;
    for (uint32_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        const uint32_t i0 = blk * PB, i1 = min(i0 + PB, C.n);
        uint32_t m = 0;
        for (uint32_t i = i0 + threadIdx.x; i < i1; i += 256) {
            const int32_t t = C.tok[i];
            if (i == 0 || C.tok[i - 1] != t) m = i;   // (i grows: the last one wins)
            C.nxt[i] = i + 1 < C.n ? i + 1 : PIX_NONE;
            C.prv[i] = i > 0 ? i - 1 : PIX_NONE;
        }
        m = block_max_u32(m, red);
        if (threadIdx.x == 0) blast[blk] = m;
    }
}

// In place: v[b] <- max(v[0 .. b-1]) (0 for b = 0).  One block of 1024.
__global__ void __launch_bounds__(1024) k_pix_scan_max(uint32_t *__restrict__ v, uint32_t n) {
    __shared__ uint32_t part[1024];
    const uint32_t per = (n + 1023) / 1024, t = threadIdx.x;
    uint32_t acc = 0;
    for (uint32_t k = 0; k < per; ++k) {
        const uint32_t i = t * per + k;
        if (i < n) acc = max(acc, v[i]);
    }
    part[t] = acc;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint32_t o = t >= d ? part[t - d] : 0u;
        __syncthreads();
        part[t] = max(part[t], o);
        __syncthreads();
    }
    uint32_t run = t ? part[t - 1] : 0u;
    for (uint32_t k = 0; k < per; ++k) {
        const uint32_t i = t * per + k;
        if (i < n) {
            const uint32_t x = v[i];
            v[i] = run;
            run = max(run, x);
        }
    }
}

// In place: v[b] <- v[0] + ... + v[b-1] (u32).  One block of 1024.
__global__ void __launch_bounds__(1024) k_pix_scan_sum(uint32_t *__restrict__ v, uint32_t n,
                                                       uint32_t *__restrict__ total) {
    __shared__ uint32_t part[1024];
    const uint32_t per = (n + 1023) / 1024, t = threadIdx.x;
    uint32_t acc = 0;
    for (uint32_t k = 0; k < per; ++k) {
        const uint32_t i = t * per + k;
        if (i < n) acc += v[i];
    }
    part[t] = acc;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint32_t o = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += o;
        __syncthreads();
    }
    uint32_t run = t ? part[t - 1] : 0;
    for (uint32_t k = 0; k < per; ++k) {
        const uint32_t i = t * per + k;
        if (i < n) {
            const uint32_t x = v[i];
            v[i] = run;
            run += x;
        }
    }
    if (t == 1023 && total) *total = part[1023];
}

// The hot passes: PH_WG workgroups (one per CU) of PH_T threads, each over the blocks blk =
// workgroup, workgroup + PH_WG, ...; per block, each thread takes PH_PER consecutive positions.
constexpr int PH_T = 1024;
constexpr int PH_PER = PB / PH_T;
constexpr int PH_HALF = 32768;     // hot pairs per pass: (x, y) with y >> 7 == half
constexpr int PH_WG_MAX = 256;

__device__ __forceinline__ uint32_t ph_local(int32_t x, int32_t y) {
    return ((uint32_t)x << 7) | ((uint32_t)y & 127u);
}

// the hot pair of pass `half`, local index i -> (x << 8) | y
__device__ __forceinline__ uint32_t ph_index(uint32_t half, uint32_t i) {
    return ((i >> 7) << 8) | (half << 7) | (i & 127u);
}

// Stages block blk's PB tokens and the one after them in tk.  RS: also the run start that this
// thread's first position continues (an inclusive max-scan of the threads' last run starts: by
// shuffles in the wave, across the waves through sc, seeded with the block's carry).
// (the loads of a block's tokens into registers, a block ahead of their store into tk, so the
// next block's loads overlap this block's work)
struct PhNext {
    int32_t v[PB / PH_T + 1];
};

__device__ __forceinline__ void ph_fetch(const PixCorpus &C, uint32_t blk, PhNext &r) {
    const uint32_t b0 = blk * PB;
#pragma unroll
    for (int q = 0; q <= PB / PH_T; ++q) {
        const uint32_t k = threadIdx.x + q * PH_T, i = b0 + k;
        r.v[q] = k <= (uint32_t)PB && i < C.n ? __builtin_nontemporal_load(C.tok + i) : SEP;
    }
}

__device__ __forceinline__ void ph_put(int32_t *tk, const PhNext &r) {
#pragma unroll
    for (int q = 0; q <= PB / PH_T; ++q) {
        const uint32_t k = threadIdx.x + q * PH_T;
        if (k <= (uint32_t)PB) tk[k] = r.v[q];
    }
    __syncthreads();
}

template <bool RS>
__device__ __forceinline__ uint32_t ph_runs(const PixCorpus &C, int32_t *tk, uint32_t *sc,
                                            uint32_t blk, uint32_t carry);

template <bool RS>
__device__ __forceinline__ uint32_t ph_span(const PixCorpus &C, int32_t *tk, uint32_t *sc,
                                            uint32_t blk, uint32_t carry) {
    const uint32_t b0 = blk * PB;
    for (uint32_t k = threadIdx.x; k <= (uint32_t)PB; k += PH_T) {
        const uint32_t i = b0 + k;
        tk[k] = i < C.n ? C.tok[i] : SEP;
    }
    __syncthreads();
    return ph_runs<RS>(C, tk, sc, blk, carry);
}

// The run start that this thread's first position continues (tk staged)
template <bool RS>
__device__ __forceinline__ uint32_t ph_runs(const PixCorpus &C, int32_t *tk, uint32_t *sc,
                                            uint32_t blk, uint32_t carry) {
    if (!RS) return 0;
    const uint32_t b0 = blk * PB;
    const uint32_t l0 = threadIdx.x * PH_PER;
    uint32_t last = 0;   // (0: none here; the max over the positions before still holds one)
#pragma unroll
    for (int k = 0; k < PH_PER; ++k) {
        const uint32_t l = l0 + k, i = b0 + l;
        if (i < C.n && (i == 0 || (l ? tk[l - 1] : C.tok[i - 1]) != tk[l])) last = i;
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t v = last;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(v, d);
        if (lane >= d) v = max(v, o);
    }
    if (lane == 63) sc[wv] = v;
    __syncthreads();
    uint32_t rs = carry;
    for (int w = 0; w < wv; ++w) rs = max(rs, sc[w]);
    const uint32_t ex = __shfl_up(v, 1);
    return lane ? max(rs, ex) : rs;
}

// One pass over the corpus for both halves: 16-bit LDS counters, two per dword (pair
// p = (x << 8) | y: dword p >> 1, half p & 1).  Every add returns the dword it found; a block
// whose adds saw some half at >= 0x4000 ends with a sweep that moves every such half into the
// workgroup's slab entry (global, zeroed by the host), so no half passes 0x4000 + PB.
__global__ void __launch_bounds__(PH_T) k_pix_hot_count(PixCorpus C, PixTable t, PixCtl *ctl,
                                                        const uint32_t *__restrict__ carry,
                                                        uint32_t *__restrict__ slab,
                                                        unsigned long long *__restrict__ oddxx) {
    __shared__ uint32_t cnt[32768];
    __shared__ int32_t tk[PB + 1];
    __shared__ uint32_t sc[PH_T / 64];
    __shared__ uint32_t odd[256];
    __shared__ uint32_t s_sweep;
    const uint32_t G = gridDim.x;
    // (slab index of pair p: the layout of the two half passes, [half][workgroup][x << 7 | y & 127])
    auto slab_at = [&](uint32_t p) {
        return ((size_t)((p >> 7) & 1u) * G + blockIdx.x) * PH_HALF + ((p >> 8) << 7) + (p & 127u);
    };
    for (int i = threadIdx.x; i < 32768; i += PH_T) cnt[i] = 0;
    if (threadIdx.x < 256) odd[threadIdx.x] = 0;
    bool swept = false;
    const uint32_t nblk = (C.n + PB - 1) / PB;
    PhNext nx;
    if (blockIdx.x < nblk) ph_fetch(C, blockIdx.x, nx);
    for (uint32_t blk = blockIdx.x; blk < nblk; blk += G) {
        __syncthreads();   // (tk and sc of the previous block are read; so is s_sweep)
        if (threadIdx.x == 0) s_sweep = 0;
        ph_put(tk, nx);
        if (blk + G < nblk) ph_fetch(C, blk + G, nx);
        uint32_t rs = ph_runs<true>(C, tk, sc, blk, carry[blk]);
        const uint32_t l0 = threadIdx.x * PH_PER, i0 = blk * PB + l0;
        uint32_t seen = 0;
#pragma unroll
        for (int k = 0; k < PH_PER; ++k) {
            const uint32_t l = l0 + k, i = i0 + k;
            if (i >= C.n) break;
            const int32_t x = tk[l], y = i + 1 < C.n ? tk[l + 1] : SEP;
            if (i == 0 || (l ? tk[l - 1] : C.tok[i - 1]) != x) rs = i;
            if ((x | y) < 0) continue;
            const bool uncounted = x == y && ((i - rs) & 1u);
            if ((x | y) < 256) {
                const uint32_t p = ((uint32_t)x << 8) | (uint32_t)y;
                seen |= atomicAdd(&cnt[p >> 1], 1u << ((p & 1u) << 4));
                if (uncounted) atomicAdd(&odd[x], 1u);
            } else {
                const uint32_t s = pix_slot(t, ctl, pix_key(x, y), true, true);
                if (s == PIX_NONE) {
                    atomicOr(&ctl->err, 9);   // (the table is too full: the host builds a bigger one)
                    continue;
                }
                atomicAdd(&t.len[s], 1u);
                if (!uncounted) atomicAdd(&t.cnt[s], 1ull);
            }
        }
        if (seen & 0xC000C000u) s_sweep = 1;
        __syncthreads();
        if (s_sweep) {   // (uniform: read by every thread between the two barriers)
            swept = true;
            for (uint32_t w = threadIdx.x; w < 32768u; w += PH_T) {
                uint32_t v = cnt[w];
                if (!(v & 0xC000C000u)) continue;
                for (uint32_t h = 0; h < 2; ++h) {
                    const uint32_t c = (v >> (h << 4)) & 0xFFFFu;
                    if (c < 0x4000u) continue;
                    atomicAdd(&slab[slab_at(2 * w + h)], c);
                    v &= ~(0xFFFFu << (h << 4));
                }
                cnt[w] = v;
            }
        }
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < 65536u; j += PH_T) {
        // (slab order: half, then x, then y & 127)
        const uint32_t half = j >> 15, loc = j & 32767u;
        const uint32_t p = ((loc >> 7) << 8) | (half << 7) | (loc & 127u);
        const uint32_t c = (cnt[p >> 1] >> ((p & 1u) << 4)) & 0xFFFFu;
        uint32_t *o = slab + ((size_t)half * G + blockIdx.x) * PH_HALF + loc;
        if (swept) atomicAdd(o, c);
        else *o = c;
    }
    if (threadIdx.x < 256 && odd[threadIdx.x])
        atomicAdd(&oddxx[threadIdx.x], (unsigned long long)odd[threadIdx.x]);
}

// One thread per hot pair: the workgroups' counts (G slabs of the pair's half) become their
// exclusive offsets, and the total goes to htot[(x << 8) | y].  Loads issued 16 at a time.
__global__ void __launch_bounds__(256) k_pix_hot_scan(uint32_t *__restrict__ slab, int G,
                                                      uint32_t *__restrict__ htot) {
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j >= 2u * PH_HALF) return;
    const uint32_t half = j / PH_HALF, i = j % PH_HALF;
    uint32_t *p = slab + (size_t)half * G * PH_HALF + i;
    uint32_t run = 0;
    for (int w0 = 0; w0 < G; w0 += 16) {
        uint32_t v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = w0 + q < G ? p[(size_t)(w0 + q) * PH_HALF] : 0u;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            if (w0 + q < G) p[(size_t)(w0 + q) * PH_HALF] = run;
            run += v[q];
        }
    }
    htot[ph_index(half, i)] = run;
}

// A table slot for every hot pair that occurs, with its list length and count.
__global__ void __launch_bounds__(256) k_pix_hot_claim(PixTable t, PixCtl *ctl,
                                                       const uint32_t *__restrict__ htot,
                                                       const unsigned long long *__restrict__ oddxx,
                                                       uint32_t *__restrict__ hslot) {
    const uint32_t idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= 65536u) return;
    const uint32_t n = htot[idx];
    uint32_t s = PIX_NONE;
    if (n) {
        const int32_t x = (int32_t)(idx >> 8), y = (int32_t)(idx & 255u);
        s = pix_slot(t, ctl, pix_key(x, y), true, true);
        if (s == PIX_NONE) {
            atomicOr(&ctl->err, 9);
        } else {
            t.len[s] = n;
            t.cnt[s] = (unsigned long long)n - (x == y ? oddxx[x] : 0ull);
        }
    }
    hslot[idx] = s;
}

__device__ __forceinline__ bool pix_hot_key(uint32_t k) {
    return k != PIX_NONE && (k >> 16) < 256u && (k & 0xFFFFu) < 256u;
}

// (skip_hot: the hot pairs' segments were placed by k_pix_hot_seg, in (x, y) order)
__global__ void __launch_bounds__(256) k_pix_build_alloc(PixTable t, PixCtl *ctl, uint32_t cap,
                                                         int skip_hot = 0) {
    const int lane = threadIdx.x & 63;
    for (uint32_t s0 = (blockIdx.x * blockDim.x) & ~63u; s0 < cap; s0 += gridDim.x * blockDim.x) {
        const uint32_t s = s0 + lane + (threadIdx.x & ~63u);
        const uint32_t len = s < cap && !(skip_hot && pix_hot_key(t.keys[s])) ? t.len[s] : 0u;
        uint32_t incl = len;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(incl, d);
            if (lane >= d) incl += o;
        }
        const uint32_t tot = __shfl(incl, 63);
        unsigned long long base = 0;
        if (lane == 0 && tot) base = atomicAdd(&ctl->pool_top, (unsigned long long)tot);
        base = __shfl(base, 0);
        if (len) {
            t.off[s] = (uint32_t)(base + incl - len);
            t.fill[s] = 0;
        }
    }
}

// Every position into its pair's segment.  Hot pairs of this pass: a per-workgroup LDS cursor
// per pair, starting at the pair's segment + this workgroup's offset (k_pix_hot_scan), so no two
// workgroups share a global counter.  Other pairs (pass 0): the pair's global fill counter.
__global__ void __launch_bounds__(PH_T) k_pix_hot_fill(PixCorpus C, PixTable t, PixBufs B, int half,
                                                       const uint32_t *__restrict__ slab,
                                                       const uint32_t *__restrict__ hslot) {
    __shared__ uint32_t cur[PH_HALF];
    __shared__ int32_t tk[PB + 1];
    const uint32_t *base = slab + ((size_t)half * gridDim.x + blockIdx.x) * PH_HALF;
    for (uint32_t i = threadIdx.x; i < (uint32_t)PH_HALF; i += PH_T) {
        const uint32_t s = hslot[ph_index((uint32_t)half, i)];
        cur[i] = s != PIX_NONE ? t.off[s] + base[i] : 0u;
    }
    const uint32_t nblk = (C.n + PB - 1) / PB;
    for (uint32_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        __syncthreads();
        ph_span<false>(C, tk, nullptr, blk, 0);
        const uint32_t l0 = threadIdx.x * PH_PER, i0 = blk * PB + l0;
#pragma unroll
        for (int k = 0; k < PH_PER; ++k) {
            const uint32_t l = l0 + k, i = i0 + k;
            if (i + 1 >= C.n) break;
            const int32_t x = tk[l], y = tk[l + 1];
            if ((x | y) < 0) continue;
            if ((x | y) < 256) {
                if ((y >> 7) != half) continue;
                B.pool[atomicAdd(&cur[ph_local(x, y)], 1u)] = i;
            } else if (half == 0) {
                const uint32_t key = pix_key(x, y);
                uint32_t s = pix_hash(key) & t.mask;
                // (present: claimed by the count, within its probe bound)
                for (int p = 0; p < PIX_PROBE && t.keys[s] != key; ++p) s = (s + 1) & t.mask;
                if (t.keys[s] != key) continue;
                B.pool[t.off[s] + atomicAdd(&t.fill[s], 1u)] = i;
            }
        }
    }
}

// The two-level fill (the corpus's hot pairs are not skewed towards a few first tokens): the hot
// pairs' segments lie in (x, y) order, so the segments of first token x form one bucket.
//   k_pix_hot_seg    per hot pair its segment (an exclusive scan of the totals in (x, y) order),
//                    per x its bucket; the cold pairs' segments follow (pool_top)
//   k_pix_hot_xoff   per (workgroup, x) where that workgroup's positions of bucket x start (its
//                    count from the slabs, an exclusive scan over the workgroups)
//   k_pix_fill_x     every hot position (y, i) into its bucket, through 256 LDS cursors per
//                    workgroup; cold positions through their pair's global fill counter
//   k_pix_fill_y     one workgroup per bucket: every (y, i) into segment (x, y), 256 LDS cursors
// Each workgroup writes 256 streams at a time (k_pix_hot_fill: 32768), few enough for L2 to
// combine the 4- and 8-byte stores into lines.
__global__ void __launch_bounds__(1024) k_pix_hot_seg(PixTable t, PixCtl *ctl,
                                                      const uint32_t *__restrict__ htot,
                                                      const uint32_t *__restrict__ hslot,
                                                      uint32_t *__restrict__ hseg,
                                                      uint32_t *__restrict__ bucket) {
    __shared__ uint32_t part[1024];
    const uint32_t tid = threadIdx.x, i0 = tid * 64;   // 64 hot pairs per thread, (x, y) order
    uint32_t acc = 0;
    for (int k = 0; k < 64; ++k) acc += htot[i0 + k];
    part[tid] = acc;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint32_t o = tid >= d ? part[tid - d] : 0u;
        __syncthreads();
        part[tid] += o;
        __syncthreads();
    }
    uint32_t run = tid ? part[tid - 1] : 0u;
    for (int k = 0; k < 64; ++k) {
        const uint32_t idx = i0 + k, n = htot[idx];
        hseg[idx] = run;
        if ((idx & 255u) == 0) bucket[idx >> 8] = run;
        const uint32_t sl = hslot[idx];
        if (n && sl != PIX_NONE) {
            t.off[sl] = run;
            t.fill[sl] = 0;
        }
        run += n;
    }
    if (tid == 1023) {
        bucket[256] = run;
        ctl->pool_top = run;   // (the cold pairs' segments after the hot ones)
    }
}

// block x, thread w: workgroup w's positions with first token x start at bucket[x] +
// xoff[w * 256 + x].  (Runs on the slabs' counts, before k_pix_hot_scan turns them into offsets.)
__global__ void __launch_bounds__(256) k_pix_hot_xoff(const uint32_t *__restrict__ slab, int G,
                                                      uint32_t *__restrict__ xoff) {
    __shared__ uint32_t part[256];
    const uint32_t x = blockIdx.x, w = threadIdx.x;
    uint32_t c = 0;
    if ((int)w < G)
        for (uint32_t half = 0; half < 2; ++half) {
            const uint4 *p = reinterpret_cast<const uint4 *>(slab + ((size_t)half * G + w) * PH_HALF +
                                                             (x << 7));
#pragma unroll 8
            for (int k = 0; k < 32; ++k) {
                const uint4 v = p[k];
                c += v.x + v.y + v.z + v.w;
            }
        }
    part[w] = c;
    __syncthreads();
    for (uint32_t d = 1; d < 256; d <<= 1) {
        const uint32_t o = w >= d ? part[w - d] : 0u;
        __syncthreads();
        part[w] += o;
        __syncthreads();
    }
    if ((int)w < G) xoff[w * 256 + x] = w ? part[w - 1] : 0u;
}

// (staged: a bucket's entries collect in LDS, FX_SB per bucket, and leave as runs of at least
// FX_FLUSH consecutive entries of this workgroup's range; what does not fit goes straight out)
constexpr int FX_SB = 32;
constexpr int FX_FLUSH = 16;

__device__ __forceinline__ void fx_flush(uint2 *__restrict__ stage, uint32_t *cur, uint32_t *lc,
                                         const uint2 *buf, uint32_t min_n) {
    // two buckets per wave and round, FX_SB lanes each
    const int lane = threadIdx.x & 63, half = lane >> 5, sl = lane & 31;
    for (uint32_t b = (threadIdx.x >> 6) * 2 + half; b < 256; b += (PH_T / 64) * 2) {
        const uint32_t n = min(lc[b], (uint32_t)FX_SB);
        if (n >= min_n && n > 0) {
            const uint32_t at = cur[b];
            if ((uint32_t)sl < n) stage[at + sl] = buf[b * FX_SB + sl];
            // (every lane of the half has read cur[b] and lc[b] before lane 0 updates them:
            // the reads and the writes are one wave's instructions, in program order)
            if (sl == 0) { cur[b] = at + n; lc[b] = 0; }
        } else if (sl == 0) {
            lc[b] = n;
        }
    }
}

__global__ void __launch_bounds__(PH_T) k_pix_fill_x(PixCorpus C, PixTable t, PixBufs B,
                                                     const uint32_t *__restrict__ xoff,
                                                     const uint32_t *__restrict__ bucket,
                                                     uint2 *__restrict__ stage) {
    __shared__ uint32_t cur[256], lc[256];
    __shared__ uint2 buf[256 * FX_SB];
    __shared__ int32_t tk[PB + 1];
    if (threadIdx.x < 256) {
        cur[threadIdx.x] = bucket[threadIdx.x] + xoff[blockIdx.x * 256 + threadIdx.x];
        lc[threadIdx.x] = 0;
    }
    const uint32_t nblk = (C.n + PB - 1) / PB;
    PhNext nx;
    if (blockIdx.x < nblk) ph_fetch(C, blockIdx.x, nx);
    for (uint32_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        __syncthreads();
        ph_put(tk, nx);
        if (blk + gridDim.x < nblk) ph_fetch(C, blk + gridDim.x, nx);
        const uint32_t l0 = threadIdx.x * PH_PER, i0 = blk * PB + l0;
        // (the hot positions' slot claims first, all of them, then their stores)
        uint32_t at[PH_PER];
#pragma unroll
        for (int k = 0; k < PH_PER; ++k) {
            const int32_t x = tk[l0 + k], y = tk[l0 + k + 1];
            const bool hot = i0 + k + 1 < C.n && (x | y) >= 0 && (x | y) < 256;
            at[k] = hot ? atomicAdd(&lc[x], 1u) : PIX_NONE;
        }
#pragma unroll
        for (int k = 0; k < PH_PER; ++k) {
            if (at[k] == PIX_NONE) continue;
            const int32_t x = tk[l0 + k];
            const uint2 e = make_uint2((uint32_t)tk[l0 + k + 1], i0 + k);
            if (at[k] < (uint32_t)FX_SB) buf[x * FX_SB + at[k]] = e;
            else stage[atomicAdd(&cur[x], 1u)] = e;
        }
#pragma unroll
        for (int k = 0; k < PH_PER; ++k) {
            const uint32_t l = l0 + k, i = i0 + k;
            if (i + 1 >= C.n) break;
            const int32_t x = tk[l], y = tk[l + 1];
            if ((x | y) < 256) continue;   // (a separator, or hot: above)
            const uint32_t key = pix_key(x, y);
            uint32_t s = pix_hash(key) & t.mask;
            // (present: claimed by the count, within its probe bound)
            for (int p = 0; p < PIX_PROBE && t.keys[s] != key; ++p) s = (s + 1) & t.mask;
            if (t.keys[s] != key) continue;
            B.pool[t.off[s] + atomicAdd(&t.fill[s], 1u)] = i;
        }
        __syncthreads();
        fx_flush(stage, cur, lc, buf, FX_FLUSH);
    }
    __syncthreads();
    fx_flush(stage, cur, lc, buf, 1);
}

// (staged as in k_pix_fill_x: a segment's positions collect in LDS, FY_SB per segment, and
// leave as runs of at least FY_FLUSH; the stage is read a round ahead)
constexpr int FY_SB = 64;
constexpr int FY_FLUSH = 32;
constexpr int FY_PER = 8;   // entries per thread and round

__global__ void __launch_bounds__(1024) k_pix_fill_y(PixBufs B, const uint32_t *__restrict__ hseg,
                                                     const uint32_t *__restrict__ bucket,
                                                     const uint2 *__restrict__ stage) {
    __shared__ uint32_t cur[256], lc[256];
    __shared__ uint32_t buf[256 * FY_SB];
    const uint32_t x = blockIdx.x;
    if (threadIdx.x < 256) {
        cur[threadIdx.x] = hseg[x * 256 + threadIdx.x];
        lc[threadIdx.x] = 0;
    }
    const uint32_t b0 = bucket[x], b1 = bucket[x + 1];
    uint2 nx[FY_PER];
    auto fetch = [&](uint32_t r0) {
#pragma unroll
        for (int k = 0; k < FY_PER; ++k) {
            const uint32_t j = r0 + threadIdx.x + 1024 * k;
            if (j < b1) {
                const unsigned long long v = __builtin_nontemporal_load(
                    reinterpret_cast<const unsigned long long *>(stage + j));
                nx[k] = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
            } else {
                nx[k] = make_uint2(256u, 0u);
            }
        }
    };
    // one segment per wave and round, a lane per buffered position
    auto flush = [&](uint32_t min_n) {
        const int lane = threadIdx.x & 63;
        for (uint32_t y = threadIdx.x >> 6; y < 256; y += 16) {
            const uint32_t n = min(lc[y], (uint32_t)FY_SB);
            if (n >= min_n && n > 0) {
                const uint32_t at = cur[y];
                if ((uint32_t)lane < n) B.pool[at + lane] = buf[y * FY_SB + lane];
                // (the wave's reads of cur[y] and lc[y] precede lane 0's writes, in program order)
                if (lane == 0) { cur[y] = at + n; lc[y] = 0; }
            } else if (lane == 0) {
                lc[y] = n;
            }
        }
    };
    fetch(b0);
    for (uint32_t r0 = b0; r0 < b1; r0 += FY_PER * 1024) {
        __syncthreads();   // (the last flush is done)
        uint2 e[FY_PER];
        uint32_t at[FY_PER];
#pragma unroll
        for (int k = 0; k < FY_PER; ++k) e[k] = nx[k];
        fetch(r0 + FY_PER * 1024);
#pragma unroll
        for (int k = 0; k < FY_PER; ++k) at[k] = e[k].x < 256u ? atomicAdd(&lc[e[k].x], 1u) : PIX_NONE;
#pragma unroll
        for (int k = 0; k < FY_PER; ++k) {
            if (at[k] == PIX_NONE) continue;
            if (at[k] < (uint32_t)FY_SB) buf[e[k].x * FY_SB + at[k]] = e[k].y;
            else B.pool[atomicAdd(&cur[e[k].x], 1u)] = e[k].y;
        }
        __syncthreads();
        flush(FY_FLUSH);
    }
    __syncthreads();
    flush(1);
}

// Block maxima: of every block (build), or recomputed for the blocks whose max entry fell
// (after a merge; one wave per block).  A block whose max fell may take its superblock's max
// with it: that superblock is recomputed next (k_pix_sbmax).
__global__ void __launch_bounds__(256) k_pix_bmax_all(PixTable t) {
    const int lane = threadIdx.x & 63;
    for (uint32_t blk = blockIdx.x * 4 + (threadIdx.x >> 6); blk < t.nblocks; blk += gridDim.x * 4) {
        unsigned long long m = 0;
        for (int k = lane; k < PIX_B; k += 64) m = max(m, pix_sel(t, blk * PIX_B + k));
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) m = max(m, (unsigned long long)__shfl_xor(m, d));
        if (lane == 0) t.bmax[blk] = m;
    }
}

// (rank: this workgroup's place in the grid; k_pix_alloc counts from the end, where the
// workgroups without entries are)
__device__ __forceinline__ void pix_bmax_dirty(const PixTable &t, const PixBufs &B, PixCtl *ctl,
                                               uint32_t rank) {
    const int lane = threadIdx.x & 63;
    const uint32_t nb = min(ctl->n_dblocks, t.nblocks);
    for (uint32_t i = rank * 4 + (threadIdx.x >> 6); i < nb; i += gridDim.x * 4) {
        const uint32_t blk = B.dblocks[i];
        unsigned long long m = 0;
        for (int k = lane; k < PIX_B; k += 64) m = max(m, pix_sel(t, blk * PIX_B + k));
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) m = max(m, (unsigned long long)__shfl_xor(m, d));
        if (lane == 0) {
            const unsigned long long old = t.bmax[blk];
            t.bmax[blk] = m;
            t.bdirty[blk] = 0;
            const uint32_t sb = blk / PIX_SB;
            if (m < old && old >= t.sbmax[sb] && atomicExch(&t.sbdirty[sb], 1u) == 0u) {
                const uint32_t k = atomicAdd(&ctl->n_dsuper, 1u);
                if (k < t.nsuper) B.dsuper[k] = sb;
            }
        }
    }
}

__global__ void __launch_bounds__(256) k_pix_sbmax(PixTable t, PixBufs B, PixCtl *ctl, int all) {
    __shared__ unsigned long long red[4];
    __shared__ uint32_t s_ns;
    if (threadIdx.x == 0)   // (read once and broadcast: the loop around the barriers is uniform)
        s_ns = all ? t.nsuper : (ctl->status != PIX_RUN ? 0u : min(ctl->n_dsuper, t.nsuper));
    __syncthreads();
    const uint32_t ns = s_ns;
    for (uint32_t i = blockIdx.x; i < ns; i += gridDim.x) {
        const uint32_t sb = all ? i : B.dsuper[i];
        const uint32_t blk = sb * PIX_SB + threadIdx.x;
        unsigned long long m = blk < t.nblocks ? t.bmax[blk] : 0;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) m = max(m, (unsigned long long)__shfl_xor(m, d));
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            t.sbmax[sb] = max(max(red[0], red[1]), max(red[2], red[3]));
            t.sbdirty[sb] = 0;
        }
        __syncthreads();
    }
}

// a batch of n merges from the next vocabulary id on
__global__ void k_pix_begin(PixCtl *ctl, long long n, int32_t next_id, long long min_weight) {
    if (ctl->status == PIX_PAUSE) ctl->status = PIX_RUN;
    ctl->n_done = 0;
    ctl->n_want = n;
    ctl->next_id = next_id;
    ctl->min_weight = min_weight;
}

// ---- one merge --------------------------------------------------------------------------------
// R3 (core.ts:294-305) costs one iteration of the kernel sequence, not a launch per merge: when the
// best key is tied, k_pix_select publishes the candidates and sets tie = 1; k_pix_sites then scans
// their lists on the whole grid instead of merging (the last block decides: tie = 2), k_pix_alloc
// and k_pix_apply do nothing; the next k_pix_select commits the decided pair.  (A separate tie
// launch cost 5.5 us per merge for the 372 ties among the 8000 C3 merges; one block scanning the
// lists took ~240 us per tie.)
// Sharded: the scan leaves this shard's last counted occurrences (PIX_TIE_WAIT); pix_decide (block 0
// of k_pix_alloc) takes the earliest of the all-reduced (shard << 40 | position) after the exchange.
enum PixTie { PIX_TIE_NONE = 0, PIX_TIE_SCAN = 1, PIX_TIE_DECIDED = 2, PIX_TIE_WAIT = 3 };

// The merge of pair slot s (key `key`, list length len): vocabulary and table-room checks, then
// the decision every later kernel reads.  (Thread 0 of k_pix_select.)
__device__ void pix_commit(const PixTable &t, PixCtl *ctl, uint32_t s, uint32_t key, uint32_t len) {
    if (ctl->next_id >= ctl->max_id) {
        ctl->status = PIX_HOST;                                       // vocabulary limit
        ctl->err = 5;
        return;
    }
    // room for this merge's claims (<= 2 per site; sharded: also the pairs other shards create,
    // <= 2 per global occurrence) within the table's fill limit
    const unsigned long long need = 2 * max((unsigned long long)len, t.delta ? ctl->W : 0ull) + 64;
    if (ctl->used + need > ctl->used_cap) {
        ctl->status = PIX_HOST;
        ctl->err = 6;
        return;
    }
    const int32_t c = ctl->next_id, a = (int32_t)(key >> 16), b = (int32_t)(key & 0xFFFF);
    ctl->c = c;
    ctl->pair_slot = s;
    ctl->a = a;
    ctl->b = b;
    ctl->tie = PIX_TIE_NONE;
    // c's length before this merge's new pairs are ranked (their block maxima in k_pix_alloc and
    // k_pix_apply read it under max_length)
    t.len16[c] = t.len16[a] + t.len16[b];                             // core.ts:318
}

// Best key, candidates (every pair sharing it), the decision.  One block of 1024.
__global__ void __launch_bounds__(1024) k_pix_select(PixTable t, PixBufs B, PixCtl *ctl) {
    __shared__ unsigned long long red[16];
    __shared__ uint32_t lst[64];
    __shared__ uint32_t n_lst, n_blk, n_cs;
    __shared__ uint32_t blks[64], cs[MAX_CAND], cs_key[MAX_CAND], cs_len[MAX_CAND];
    __shared__ uint32_t s_go, s_nd, s_tie;
    __shared__ long long s_mw;
    const int tid = threadIdx.x;
    // (every control value a branch below depends on is read by one thread and broadcast through
    // LDS, so the whole block takes the same path: each barrier is reached by all of its threads)
    if (tid == 0) {
        s_go = ctl->status != PIX_RUN ? 0u : ctl->n_done >= ctl->n_want ? 1u : 2u;
        s_nd = min(ctl->n_dsuper, t.nsuper);
        s_mw = ctl->min_weight;
        s_tie = (uint32_t)ctl->tie;
    }
    __syncthreads();
    if (s_go == 0) return;
    if (s_go == 2 && s_tie == PIX_TIE_DECIDED) {
        // the tie the last iteration's scan decided (nothing changed since): commit its pair
        if (tid == 0) {
            const uint32_t sl = ctl->pair_slot;
            ctl->n_sites = ctl->n_ent = ctl->n_dblocks = ctl->n_dsuper = 0;
            ctl->n_check = 0;
            pix_commit(t, ctl, sl, t.keys[sl], t.len[sl]);
        }
        return;
    }
    {
        // the superblocks the previous merge may have lowered (one wave each)
        const int lane = tid & 63, wv = tid >> 6;
        const uint32_t nd = s_nd;
        for (uint32_t q = wv; q < nd; q += 16) {
            const uint32_t sb = B.dsuper[q];
            unsigned long long m = 0;
            for (int k = lane; k < PIX_SB; k += 64) {
                const uint32_t blk = sb * PIX_SB + k;
                if (blk < t.nblocks) m = max(m, t.bmax[blk]);
            }
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) m = max(m, (unsigned long long)__shfl_xor(m, d));
            if (lane == 0) {
                t.sbmax[sb] = m;
                t.sbdirty[sb] = 0;
            }
        }
        // (their new maxima are read below by other waves of this block, on this CU: a
        // workgroup-scope fence, i.e. the stores complete before the barrier.  No other wave
        // loaded those lines in this launch, so no L1 line can be stale.  Agent-scope fences
        // here cost ~2 us each)
        __threadfence_block();
        __syncthreads();
    }
    if (tid == 0) {
        // counters of the previous merge (nothing else reads them now)
        ctl->n_sites = ctl->n_ent = ctl->n_dblocks = ctl->n_dsuper = 0;
        ctl->n_cand = 0;
        ctl->n_check = 0;
        ctl->merged = 0;   // (sharded: its delta rows were added by k_pix_apply_delta)
        n_lst = n_blk = n_cs = 0;
    }
    if (s_go == 1) {
        if (tid == 0) ctl->status = PIX_PAUSE;
        return;
    }
    unsigned long long m = 0;
    for (uint32_t i = tid; i < t.nsuper; i += 1024) m = max(m, t.sbmax[i]);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) m = max(m, (unsigned long long)__shfl_xor(m, d));
    if ((tid & 63) == 0) red[tid >> 6] = m;
    __syncthreads();
    unsigned long long best = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) best = max(best, red[i]);
    const long long W = (long long)(best >> 17);
    if (best == 0 || W < s_mw) {                                      // core.ts:312-313
        if (tid == 0) ctl->status = PIX_DONE;
        return;
    }
    // superblocks, then blocks, then slots holding the best key
    for (uint32_t i = tid; i < t.nsuper; i += 1024)
        if (t.sbmax[i] == best) {
            const uint32_t k = atomicAdd(&n_lst, 1u);
            if (k < 64) lst[k] = i;
        }
    __syncthreads();
    const uint32_t ns = min(n_lst, 64u);
    for (uint32_t q = 0; q < ns; ++q) {
        const uint32_t blk = lst[q] * PIX_SB + tid;
        if (tid < PIX_SB && blk < t.nblocks && t.bmax[blk] == best) {
            const uint32_t k = atomicAdd(&n_blk, 1u);
            if (k < 64) blks[k] = blk;
        }
    }
    __syncthreads();
    // the candidates gather in LDS with their keys and list lengths (a global counter that other
    // waves of this block add to while thread 0 has just stored it, then reads back, is not
    // ordered by the barrier: a candidate could be lost, and a tie with it)
    const uint32_t nbk = min(n_blk, 64u);
    for (uint32_t q = 0; q < nbk; ++q) {
        if (tid < PIX_B) {
            const uint32_t s = blks[q] * PIX_B + tid;
            if (pix_sel(t, s) == best) {
                const uint32_t k = atomicAdd(&n_cs, 1u);
                if (k < MAX_CAND) {
                    cs[k] = s;
                    cs_key[k] = t.keys[s];
                    cs_len[k] = t.len[s];
                }
            }
        }
    }
    __syncthreads();
    if (tid == 0) {
        const uint32_t nc = n_cs;
        ctl->n_cand = nc;
        if (n_lst > 64 || n_blk > 64 || nc > (uint32_t)MAX_CAND || nc == 0) {
            ctl->status = PIX_HOST;
            ctl->err = nc == 0 ? 10 : 4;
            return;
        }
        ctl->best = best;
        ctl->W = (unsigned long long)W;
        if (t.lane_w && t.lane_w < 64 && ((unsigned long long)W >> t.lane_w) != 0ull) {
            // (cannot happen while counts only fall: the lanes hold the last merge's W; a pause
            // before any shard makes the merge, alike on every shard, rather than a carry)
            ctl->status = PIX_PAUSE;
            ctl->lane_over = 1;
            return;
        }
        // (sorted by key: the shards of a sharded corpus index their tie words alike)
        for (uint32_t i = 1; i < nc; ++i)
            for (uint32_t j = i; j > 0 && cs_key[j - 1] > cs_key[j]; --j) {
                const uint32_t k0 = cs_key[j], s0 = cs[j], l0 = cs_len[j];
                cs_key[j] = cs_key[j - 1];
                cs[j] = cs[j - 1];
                cs_len[j] = cs_len[j - 1];
                cs_key[j - 1] = k0;
                cs[j - 1] = s0;
                cs_len[j - 1] = l0;
            }
        if (nc == 1) {
            pix_commit(t, ctl, cs[0], cs_key[0], cs_len[0]);
        } else {
            // tied: k_pix_sites scans the candidates' lists this iteration
            for (uint32_t j = 0; j < nc; ++j) {
                ctl->cand_slot[j] = cs[j];
                ctl->last[j] = 0;
            }
            ctl->tie_done = 0;
            ctl->tie = PIX_TIE_SCAN;
        }
    }
}

// The tie scan (k_pix_sites with tie == PIX_TIE_SCAN, the whole grid): the last valid slot of
// each candidate's list (atomicMax into ctl->last), then the last block to finish turns it into
// the last counted occurrence (for (x, x): the last valid slot at an even offset of its run) and
// the earliest of those wins (tie = PIX_TIE_DECIDED, pair_slot = the winner).
__device__ void pix_tie_scan(const PixCorpus &C, const PixTable &t, const PixBufs &B, PixCtl *ctl,
                             uint32_t nc) {
    __shared__ unsigned long long red[4];
    __shared__ bool last_block;
    for (uint32_t j = 0; j < nc; ++j) {
        const uint32_t s = ctl->cand_slot[j];
        const uint32_t key = t.keys[s];
        const int32_t u = (int32_t)(key >> 16), v = (int32_t)(key & 0xFFFF);
        const uint32_t off = t.off[s], len = t.len[s];
        unsigned long long m = 0;
        for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < len; i += gridDim.x * 256) {
            const uint32_t p = B.pool[off + i];
            if (C.tok[p] == u && pix_tok_is(C, C.nxt[p], v)) m = max(m, (unsigned long long)p + 1);
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) m = max(m, (unsigned long long)__shfl_xor(m, d));
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            m = max(max(red[0], red[1]), max(red[2], red[3]));
            if (m) atomicMax(&ctl->last[j], m);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        __threadfence();
        last_block = atomicAdd(&ctl->tie_done, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!(last_block && threadIdx.x == 0 && ctl->status == PIX_RUN)) return;
    __threadfence();
    unsigned long long bp = ~0ull;
    uint32_t bj = 0;
    for (uint32_t q = 0; q < nc; ++q) {
        unsigned long long m = atomicAdd(&ctl->last[q], 0ull);
        const uint32_t s = ctl->cand_slot[q];
        const int32_t u = (int32_t)(t.keys[s] >> 16), v = (int32_t)(t.keys[s] & 0xFFFF);
        if (m && u == v) {
            // offset of the last (x, x) slot in its run: odd -> the one before it is counted
            const uint32_t p = (uint32_t)(m - 1);
            uint32_t x = p;
            int k = 0;
            while (k <= PIX_WALK && pix_tok_is(C, C.prv[x], u)) {
                x = C.prv[x];
                ++k;
            }
            if (k > PIX_WALK) {
                pix_fail(ctl, 7);
                return;
            }
            if (k & 1) m = (unsigned long long)C.prv[p] + 1;
        }
        if (t.delta) {
            ctl->last[q] = m;   // (this shard's; the decision waits for the exchange)
            continue;
        }
        if (m && m < bp) {
            bp = m;
            bj = q;
        }
    }
    if (t.delta) {
        ctl->tie = PIX_TIE_WAIT;
        return;
    }
    if (bp == ~0ull) {
        ctl->status = PIX_ERROR;
        ctl->err = 8;
        return;
    }
    ctl->pair_slot = ctl->cand_slot[bj];
    ctl->tie = PIX_TIE_DECIDED;
}

// a != b: the count changes around each site p (q = next, l = prev of p, r = next of q).
//   left adjacency: chained to a site ending at l -> (b, a) is lost and (c, c) is counted by the
//   chain's head; else (l, a) -> (l, c), where l == a shortens a run of a's: one pair fewer when
//   that run had even length;
//   right adjacency (unless a site starts at r): (b, r) -> (c, r), likewise for a run of b's;
//   a chain of m consecutive sites becomes m c's: floor(m/2) pairs (c, c).
// (two lanes per site: the even one takes the left adjacency and the chain, the odd one the right
// adjacency; each writes its entry, [2 idx] / [2 idx + 1], or an empty one)
// (l = prv[p], tl its token, ll = prv[l]: loaded by the caller ahead of the site index)
__device__ void pix_site_left(const PixCorpus &C, const PixTable &t, const PixBufs &B,
                              PixCtl *ctl, uint32_t p, uint32_t q, uint32_t idx, int32_t a,
                              int32_t b, int32_t c, uint32_t l, int32_t tl, uint32_t ll) {
    // the two pairs this adjacency touches (k1 loses one, k2 is new), their first probes issued
    // together
    const bool chained = tl == b && pix_tok_is(C, ll, a);
    const uint32_t k1 = chained ? pix_key(b, a) : pix_key(tl, a);
    const uint32_t k2 = chained ? pix_key(c, c) : pix_key(tl, c);
    PixProbe p1{0, PIX_NONE}, p2{0, PIX_NONE};
    if (chained || tl >= 0) {
        p1 = pix_probe(t, k1);
        p2 = pix_probe(t, k2);
    }
    if (chained) {
        // chained to the site before: (b, a) is lost, (c, c) from that site's slot
        pix_add(t, B, ctl, k1, -1, p1);
        pix_entry(t, B, ctl, k2, ll, 0, 2 * idx, p2);
        return;
    }
    // the head of a chain: its length m, floor(m/2) pairs (c, c)
    uint32_t m = 1, xq = q;
    for (;;) {
        const uint32_t xr = C.nxt[xq];
        if (!pix_tok_is(C, xr, a)) break;
        const uint32_t xrq = C.nxt[xr];
        if (!pix_tok_is(C, xrq, b)) break;
        xq = xrq;
        if (++m > (uint32_t)PIX_WALK) {
            pix_fail(ctl, 14);
            return;
        }
    }
    if (tl >= 0) {
        if (tl == a) {
            // (k1 = (a, a): one fewer when the run of a's ending at l had even length)
            uint32_t L = 1, x = l;
            while (pix_tok_is(C, x, a)) {
                ++L;
                x = C.prv[x];
                if (L > (uint32_t)PIX_WALK) {
                    pix_fail(ctl, 13);
                    return;
                }
            }
            if ((L & 1u) == 0) pix_add(t, B, ctl, k1, -1, p1);
        } else {
            pix_add(t, B, ctl, k1, -1, p1);
        }
        pix_entry(t, B, ctl, k2, l, 1, 2 * idx, p2);
    } else if (2 * idx < B.ent_cap) {
        B.ent[2 * idx] = make_uint2(PIX_NONE, 0);
    }
    if (m >= 2) pix_add(t, B, ctl, c, c, (long long)(m / 2));
}

// (r = nxt[q], tr its token, rr = nxt[r]: loaded by the caller ahead of the site index)
__device__ void pix_site_right(const PixCorpus &C, const PixTable &t, const PixBufs &B,
                               PixCtl *ctl, uint32_t p, uint32_t q, uint32_t idx, int32_t a,
                               int32_t b, int32_t c, uint32_t r, int32_t tr, uint32_t rr) {
    // (a site starting at r takes this adjacency as its left one)
    const bool rchain = tr == a && pix_tok_is(C, rr, b);
    if (!rchain && tr >= 0) {
        const uint32_t k1 = pix_key(b, tr), k2 = pix_key(c, tr);   // (tr == b: k1 = (b, b))
        const PixProbe p1 = pix_probe(t, k1), p2 = pix_probe(t, k2);
        if (tr == b) {
            uint32_t L = 1, x = r;
            while (pix_tok_is(C, x, b)) {
                ++L;
                x = C.nxt[x];
                if (L > (uint32_t)PIX_WALK) {
                    pix_fail(ctl, 15);
                    return;
                }
            }
            if ((L & 1u) == 0) pix_add(t, B, ctl, k1, -1, p1);
        } else {
            pix_add(t, B, ctl, k1, -1, p1);
        }
        pix_entry(t, B, ctl, k2, p, 1, 2 * idx + 1, p2);
    } else if (2 * idx + 1 < B.ent_cap) {
        B.ent[2 * idx + 1] = make_uint2(PIX_NONE, 0);
    }
}

__device__ __forceinline__ void pix_push_site(const PixBufs &B, PixCtl *ctl, uint32_t p) {
    const uint32_t i = atomicAdd(&ctl->n_sites, 1u);
    if (i < B.site_cap) B.sites[i] = p;
    else pix_fail(ctl, 11);
}

// The merge sites and their count changes.  a != b: every valid slot of the (a, b) list, each
// with pix_site_delta.  a == b: the runs of a, each
// walked by the thread holding its head: sites at even offsets (replaceAll's left-to-right
// matches), and the run's count changes: L a's become floor(L/2) c's (+ a trailing a when L is
// odd), so (l, a) -> (l, c) on the left, (a, r) -> (c, r) on the right when L is even, (c, a)
// when L is odd, and floor(m/2) pairs (c, c) for the m c's.
__global__ void __launch_bounds__(256) k_pix_sites(PixCorpus C, PixTable t, PixBufs B, PixCtl *ctl) {
    __shared__ uint32_t s_run, s_len, s_tie;
    if (threadIdx.x == 0) {   // (read once and broadcast: the loop around the barriers is uniform)
        s_run = ctl->status == PIX_RUN;
        s_tie = s_run && ctl->tie == PIX_TIE_SCAN ? min(ctl->n_cand, (uint32_t)MAX_CAND) : 0u;
        s_len = s_run && !s_tie ? t.len[ctl->pair_slot] : 0u;
    }
    __syncthreads();
    if (!s_run) return;
    if (s_tie) {
        pix_tie_scan(C, t, B, ctl, s_tie);
        return;
    }
    const int32_t a = ctl->a, b = ctl->b, c = ctl->c;
    const uint32_t s = ctl->pair_slot;
    const uint32_t off = t.off[s], len = s_len;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // every (a, b) is merged (no count change below touches the pair itself)
        t.cnt[s] = 0;
        pix_mark(t, B, ctl, s);           // (it was the global max: its block is recomputed)
    }
    const int lane = threadIdx.x & 63;
    if (a != b) {
        // two lanes per list entry (pix_site_left / pix_site_right); one atomic per wave for the
        // site indices
        const uint64_t total = 2ull * len;
        const int role = lane & 1, wv = threadIdx.x >> 6;
        __shared__ uint32_t wcnt[4], bbase;
        for (uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x; g0 < total;
             g0 += (uint64_t)gridDim.x * blockDim.x) {
            const uint64_t g = g0 + threadIdx.x;
            uint32_t p = 0, q = PIX_NONE, x = PIX_NONE, xx = PIX_NONE;
            int32_t tx = SEP;
            bool valid = false;
            if (g < total) {
                // (every load the lane's adjacency needs, issued before the site index: the
                // neighbour x (prv[p] / nxt[q]), its token and its own neighbour xx)
                p = B.pool[off + (uint32_t)(g >> 1)];
                const int32_t tp = C.tok[p];
                q = C.nxt[p];
                if (role == 0) x = C.prv[p];
                const int32_t tq = q != PIX_NONE ? C.tok[q] : SEP;
                if (role == 1 && q != PIX_NONE) x = C.nxt[q];
                if (x != PIX_NONE) {
                    tx = C.tok[x];
                    xx = role == 0 ? C.prv[x] : C.nxt[x];
                }
                valid = tp == a && tq == b;
            }
            // one atomic per block for the site indices
            const unsigned long long m0 = __ballot(valid && role == 0);
            if (lane == 0) wcnt[wv] = (uint32_t)__popcll(m0);
            __syncthreads();
            if (threadIdx.x == 0) {
                const uint32_t tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
                bbase = tot ? atomicAdd(&ctl->n_sites, tot) : 0;
            }
            __syncthreads();
            uint32_t base = bbase;
            for (int w = 0; w < wv; ++w) base += wcnt[w];
            __syncthreads();
            if (!valid) continue;
            const uint32_t idx = base + (uint32_t)__popcll(m0 & ((1ull << (lane & ~1)) - 1));
            if (idx >= B.site_cap) {
                pix_fail(ctl, 11);
                continue;
            }
            if (role == 0) {
                B.sites[idx] = p;
                pix_site_left(C, t, B, ctl, p, q, idx, a, b, c, x, tx, xx);
            } else {
                pix_site_right(C, t, B, ctl, p, q, idx, a, b, c, x, tx, xx);
            }
        }
        return;
    }
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < len; i += gridDim.x * blockDim.x) {
        const uint32_t p = B.pool[off + i];
        const bool valid = C.tok[p] == a && pix_tok_is(C, C.nxt[p], b);
        if (!valid) continue;
        const uint32_t l = C.prv[p];
        if (pix_tok_is(C, l, a)) continue;             // not the head of its run
        // walk the run: s_0 = p, s_1, ...; sites at even offsets followed by another a
        uint32_t cur = p, prev_site = PIX_NONE;
        uint32_t k = 0;
        unsigned long long m = 0;
        for (;;) {
            const uint32_t nx = C.nxt[cur];
            if (!pix_tok_is(C, nx, a)) break;
            if ((k & 1u) == 0) {
                pix_push_site(B, ctl, cur);
                if (prev_site != PIX_NONE) pix_entry(t, B, ctl, c, c, prev_site, 0);
                prev_site = cur;
                ++m;
            }
            cur = nx;
            if (++k > (uint32_t)PIX_WALK) {
                pix_fail(ctl, 12);
                return;
            }
        }
        const uint32_t L = k + 1;                       // run length (cur = its last slot)
        atomicAdd(&ctl->n_check, m);
        if (l != PIX_NONE && C.tok[l] >= 0) {
            pix_add(t, B, ctl, C.tok[l], a, -1);
            pix_entry(t, B, ctl, C.tok[l], c, l, 1);
        }
        if (m >= 2) pix_add(t, B, ctl, c, c, (long long)(m / 2));
        if (L & 1u) {
            pix_entry(t, B, ctl, c, a, prev_site, 1);   // the trailing a
        } else {
            const uint32_t r = C.nxt[cur];
            if (r != PIX_NONE && C.tok[r] >= 0) {
                pix_add(t, B, ctl, a, C.tok[r], -1);
                pix_entry(t, B, ctl, c, C.tok[r], prev_site, 1);
            }
        }
    }
}

constexpr int PIX_VOTE = MAX_CAND;       // tie word of the hand-off vote (BPE_TIE_WORDS >= 17)
__device__ void pix_decide(PixCtl *ctl, const unsigned long long *__restrict__ tie);

// Segments for this merge's new pairs, from their owner entries (one pool atomic per block), and
// the new pairs' maxima: their counts are final now.
// A shard of a sharded corpus (tie != nullptr): block 0 first makes k_pix_decide's decision from
// the all-reduced tie words (one launch fewer per iteration, round 5).  Every block reads the
// vote from the tie words itself (block 0 may not have written the status yet); a tie scan's
// iteration (ctl->tie WAIT, then DECIDED) makes no merge either way.
__global__ void __launch_bounds__(256) k_pix_alloc(PixTable t, PixBufs B, PixCtl *ctl,
                                                   const unsigned long long *__restrict__ tie = nullptr) {
    __shared__ unsigned long long wsum[4], wown[4], base_s;
    __shared__ uint32_t s_ne;
    if (threadIdx.x == 0) {   // (read once and broadcast: the loop around the barriers is uniform)
        if (tie && blockIdx.x == 0) pix_decide(ctl, tie);
        const bool vote = tie && tie[PIX_VOTE];
        s_ne = vote || ctl->status != PIX_RUN || ctl->tie != PIX_TIE_NONE
                   ? 0u
                   : min(ctl->a != ctl->b ? 2 * ctl->n_sites : ctl->n_ent, B.ent_cap);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t ne = s_ne;
    for (uint32_t i0 = blockIdx.x * 256; i0 < ne; i0 += gridDim.x * 256) {
        const uint32_t i = i0 + threadIdx.x;
        uint2 e = make_uint2(PIX_NONE, 0);
        if (i < ne) e = B.ent[i];
        const bool own = e.x != PIX_NONE && (e.x & PIX_OWNER);
        const unsigned long long len = own ? t.len[e.x & ~PIX_OWNER] : 0;
        unsigned long long incl = len;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long o = __shfl_up(incl, d);
            if (lane >= d) incl += o;
        }
        const unsigned long long nown = __popcll(__ballot(own));
        if (lane == 63) {
            wsum[wv] = incl;
            wown[wv] = nown;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned long long tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
            const unsigned long long no = wown[0] + wown[1] + wown[2] + wown[3];
            base_s = tot ? atomicAdd(&ctl->pool_top, tot) : 0;
            if (no) atomicAdd(&ctl->used, no);
        }
        __syncthreads();
        unsigned long long o = base_s + incl - len;
        for (int w = 0; w < wv; ++w) o += wsum[w];
        __syncthreads();
        if (!own) continue;
        if (o + len > ctl->pool_cap) {
            pix_fail(ctl, 16);
            continue;
        }
        const uint32_t s = e.x & ~PIX_OWNER;
        t.off[s] = (uint32_t)o;
        t.fill[s] = 0;
        if (t.delta) continue;   // (sharded: the counts and maxima move in k_pix_apply_delta)
        const unsigned long long sel = pix_sel(t, s);
        const uint32_t blk = s / PIX_B;
        if (sel > t.bmax[blk]) {
            atomicMax(&t.bmax[blk], sel);
            atomicMax(&t.sbmax[blk / PIX_SB], sel);
        }
    }
    // The blocks whose max fell (the counts are final after k_pix_sites, and c's length was set
    // by pix_commit).  A new pair lifted above keeps its block's max either way: the recompute
    // reads its final count, so its store is >= the lift.  (No merge, no dirty block: k_pix_select
    // zeroes n_dblocks.)
    if (!t.delta) pix_bmax_dirty(t, B, ctl, gridDim.x - 1 - blockIdx.x);
}

// The corpus rewrite: c at every site, its right slot merged away, the links around it; the new
// pairs' slots into their segments.  The merge is then logged;
// W must equal the sites found.
__global__ void __launch_bounds__(256) k_pix_apply(PixCorpus C, PixTable t, PixBufs B, PixCtl *ctl,
                                                   long long *log) {
    if (ctl->status != PIX_RUN || ctl->tie != PIX_TIE_NONE) return;   // (a tie scan: no merge)
    const unsigned long long W = ctl->W;
    // (sharded: this shard's sites; their sum over the shards is checked against W by
    // k_pix_apply_delta)
    const unsigned long long nw = t.delta ? ctl->n_sites : W;
    if (ctl->n_sites != nw || (ctl->a == ctl->b && ctl->n_check != nw)) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            ctl->status = PIX_ERROR;
            ctl->err = 20;
        }
        return;
    }
    const int32_t c = ctl->c;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
    for (uint32_t i = tid; i < (uint32_t)nw; i += stride) {
        const uint32_t p = B.sites[i];
        const uint32_t q = C.nxt[p];
        const uint32_t r = C.nxt[q];
        C.tok[p] = c;
        C.tok[q] = TOMB;
        C.nxt[p] = r;
        if (r != PIX_NONE) C.prv[r] = p;
    }
    // (a != b: two entries per site, some empty; a == b: packed)
    const uint32_t ne = min(ctl->a != ctl->b ? 2 * (uint32_t)nw : ctl->n_ent, B.ent_cap);
    for (uint32_t i = tid; i < ne; i += stride) {
        const uint2 e = B.ent[i];
        if (e.x == PIX_NONE) continue;
        const uint32_t sl = e.x & ~PIX_OWNER;
        const uint32_t k = atomicAdd(&t.fill[sl], 1u);
        B.pool[t.off[sl] + k] = e.y;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const long long k = ctl->n_done;
        log[PIX_LOG * k] = ctl->a;
        log[PIX_LOG * k + 1] = ctl->b;
        log[PIX_LOG * k + 2] = (long long)W;
        log[PIX_LOG * k + 3] = (long long)nw;   // (this shard's replacements)
        ctl->n_done = k + 1;
        ctl->next_id = c + 1;
        ctl->merged = t.delta ? 1u : 0u;
    }
}

// The dense corpus back from the slot array: its live slots (tokens and SEPs) in order.  Per
// block of PB slots the live count (k_pix_live_count), an exclusive sum over the blocks
// (k_pix_scan_sum), then each block writes its live slots at its offset (k_pix_live_scatter).
__global__ void __launch_bounds__(256) k_pix_live_count(const int32_t *__restrict__ tok, uint32_t n,
                                                        uint32_t *__restrict__ cnt) {
    __shared__ uint32_t red[4];
    const uint32_t nblk = (n + PB - 1) / PB;
    for (uint32_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        uint32_t c = 0;
        for (uint32_t i = blk * PB + threadIdx.x; i < min(blk * PB + PB, n); i += 256)
            c += tok[i] >= SEP;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
        __syncthreads();
        if (threadIdx.x == 0) cnt[blk] = red[0] + red[1] + red[2] + red[3];
        __syncthreads();
    }
}

__global__ void __launch_bounds__(256) k_pix_live_scatter(const int32_t *__restrict__ tok, uint32_t n,
                                                          const uint32_t *__restrict__ off,
                                                          int32_t *__restrict__ out) {
    __shared__ uint32_t wsum[4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t nblk = (n + PB - 1) / PB;
    for (uint32_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        uint32_t o = off[blk];
        for (uint32_t j0 = blk * PB; j0 < min(blk * PB + PB, n); j0 += 256) {
            const uint32_t i = j0 + threadIdx.x;
            const int32_t v = i < n ? tok[i] : TOMB;
            const bool live = v >= SEP;
            const unsigned long long m = __ballot(live);
            if (lane == 0) wsum[wv] = (uint32_t)__popcll(m);
            __syncthreads();
            uint32_t b = o;
            for (int w = 0; w < wv; ++w) b += wsum[w];
            if (live) out[b + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = v;
            o += wsum[0] + wsum[1] + wsum[2] + wsum[3];
            __syncthreads();
        }
    }
}

// ---- a shard of a sharded corpus: the index inside the rank loop (include/bpe.h bpe_rank_loop_*) --
// Every shard indexes its own samples (pairs never cross samples, core.ts:265-267) and holds the
// GLOBAL count of every pair in its table, so every shard selects the same merge.  Per iteration,
// on each shard's stream, between the caller's two all-reduces:
//   [all-reduce(SUM) of the exchange: the last merge's delta rows]
//   rank_loop_select   k_pix_apply_delta (the summed rows into the counts, the replacement check),
//                      k_pix_dirty, k_pix_select, k_pix_sites (this shard's sites and count changes
//                      into its delta rows; or the tie scan), k_pix_export (tie words and vote)
//   [all-reduce(MAX) of the tie words]
//   rank_loop_decide   nothing (round 5: its decision is the first thing k_pix_alloc does)
//   rank_loop_count    k_pix_alloc: pix_decide in block 0 (a vote hands the iteration to the host
//                      on every shard alike; a tie goes to the earliest (shard << 40 | last
//                      counted occurrence)), then the new pairs' segments; k_pix_apply (this
//                      shard's corpus and lists)

// the batch: n iterations (each a merge or a tie scan) from vocabulary id next_id on
__global__ void k_pix_rank_begin(PixCtl *ctl, long long n, int32_t next_id, long long min_weight) {
    if (ctl->status == PIX_PAUSE) ctl->status = PIX_RUN;
    ctl->n_done = 0;
    ctl->n_want = n;
    ctl->next_id = next_id;
    ctl->min_weight = min_weight;
}

// One summed count change into this shard's global counts: a fall marks the block when the entry
// was its max, a rise (only pairs with c rise) lifts the block and superblock maxima; a pair new to
// this shard gets a slot (no list here).
__device__ __forceinline__ void pix_global_add(const PixTable &t, const PixBufs &B, PixCtl *ctl,
                                               uint32_t key, unsigned long long v) {
    const bool rise = (long long)v > 0;
    const uint32_t s = pix_slot(t, ctl, key, rise, true);
    if (s == PIX_NONE) {   // (a fall of a pair no shard holds: the tables disagree)
        if (rise) pix_fail(ctl, 1);
        else if (atomicCAS(&ctl->status, PIX_RUN, PIX_ERROR) == PIX_RUN) ctl->err = 22;
        return;
    }
    const unsigned long long bm = t.bmax[s / PIX_B];
    const unsigned long long old = atomicAdd(&t.cnt[s], v);
    if (rise) {
        const unsigned long long sel = pix_sel_of(t, key, old + v);
        const uint32_t blk = s / PIX_B;
        if (sel > bm) {
            atomicMax(&t.bmax[blk], sel);
            atomicMax(&t.sbmax[blk / PIX_SB], sel);
        }
    } else {
        const unsigned long long sel = pix_sel_of(t, key, old);
        if (sel && sel >= bm) pix_mark(t, B, ctl, s);
    }
}

// The summed exchange of the last merge (a, b) -> c into this shard's global counts.  The words
// read are zeroed for this iteration's own changes; the header's first word, the shards'
// replacements summed, must equal W.
__global__ void __launch_bounds__(256) k_pix_apply_delta(PixTable t, PixBufs B, PixCtl *ctl,
                                                         unsigned long long *__restrict__ xchg) {
    __shared__ uint32_t s_go;
    if (threadIdx.x == 0) s_go = ctl->status == PIX_RUN && ctl->merged;
    __syncthreads();
    if (!s_go) return;
    const int32_t a = ctl->a, b = ctl->b, c = ctl->c;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const unsigned long long got = xchg[0];
        if (got != ctl->W) {
            ctl->status = PIX_ERROR;
            ctl->err = 21;
            ctl->n_check = got;
        }
    }
    unsigned long long *d = xchg + XCHG_HDR;
    if (t.lane_w) {
        // lanes: a thread per special word, then per token id <= c and side: its lane (cleared
        // with an atomic AND, since other threads read the other lanes of the word), n = the sites
        // with that neighbour: the left side loses (o, a) and gains (o, c), the right side loses
        // (b, o) and gains (c, o)
        const uint32_t nid = (uint32_t)c + 1u;
        const uint32_t n = PIX_XCHG_SPECIAL + 2u * nid;
        const unsigned long long mask = t.lane_w >= 64 ? ~0ull : (1ull << t.lane_w) - 1ull;
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
            if (i < PIX_XCHG_SPECIAL) {
                if (i >= 9) continue;   // (never written)
                const unsigned long long v = d[i];
                if (!v) continue;
                d[i] = 0;
                const int32_t abc[3] = {a, b, c};
                pix_global_add(t, B, ctl, pix_key(abc[i / 3], abc[i % 3]), v);
                continue;
            }
            const uint32_t k = i - PIX_XCHG_SPECIAL;
            const int side = k >= nid;
            const int32_t o = (int32_t)(side ? k - nid : k);
            uint32_t shift;
            unsigned long long *p = d + PIX_XCHG_SPECIAL + lane_word(t, side, (uint32_t)o, shift);
            const unsigned long long cnt = (*p >> shift) & mask;
            if (!cnt) continue;
            if (t.lane_q == 1) *p = 0;
            else atomicAnd(p, ~(mask << shift));
            pix_global_add(t, B, ctl, side ? pix_key(b, o) : pix_key(o, a), (unsigned long long)-(long long)cnt);
            pix_global_add(t, B, ctl, side ? pix_key(c, o) : pix_key(o, c), cnt);
        }
    } else {
        // dense rows: every token id <= c
        const uint32_t n = (uint32_t)DELTA_ROWS * (uint32_t)(c + 1);
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
            const unsigned long long v = d[i];
            if (!v) continue;
            d[i] = 0;
            const uint32_t row = i % DELTA_ROWS;
            const int32_t o = (int32_t)(i / DELTA_ROWS);
            const int32_t m = row == 0 || row == 2 ? a : row == 1 || row == 3 ? b : c;
            const bool left = row == 0 || row == 1 || row == 4;   // (m, o), else (o, m)
            pix_global_add(t, B, ctl, pix_key(left ? m : o, left ? o : m), v);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) xchg[0] = 0;
}

// The blocks whose max entry fell (marked by k_pix_sites and k_pix_apply_delta)
__global__ void __launch_bounds__(256) k_pix_dirty(PixTable t, PixBufs B, PixCtl *ctl) {
    pix_bmax_dirty(t, B, ctl, blockIdx.x);
}

// This iteration's exchange words: this shard's sites of the merge (the header's first word; the
// rows hold its count changes), the tie scan's last counted occurrences as (shard << 40 | position)
// and the hand-off vote.  Every tie word is written, each iteration.
__global__ void k_pix_export(PixCtl *ctl, unsigned long long *__restrict__ xchg,
                             unsigned long long *__restrict__ tie, int rank) {
    const int i = threadIdx.x;
    if (i == 0 && ctl->status == PIX_RUN && ctl->tie == PIX_TIE_NONE) {
        // the pool must take this merge's new entries (k_pix_alloc): a shard that cannot votes
        // now, before any shard applies the merge
        const unsigned long long ne = ctl->a != ctl->b ? 2ull * ctl->n_sites : ctl->n_ent;
        if (ctl->pool_top + ne > ctl->pool_cap) {
            ctl->status = PIX_HOST;
            ctl->err = 16;
        }
    }
    __syncthreads();
    const int st = ctl->status;
    if (i < MAX_CAND) {
        const unsigned long long m = ctl->tie == PIX_TIE_WAIT && i < (int)ctl->n_cand ? ctl->last[i] : 0;
        tie[i] = m ? ((unsigned long long)rank << 40) | m : 0ull;
    } else if (i == PIX_VOTE) {
        tie[i] = st == PIX_HOST ? 1ull : 0ull;
    } else if (i < 32) {
        tie[i] = 0;
    }
    if (i == 0) xchg[0] = st == PIX_RUN && ctl->tie == PIX_TIE_NONE ? ctl->n_sites : 0u;
}

// After the all-reduce(MAX) of the tie words, alike on every shard: a vote hands the iteration to
// the host (the corpus is still the last merge's: k_pix_apply has not run), a tie scan's winner is
// the candidate whose last counted occurrence is earliest (R3, core.ts:294-305), committed by the
// next k_pix_select.
__device__ void pix_decide(PixCtl *ctl, const unsigned long long *__restrict__ tie) {
    if (ctl->status == PIX_ERROR || ctl->status == PIX_DONE || ctl->status == PIX_PAUSE) return;
    if (tie[PIX_VOTE]) {
        if (ctl->status == PIX_RUN) {
            ctl->status = PIX_HOST;
            ctl->err = 30;
        }
        return;
    }
    if (ctl->status != PIX_RUN || ctl->tie != PIX_TIE_WAIT) return;
    unsigned long long bp = ~0ull;
    uint32_t bj = 0;
    for (uint32_t q = 0; q < min(ctl->n_cand, (uint32_t)MAX_CAND); ++q)
        if (tie[q] && tie[q] < bp) {
            bp = tie[q];
            bj = q;
        }
    if (bp == ~0ull) {
        ctl->status = PIX_ERROR;
        ctl->err = 8;
        return;
    }
    ctl->pair_slot = ctl->cand_slot[bj];
    ctl->tie = PIX_TIE_DECIDED;
}

// The global counts into a freshly built index (bpe_set_global_counts): the hot bins of the summed
// table and every shard's cold (key, count) entries (duplicates summed), over counts zeroed first;
// a pair no list of this shard holds gets a slot.
__global__ void __launch_bounds__(256) k_pix_load_global(PixTable t, PixCtl *ctl,
                                                         const unsigned long long *__restrict__ hot,
                                                         const uint32_t *__restrict__ keys,
                                                         const unsigned long long *__restrict__ counts,
                                                         int64_t n) {
    const int64_t total = (int64_t)HOT_BINS + n;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t key;
        unsigned long long v;
        if (i < HOT_BINS) {
            v = hot[i];
            const uint32_t x = (uint32_t)i & 255u, y = (uint32_t)i >> 8;   // (hot_bin: y << 8 | x)
            key = pix_key((int32_t)x, (int32_t)y);
        } else {
            key = keys[i - HOT_BINS];
            v = counts[i - HOT_BINS];
        }
        if (!v || key == PIX_NONE) continue;
        const uint32_t s = pix_slot(t, ctl, key, true, true);
        if (s == PIX_NONE) {
            atomicOr(&ctl->err, 9);
            continue;
        }
        atomicAdd(&t.cnt[s], v);
    }
}

// Growth in place, between batches (pix_reserve): every claimed pair into a table twice as large,
// with its count and its list; the block maxima are then recomputed in full.
__global__ void __launch_bounds__(256) k_pix_rehash(PixTable o, PixTable t, PixCtl *ctl, uint32_t ocap) {
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < ocap; s += gridDim.x * blockDim.x) {
        const uint32_t key = o.keys[s];
        if (key == PIX_NONE) continue;
        const uint32_t ns = pix_slot(t, ctl, key, true, false);
        if (ns == PIX_NONE) {
            atomicOr(&ctl->err, 9);
            continue;
        }
        t.cnt[ns] = o.cnt[s];
        t.off[ns] = o.off[s];
        t.len[ns] = o.len[s];
        t.fill[ns] = o.fill[s];
    }
}

}  // namespace bpe
