// bpe_kernels.hip.h — CDNA4 (gfx950) kernels of the BPE merge-training hot path.
//
// Reference semantics: /root/reference/core.ts findNextMerge (247-326) and applyMerge (332-360);
// order-free restatement in SURVEY.md Appendix A (R1-R5).
//
// Corpus layout in HBM: one flat int32 slot array.  Every sample (one `corpus_in_code` element,
// core.ts:106) is stored as its token ids followed by one SEP (-1) slot.  The array is padded with
// SEP to a whole number of 256-slot chunks plus one spare chunk, so a chunk's "next token" load is
// always in bounds.
//
// Work decomposition: the chunks are cut into R contiguous *regions*; one wave (64 lanes) owns
// one region and streams it chunk by chunk (lane L holds slots 4L..4L+3 of the chunk as one int4
// — a 1 KiB fully coalesced load per wave-instruction).  The only state crossing chunk
// boundaries is the open run of equal tokens (needed for the `X X X` skip rule, core.ts:285-290);
// it is carried in wave-uniform registers inside a region and resolved between regions by k_runs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bpe {

constexpr int32_t SEP = -1;
constexpr int CHUNK = 256;                  // slots per wave-chunk (64 lanes x int4)
constexpr int WAVES_PER_WG = 16;
constexpr int WG = WAVES_PER_WG * 64;       // 1024 threads, one workgroup per CU (LDS-bound)
constexpr int MAX_WG = 256;                 // one per CU on MI355X
constexpr int MAX_REGIONS = MAX_WG * WAVES_PER_WG;
constexpr int HOT = 256;                    // ids < HOT form the dense LDS histogram
constexpr int HOT_BINS = HOT * HOT;
constexpr int HIST_WORDS = HOT_BINS / 2;    // two 16-bit counters per LDS dword (128 KiB)
constexpr int MAX_CAND = 16;               // candidates resolved per tie pass
constexpr int CAND_CAP = 65536;             // candidates collected per iteration
constexpr uint32_t EMPTY = 0xFFFFFFFFu;

struct RegionRun {
    int64_t head_len;   // leading slots equal to the token before the region (continued run)
    int64_t tail_len;   // length (inside the region) of a run still open at the region end
    int32_t tail_x;     // token of that open run, -1 when none
    int32_t uniform;    // 1 when the whole region continues the previous region's run
};

// Sparse pair table for pairs with an id >= HOT: open addressing on key = a << 16 | b.
struct ColdTable {
    uint32_t *keys;
    uint32_t *counts;
    uint32_t *used;      // slots claimed this pass (for clearing and for argmax)
    uint32_t *n_used;
    uint32_t *overflow;  // set when a probe sequence wraps the table (capacity bug guard)
    uint32_t mask;
    uint32_t shift;
};

struct Result {
    unsigned long long best;     // packed (W << 17) | (0x1FFFF - c_index), 0 = no pair
    unsigned int n_cand;                 // pairs sharing the best packed key (list in `cand`)
    unsigned int pad0;
    unsigned long long last[MAX_CAND];   // R3: position + 1 of the last counted occurrence
    unsigned long long replaced;         // apply: replacement count
    unsigned long long kept_total;       // apply: slots after compaction
};

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

__device__ __forceinline__ void cold_add(const ColdTable &ct, uint32_t key, uint32_t inc) {
    uint32_t h = (key * 0x9E3779B1u) >> ct.shift;
    for (uint32_t probes = 0;; ++probes) {
        if (probes > ct.mask) {
            atomicOr(ct.overflow, 1u);
            return;
        }
        uint32_t k = __hip_atomic_load(&ct.keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == key) {
            atomicAdd(&ct.counts[h], inc);
            return;
        }
        if (k == EMPTY) {
            uint32_t old = atomicCAS(&ct.keys[h], EMPTY, key);
            if (old == EMPTY) {
                uint32_t i = atomicAdd(ct.n_used, 1u);
                ct.used[i] = h;
                atomicAdd(&ct.counts[h], inc);
                return;
            }
            if (old == key) {
                atomicAdd(&ct.counts[h], inc);
                return;
            }
        }
        h = (h + 1) & ct.mask;
    }
}

// Adds n to count(x, x) for a run resolved outside the LDS histogram.
__device__ __forceinline__ void add_run_pairs(int32_t x, unsigned long long n,
                                              unsigned long long *spill, const ColdTable &ct) {
    if (n == 0) return;
    if (x < HOT) atomicAdd(&spill[x * HOT + x], n);
    else cold_add(ct, ((uint32_t)x << 16) | (uint32_t)x, (uint32_t)n);
}

// One counted occurrence of (x, y).  Hot pairs go to the workgroup's packed 16-bit LDS counters;
// a counter reaching 0x8000 spills 0x8000 to the global u64 spill table (exactly one lane
// observes each 0x7FFF -> 0x8000 transition, so nothing is lost or double counted).
__device__ __forceinline__ void count_pair(uint32_t *hist, int32_t x, int32_t y,
                                           unsigned long long *spill, const ColdTable &ct) {
    if ((uint32_t)x < HOT && (uint32_t)y < HOT) {
        const int bin = x * HOT + y;
        const uint32_t sh = (bin & 1) << 4;
        const uint32_t old = atomicAdd(&hist[bin >> 1], 1u << sh);
        if (((old >> sh) & 0xFFFFu) == 0x7FFFu) {
            atomicSub(&hist[bin >> 1], 0x8000u << sh);
            atomicAdd(&spill[bin], 0x8000ull);
        }
    } else {
        cold_add(ct, ((uint32_t)x << 16) | (uint32_t)y, 1u);
    }
}

// Per-chunk neighbourhood of one lane: t[0..3] its slots, t[4] the next slot, pm the previous.
struct Chunk {
    int32_t t[5];
    bool eqn[4];   // t[e] == t[e+1], non-SEP  (an X X pair at e)
    bool eqp[4];   // t[e] == t[e-1], non-SEP  (e continues a run)
};

__device__ __forceinline__ void load_chunk(Chunk &ck, const int4 v, int32_t nxt, int32_t prev,
                                           int lane) {
    const int32_t up = __shfl_up(v.w, 1);
    const int32_t dn = __shfl_down(v.x, 1);
    ck.t[0] = v.x;
    ck.t[1] = v.y;
    ck.t[2] = v.z;
    ck.t[3] = v.w;
    ck.t[4] = lane == 63 ? nxt : dn;
    const int32_t pm = lane == 0 ? prev : up;
    ck.eqp[0] = ck.t[0] == pm && ck.t[0] != SEP;
#pragma unroll
    for (int e = 1; e < 4; ++e) ck.eqp[e] = ck.t[e] == ck.t[e - 1] && ck.t[e] != SEP;
#pragma unroll
    for (int e = 0; e < 4; ++e) ck.eqn[e] = ck.t[e] == ck.t[e + 1] && ck.t[e] != SEP;
}

// Run-start scan: rs[e] = chunk index of the start of the run containing slot 4*lane+e, or -1
// when that run began before the chunk.  Returns rs of slot 255 (broadcast).
__device__ __forceinline__ int run_starts(const Chunk &ck, int lane, int rs[4]) {
    int lmax = -1;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        if (!ck.eqp[e]) lmax = 4 * lane + e;
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
    for (int e = 0; e < 4; ++e) rs[e] = rs[e] > excl ? rs[e] : excl;
    return __shfl(rs[3], 63);
}

__device__ __forceinline__ int first_start(const Chunk &ck) {
    int f = CHUNK;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        unsigned long long m = __ballot(!ck.eqp[e]);
        if (m) {
            int k = 4 * __builtin_ctzll(m) + e;
            f = k < f ? k : f;
        }
    }
    return f;
}

// ---------------------------------------------------------------------------------------------
// K1 pair count.  Counts every counted occurrence (R1) of every pair: hot pairs in LDS, cold
// pairs in the sparse table.  X X pairs of runs that cross a chunk boundary are deferred and
// added once when the run closes (floor(L/2), ≡ the skip rule core.ts:285-290); runs crossing a
// region boundary are summarised in `runs` and resolved by k_runs.
// ---------------------------------------------------------------------------------------------
template <bool FILTER>
__global__ void __launch_bounds__(WG)
k_count(const int32_t *__restrict__ ids, int64_t n_chunks, int64_t cpr, int R,
        const int32_t *__restrict__ len16, int64_t max_length, uint32_t *__restrict__ partials,
        unsigned long long *__restrict__ spill, ColdTable ct, RegionRun *__restrict__ runs) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
    {
        uint4 *h4 = reinterpret_cast<uint4 *>(hist);
        for (int i = threadIdx.x; i < HIST_WORDS / 4; i += WG) h4[i] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * WAVES_PER_WG + (threadIdx.x >> 6);
    if (r < R) {
        const int64_t c0 = (int64_t)r * cpr;
        const int64_t c1 = min(c0 + cpr, n_chunks);
        const int4 *v4 = reinterpret_cast<const int4 *>(ids);
        int32_t prev = c0 > 0 ? ids[c0 * CHUNK - 1] : SEP;
        // open run carried across chunks (wave-uniform).  Initially a pseudo-run continuing the
        // previous region's last token; it closes at once when the region starts a new run.
        int32_t run_x = prev >= 0 ? prev : -2;
        int64_t run_len = 0;
        bool run_cont = true;
        int64_t head_len = 0;
        int4 vnext = v4[c0 * 64 + lane];
        for (int64_t c = c0; c < c1; ++c) {
            const int4 v = vnext;
            if (c + 1 < c1) vnext = v4[(c + 1) * 64 + lane];
            const int32_t nxt = ids[(c + 1) * CHUNK];
            Chunk ck;
            load_chunk(ck, v, nxt, prev, lane);
            prev = __shfl(v.w, 63);
            bool slow = false;
#pragma unroll
            for (int e = 0; e < 4; ++e) slow |= ck.eqn[e] && ck.eqp[e];
            slow |= (lane == 63 && ck.eqn[3]) || (lane == 0 && ck.eqp[0]);
            bool counted[4];
            if (__ballot(slow) == 0ull) {
                // fast path: every X X pair starts a run of exactly two -> counted
#pragma unroll
                for (int e = 0; e < 4; ++e) counted[e] = ck.t[e] >= 0 && ck.t[e + 1] >= 0;
                run_x = -2;
                run_len = 0;
                run_cont = false;
            } else {
                int rs[4];
                const int rs_last = run_starts(ck, lane, rs);
                const bool end_open = __shfl((int)ck.eqn[3], 63) != 0;
                const int f = first_start(ck);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    bool ok = ck.t[e] >= 0 && ck.t[e + 1] >= 0;
                    if (ok && ck.eqn[e]) {
                        const int k = 4 * lane + e;
                        if (rs[e] < 0) ok = false;                          // carried run
                        else if (end_open && rs[e] == rs_last) ok = false;  // open tail run
                        else ok = ((k - rs[e]) & 1) == 0;
                    }
                    counted[e] = ok;
                }
                if (run_x != -2) {
                    int64_t L = -1;
                    if (f < CHUNK) L = run_len + f;
                    else if (!end_open) L = run_len + CHUNK;
                    else run_len += CHUNK;
                    if (L >= 0) {
                        if (run_cont) {
                            head_len = L;
                        } else if (lane == 0 && L >= 2 &&
                                   (!FILTER || 2 * (int64_t)len16[run_x] <= max_length)) {
                            add_run_pairs(run_x, (unsigned long long)(L >> 1), spill, ct);
                        }
                        run_x = -2;
                        run_len = 0;
                        run_cont = false;
                    }
                }
                if (run_x == -2 && end_open) {
                    run_x = __shfl(ck.t[3], 63);
                    run_len = CHUNK - rs_last;
                    run_cont = false;
                }
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (!counted[e]) continue;
                const int32_t x = ck.t[e], y = ck.t[e + 1];
                if (FILTER && (int64_t)len16[x] + len16[y] > max_length) continue;
                count_pair(hist, x, y, spill, ct);
            }
        }
        if (lane == 0) {
            RegionRun rr;
            if (run_x != -2) {
                rr.tail_x = run_x;
                rr.tail_len = run_len;
                rr.uniform = run_cont ? 1 : 0;
                rr.head_len = run_cont ? run_len : head_len;
            } else {
                rr.tail_x = -1;
                rr.tail_len = 0;
                rr.uniform = 0;
                rr.head_len = head_len;
            }
            runs[r] = rr;
        }
    }
    __syncthreads();
    uint4 *out = reinterpret_cast<uint4 *>(partials + (size_t)blockIdx.x * HIST_WORDS);
    const uint4 *h4 = reinterpret_cast<const uint4 *>(hist);
    for (int i = threadIdx.x; i < HIST_WORDS / 4; i += WG) out[i] = h4[i];
}

// Resolves runs that cross region boundaries: the run offset at each region start (for the
// exact passes) and floor(L/2) X X pairs of every crossing run (for the count).
__global__ void k_runs(const RegionRun *__restrict__ runs, int R, int64_t *__restrict__ carry_off,
                       const int32_t *__restrict__ len16, int64_t max_length, int filter,
                       unsigned long long *__restrict__ spill, ColdTable ct, int add_counts) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    const RegionRun me = runs[r];
    int64_t off = 0;
    if (me.head_len > 0) {
        for (int q = r - 1; q >= 0; --q) {
            off += runs[q].tail_len;
            if (!runs[q].uniform) break;
        }
    }
    carry_off[r] = off;
    if (add_counts && me.tail_x >= 0 && !me.uniform) {
        int64_t L = me.tail_len;
        int q = r + 1;
        while (q < R && runs[q].uniform) L += runs[q].tail_len, ++q;
        if (q < R) L += runs[q].head_len;
        const int32_t x = me.tail_x;
        if (L >= 2 && (!filter || 2 * (int64_t)len16[x] <= max_length))
            add_run_pairs(x, (unsigned long long)(L >> 1), spill, ct);
    }
}

// Sums the per-workgroup packed LDS partials and the spill table into u64 hot counts.
__global__ void k_reduce_hot(const uint32_t *__restrict__ partials, int G,
                             const unsigned long long *__restrict__ spill,
                             unsigned long long *__restrict__ hot_counts) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= HIST_WORDS) return;
    unsigned long long lo = 0, hi = 0;
    int g = 0;
    for (; g + 4 <= G; g += 4) {
        uint32_t p0 = partials[(size_t)(g + 0) * HIST_WORDS + w];
        uint32_t p1 = partials[(size_t)(g + 1) * HIST_WORDS + w];
        uint32_t p2 = partials[(size_t)(g + 2) * HIST_WORDS + w];
        uint32_t p3 = partials[(size_t)(g + 3) * HIST_WORDS + w];
        lo += (p0 & 0xFFFFu) + (p1 & 0xFFFFu) + (p2 & 0xFFFFu) + (p3 & 0xFFFFu);
        hi += (p0 >> 16) + (p1 >> 16) + (p2 >> 16) + (p3 >> 16);
    }
    for (; g < G; ++g) {
        uint32_t p = partials[(size_t)g * HIST_WORDS + w];
        lo += p & 0xFFFFu;
        hi += p >> 16;
    }
    hot_counts[2 * w] = lo + spill[2 * w];
    hot_counts[2 * w + 1] = hi + spill[2 * w + 1];
}

// argmax over the dense hot table: best = max packed key.
__global__ void k_argmax_hot(const unsigned long long *__restrict__ hot_counts, Result *res) {
    const int bin = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long k = 0;
    if (bin < HOT_BINS) k = pack_key(hot_counts[bin], bin >> 8, bin & 255);
    k = wave_max_u64(k);
    if ((threadIdx.x & 63) == 0 && k) atomicMax(&res->best, k);
}

// argmax over the claimed cold slots.
__global__ void k_argmax_cold(ColdTable ct, Result *res) {
    const uint32_t n = *ct.n_used;
    unsigned long long best = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t h = ct.used[i];
        const uint32_t key = ct.keys[h];
        const unsigned long long k = pack_key(ct.counts[h], (int32_t)(key >> 16),
                                              (int32_t)(key & 0xFFFFu));
        best = k > best ? k : best;
    }
    best = wave_max_u64(best);
    if ((threadIdx.x & 63) == 0 && best) atomicMax(&res->best, best);
}

__device__ __forceinline__ void push_cand(Result *res, int2 *cand, int32_t a, int32_t b) {
    const unsigned int i = atomicAdd(&res->n_cand, 1u);
    if (i < CAND_CAP) cand[i] = make_int2(a, b);
}

// Collects every pair whose packed key equals the best (same W and same a+b).
__global__ void k_collect(const unsigned long long *__restrict__ hot_counts, ColdTable ct,
                          Result *res, int2 *cand) {
    const unsigned long long best = res->best;
    if (best == 0) return;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    if (tid < HOT_BINS) {
        if (pack_key(hot_counts[tid], tid >> 8, tid & 255) == best) push_cand(res, cand, tid >> 8, tid & 255);
    }
    const uint32_t n = *ct.n_used;
    for (uint32_t i = tid; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t h = ct.used[i];
        const uint32_t key = ct.keys[h];
        const int32_t a = (int32_t)(key >> 16), b = (int32_t)(key & 0xFFFFu);
        if (pack_key(ct.counts[h], a, b) == best) push_cand(res, cand, a, b);
    }
}

__global__ void k_cold_clear(ColdTable ct) {
    const uint32_t n = *ct.n_used;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t h = ct.used[i];
        ct.keys[h] = EMPTY;
        ct.counts[h] = 0;
    }
}

// ---------------------------------------------------------------------------------------------
// Exact passes (tie-break R3, apply R5): need the true run offset of every X X slot, carried
// across chunks in registers and across regions via carry_off (from k_runs).
// ---------------------------------------------------------------------------------------------
enum ExactMode { TIE = 0, APPLY_COUNT = 1, APPLY_SCATTER = 2 };

struct ExactArgs {
    const int32_t *ids;
    int64_t n_chunks, cpr, n_slots;
    int R;
    const int64_t *carry_off;
    // tie
    int n_cand;
    int32_t ca[MAX_CAND], cb[MAX_CAND];
    // apply
    int32_t a, b, c;
    int64_t *kept;             // per region (APPLY_COUNT)
    const int64_t *out_off;    // per region (APPLY_SCATTER)
    int32_t *out;
    Result *res;
};

template <int MODE>
__global__ void __launch_bounds__(256) k_exact(ExactArgs A) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (r >= A.R) return;
    const int64_t c0 = (int64_t)r * A.cpr;
    const int64_t c1 = min(c0 + A.cpr, A.n_chunks);
    const int4 *v4 = reinterpret_cast<const int4 *>(A.ids);
    int32_t prev = c0 > 0 ? A.ids[c0 * CHUNK - 1] : SEP;
    // offset (within its run) of the slot before the chunk; valid when slot 0 continues it
    int64_t prev_off = A.carry_off[r] - 1;
    bool prev_match = false;       // apply: match at the slot before the chunk
    unsigned long long last[MAX_CAND];
    if (MODE == TIE)
        for (int j = 0; j < MAX_CAND; ++j) last[j] = 0;
    unsigned long long n_match = 0;
    int64_t kept = 0;
    int64_t out_pos = (MODE == APPLY_SCATTER) ? A.out_off[r] : 0;
    for (int64_t c = c0; c < c1; ++c) {
        const int4 v = v4[c * 64 + lane];
        const int32_t nxt = A.ids[(c + 1) * CHUNK];
        Chunk ck;
        load_chunk(ck, v, nxt, prev, lane);
        if (MODE != TIE && c == c0 && c0 > 0) {
            // match at the last slot of the previous region (owned by it)
            const int32_t t0 = __shfl(v.x, 0);
            if (A.a != A.b) prev_match = prev == A.a && t0 == A.b;
            else prev_match = prev == A.a && t0 == A.a && ((A.carry_off[r] - 1) & 1) == 0;
        }
        prev = __shfl(v.w, 63);
        bool slow = false;
#pragma unroll
        for (int e = 0; e < 4; ++e) slow |= ck.eqn[e] && ck.eqp[e];
        int64_t off[4];
        if (__ballot(slow) == 0ull) {
#pragma unroll
            for (int e = 0; e < 4; ++e) off[e] = 0;   // only read at X X slots: all run starts
            prev_off = 0;
        } else {
            int rs[4];
            run_starts(ck, lane, rs);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = 4 * lane + e;
                off[e] = rs[e] >= 0 ? (int64_t)(k - rs[e]) : prev_off + 1 + k;
            }
            prev_off = __shfl(off[3], 63);
        }
        const int64_t base = c * CHUNK + 4 * lane;
        if (MODE == TIE) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int32_t x = ck.t[e], y = ck.t[e + 1];
                if (x < 0 || y < 0) continue;
                for (int j = 0; j < A.n_cand; ++j) {
                    if (x == A.ca[j] && y == A.cb[j] && (x != y || (off[e] & 1) == 0)) {
                        const unsigned long long p = (unsigned long long)(base + e) + 1;
                        last[j] = p > last[j] ? p : last[j];
                    }
                }
            }
        } else {
            bool m[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (A.a != A.b) m[e] = ck.t[e] == A.a && ck.t[e + 1] == A.b;
                else m[e] = ck.eqn[e] && ck.t[e] == A.a && (off[e] & 1) == 0;
            }
            const bool m_up = __shfl_up((int)m[3], 1) != 0;
            bool keep[4];
            keep[0] = !(lane == 0 ? prev_match : m_up);
            keep[1] = !m[0];
            keep[2] = !m[1];
            keep[3] = !m[2];
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (base + e >= A.n_slots) keep[e] = false;
            prev_match = __shfl((int)m[3], 63) != 0;
            int nk = (int)keep[0] + keep[1] + keep[2] + keep[3];
            int nm = (int)m[0] + m[1] + m[2] + m[3];
            // wave inclusive scan of nk
            int incl = nk;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                int o = __shfl_up(incl, d);
                if (lane >= d) incl += o;
            }
            const int total = __shfl(incl, 63);
            if (MODE == APPLY_SCATTER) {
                int64_t p = out_pos + incl - nk;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (keep[e]) A.out[p++] = m[e] ? A.c : ck.t[e];
                }
            }
            out_pos += total;
            kept += total;
            n_match += nm;
        }
    }
    if (MODE == TIE) {
        for (int j = 0; j < A.n_cand; ++j) {
            unsigned long long v = wave_max_u64(last[j]);
            if (lane == 0 && v) atomicMax(&A.res->last[j], v);
        }
    } else {
        // n_match summed over the wave
        unsigned long long s = n_match;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
        if (lane == 0) {
            if (MODE == APPLY_COUNT) {
                A.kept[r] = kept;
                if (s) atomicAdd(&A.res->replaced, s);
            }
        }
    }
}

// Exclusive scan of the per-region kept counts (R <= MAX_REGIONS), one workgroup.
__global__ void __launch_bounds__(1024) k_scan_regions(const int64_t *__restrict__ kept, int R,
                                                       int64_t *__restrict__ out_off, Result *res) {
    __shared__ int64_t part[1024];
    const int per = (R + 1023) / 1024;
    const int t = threadIdx.x;
    int64_t s = 0;
    for (int i = 0; i < per; ++i) {
        const int r = t * per + i;
        if (r < R) s += kept[r];
    }
    part[t] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        int64_t o = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += o;
        __syncthreads();
    }
    int64_t run = part[t] - s;
    for (int i = 0; i < per; ++i) {
        const int r = t * per + i;
        if (r < R) {
            out_off[r] = run;
            run += kept[r];
        }
    }
    if (t == 1023) res->kept_total = part[1023];
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
