// bpe_encode.hip — encodeToCode (core.ts:392-409) for many texts at once: a merge-rank encoder
// on the device, behind the bpe_encoder_* / bpe_encode_batch entry
// points of include/bpe.h.
//
// The reference encodes a text by running every merge in order over it:
//     for (let [from_code, to_code] of this.merge_codes)
//       content_in_code = content_in_code.replaceAll(from_code, to_code)        (core.ts:404-406)
// i.e. M sequential leftmost-non-overlapping rewrites.  For a merge list where no merge's new token
// is an input of itself or of an earlier merge (every list findNextMerge / restoreMerge / fromJSON
// of a reference-made JSON produces: c is always a new index, core.ts:315,484), that equals the
// rank-greedy form: repeatedly take the LOWEST-ranked merge whose pair occurs in the text and
// rewrite all of its leftmost non-overlapping occurrences.  Proof sketch: rewriting rank r only
// creates pairs that contain c_r, and every merge taking c_r as input has a rank above r, so ranks
// are taken in increasing order and each one does exactly what its replaceAll does; the ranks the
// greedy skips have no occurrence, where replaceAll is a no-op.  The greedy does work only for
// the merges that fire in this text (at most n - 1 of them), instead of M passes over it.
//
// One workgroup encodes one text held in LDS (u16 token ids + u16 pair ranks, two buffers; ids
// stay below BPE_MAX_VOCAB = 55296).  Per greedy step:
//   1. every thread walks its contiguous segment and flags the counted occurrences of rank r
//      (rule R1 of SURVEY.md Appendix A: for x == y only even offsets inside a run, which needs the
//      run length before the segment: a walk back);
//   2. an exclusive scan of the flag counts gives each segment's destination after the rewrite
//      (position i + 1 of every counted i is deleted);
//   3. the segment is written compacted into the other buffer; only the pairs that now touch c_r
//      are looked up again in the rank table (a hash in HBM, L2-resident: 8 B per merge, load
//      factor <= 1/2), the others keep their rank; the minimum of the written ranks is the next r.
// Two workgroup barriers per step.  Texts longer than an LDS buffer, and merge lists for which the
// greedy would differ, go through the apply-only streaming passes of a scratch engine
// (bpe_apply_merges: the same M replaceAll rewrites, one pass each, all long texts together).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "bpe.h"
#include "bpe_multi.h"   // bpe_fail

namespace {

// A pair's rank and the merge's new token in one word, rank << 16 | c: the minimum over a text is
// the next merge together with its c (no dependent load of c), and NO_RANK is above every one.
constexpr uint32_t NO_RANK = 0xFFFFFFFFu;
// tokens per workgroup of each launch shape (LDS: 6 bytes per token, u16 id + u32 rank word)
constexpr int CAP_MAX = 16384;   // 96 KiB (the largest launch shape below)
static_assert(CAP_MAX == BPE_ENCODE_LDS_TOKENS, "include/bpe.h");
constexpr size_t LDS_BYTES = 160 * 1024 - 256;   // per workgroup (the static words aside)

#define ENC_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return bpe_fail(e_ == hipErrorOutOfMemory ? BPE_ERR_OOM : BPE_ERR_HIP,         \
                            (std::string("bpe native: ") + #expr + ": " +                   \
                             hipGetErrorString(e_)).c_str());                              \
    } while (0)

struct RankTab {
    const unsigned long long *slots;   // (a << 16 | b) << 32 | rank << 16 | c; empty = ~0
    uint32_t mask;
    uint32_t shift;                    // 32 - log2(slots)
};

__host__ __device__ __forceinline__ uint32_t rank_home(uint32_t key, uint32_t shift) {
    return (key * 0x9E3779B1u) >> shift;
}

// Wave reductions on the VALU: DPP row rotations / shifts inside each 16-lane row, then the four
// row results through v_readlane (no LDS crossbar round trips, unlike __shfl_*).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, 0xF, 0xF, false);
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
    v = min(v, dpp<0x128>(v, v));   // row_ror:8
    v = min(v, dpp<0x124>(v, v));   // row_ror:4
    v = min(v, dpp<0x122>(v, v));   // row_ror:2
    v = min(v, dpp<0x121>(v, v));   // row_ror:1
    const uint32_t a = __builtin_amdgcn_readlane((int)v, 0), b = __builtin_amdgcn_readlane((int)v, 16);
    const uint32_t c = __builtin_amdgcn_readlane((int)v, 32), d = __builtin_amdgcn_readlane((int)v, 48);
    return min(min(a, b), min(c, d));
}

__device__ __forceinline__ int wave_incl(int v, int lane) {
    uint32_t u = (uint32_t)v;
    u += dpp<0x111>(u, 0);   // row_shr:1 (lanes without a source add 0)
    u += dpp<0x112>(u, 0);   // row_shr:2
    u += dpp<0x114>(u, 0);   // row_shr:4
    u += dpp<0x118>(u, 0);   // row_shr:8
    const int r = lane >> 4;
    const int t0 = __builtin_amdgcn_readlane((int)u, 15), t1 = __builtin_amdgcn_readlane((int)u, 31);
    const int t2 = __builtin_amdgcn_readlane((int)u, 47);
    return (int)u + (r >= 1 ? t0 : 0) + (r >= 2 ? t1 : 0) + (r >= 3 ? t2 : 0);
}

// minimum over the workgroup (one barrier; `m` holds one word per wave)
template <int WG>
__device__ __forceinline__ uint32_t block_min(uint32_t v, uint32_t *m) {
    v = wave_min(v);
    if (WG == 64) return v;
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) m[w] = v;
    __syncthreads();
    uint32_t r = m[0];
#pragma unroll
    for (int i = 1; i < WG / 64; ++i) r = min(r, m[i]);
    return r;
}

// exclusive prefix and total over the workgroup (one barrier; `s` holds one word per wave)
template <int WG>
__device__ __forceinline__ int block_scan(int v, int *s, int &total) {
    const int lane = threadIdx.x & 63;
    const int incl = wave_incl(v, lane);
    if (WG == 64) {
        total = __builtin_amdgcn_readlane(incl, 63);
        __syncthreads();   // (this step's flags, written by other lanes, are read next)
        return incl - v;
    }
    const int w = threadIdx.x >> 6;
    if (lane == 63) s[w] = incl;
    __syncthreads();
    int before = 0, all = 0;
#pragma unroll
    for (int i = 0; i < WG / 64; ++i) {
        const int x = s[i];
        before += i < w ? x : 0;
        all += x;
    }
    total = all;
    return before + incl - v;
}

// The rank table copied into LDS (the latency form: few texts per call, each on a CU of its own):
// keys[m] u32 (a << 16 | b per rank), cs[m] u16 (c per rank, padded to an even count), slot[S] u32
// (fingerprint << 16 | rank + 1, or 0 = empty; S a power of two >= 2m, linear probing from
// rank_home).  A probe reads one slot; only a fingerprint match reads the key and c (one more LDS
// round).  14 B per merge: 8000 merges take 111 KiB.
struct LdsTab {
    const uint32_t *img;   // the image above in HBM, copied word by word
    uint32_t words;        // its size in u32 words
    uint32_t m;            // merges
    uint32_t mask, shift;  // slot table: S = mask + 1, home = rank_home(key, shift)
};

__host__ __device__ __forceinline__ uint32_t fingerprint(uint32_t key) {
    return (key * 0x85EBCA6Bu) >> 16;
}

template <bool TAB_LDS>
struct Lookup {
    RankTab g;
    const uint32_t *keys, *slot;
    const uint16_t *cs;
    uint32_t mask, shift;
    __device__ __forceinline__ uint32_t operator()(uint32_t key) const {
        if constexpr (!TAB_LDS) {
            uint32_t h = rank_home(key, g.shift);
            for (;;) {
                const unsigned long long e = g.slots[h];
                if ((uint32_t)(e >> 32) == key) return (uint32_t)e;
                if (e == ~0ull) return NO_RANK;
                h = (h + 1) & g.mask;
            }
        } else {
            const uint32_t fp = fingerprint(key);
            uint32_t h = rank_home(key, shift);
            for (;;) {
                const uint32_t e = slot[h];
                if (!e) return NO_RANK;
                if ((e >> 16) == fp) {
                    const uint32_t r = (e & 0xFFFFu) - 1;
                    if (keys[r] == key) return (r << 16) | cs[r];
                }
                h = (h + 1) & mask;
            }
        }
    }
};

// One text per workgroup: which[blockIdx.x] indexes the texts of this launch shape; up to
// WG * (KMAX - 1) tokens, held in LDS as u16 ids + u32 rank words, rewritten in place.  Each greedy step:
//   - every thread loads its segment [s, s + k) (k <= KMAX) plus two tokens of look-ahead and one
//     rank word of look-behind into registers (one batch of LDS reads), and flags the counted
//     occurrences of rank r there (the chain parity comes from the look-behind; a chain crossing
//     into the segment is walked back in LDS, which only x == y runs do);
//   - an exclusive scan of the counts gives the segment's destination (barrier: every read of this
//     step is done before any write);
//   - the segment is written back compacted; the pairs that now touch c get their rank word again,
//     one request per lane per round, so a wave's probes run side by side;
//   - the minimum rank word written is the next step's merge (barrier).
template <int WG, int KMAX, bool TAB_LDS>
__global__ void __launch_bounds__(WG)
k_encode(const int32_t *__restrict__ in, const int64_t *__restrict__ off,
         const int32_t *__restrict__ which, int32_t *__restrict__ out, int32_t *__restrict__ out_len,
         RankTab t, LdsTab lt, unsigned long long *__restrict__ steps_total,
         unsigned long long *__restrict__ err) {
    static_assert(KMAX & 1, "odd segment lengths");
    constexpr int CAP = WG * (KMAX - 1);
    constexpr int H = KMAX + 2;   // segment + look-ahead
    extern __shared__ uint32_t lds32[];
    __shared__ uint32_t red[WG / 64];
    __shared__ int scn[WG / 64];
    uint32_t *rk = lds32;
    uint16_t *tok = reinterpret_cast<uint16_t *>(lds32 + CAP);
    Lookup<TAB_LDS> look;
    look.g = t;
    if constexpr (TAB_LDS) {
        uint32_t *tw = lds32 + CAP + CAP / 2;
        const uint32_t w4 = lt.words & ~3u;
        for (uint32_t w = 4 * threadIdx.x; w < w4; w += 4 * WG)
            *reinterpret_cast<uint4 *>(tw + w) = *reinterpret_cast<const uint4 *>(lt.img + w);
        for (uint32_t w = w4 + threadIdx.x; w < lt.words; w += WG) tw[w] = lt.img[w];
        look.keys = tw;
        look.cs = reinterpret_cast<const uint16_t *>(tw + lt.m);
        look.slot = tw + lt.m + ((lt.m + 1) >> 1);
        look.mask = lt.mask;
        look.shift = lt.shift;
    }

    const int text = which[blockIdx.x];
    const int64_t base = off[text];
    int n = (int)(off[text + 1] - base);
    const int tid = threadIdx.x;

    bool bad = false;
    for (int i = tid; i < n; i += WG) {
        const int32_t v = in[base + i];
        bad |= (uint32_t)v >= (uint32_t)BPE_MAX_VOCAB;
        tok[i] = (uint16_t)v;
    }
    // (an id out of range: counted in *err, the call fails; the text's output is void)
    if (bad) atomicAdd(err, 1ull);
    __syncthreads();
    uint32_t lmin = NO_RANK;
    for (int i = tid; i < n; i += WG) {
        const uint32_t r = i + 1 < n ? look(((uint32_t)tok[i] << 16) | tok[i + 1]) : NO_RANK;
        rk[i] = r;
        lmin = min(lmin, r);
    }
    uint32_t r = block_min<WG>(lmin, red);
    __syncthreads();
    int steps = 0;

    while (r != NO_RANK) {   // (uniform: every thread holds the same r)
        ++steps;
        const uint32_t c = r & 0xFFFFu;
        // segment length: odd, so that lane t's j-th word (t * k + j) falls in a bank of its own
        // (an even stride would put 2..16 lanes on one bank)
        const int k = max(3, (n + WG - 1) / WG) | 1;   // (<= KMAX: n <= WG * (KMAX - 1))
        const int s = tid * k;
        const int len = max(0, min(k, n - s));       // segment [s, s + len)
        uint32_t T[H], R[H];
#pragma unroll
        for (int j = 0; j < H; ++j) {
            const bool in_seg = j < k + 2 && s + j < n;
            T[j] = in_seg ? tok[s + j] : 0u;
            R[j] = in_seg ? rk[s + j] : NO_RANK;
        }
        const uint32_t rb = (len > 0 && s > 0) ? rk[s - 1] : NO_RANK;
        // chain parity at the segment start: d = r-pairs right before s
        int d = 0;
        bool fprev = false;   // is s - 1 counted (s deleted)?
        if (rb == r) {
            for (int j = s - 1; j >= 0 && rk[j] == r; --j) ++d;
            fprev = !((d - 1) & 1);
        }
        uint32_t F = 0;   // counted flags of [s, s + k + 2)
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < H; ++j) {
            const bool m = R[j] == r;
            const bool f = m && !(d & 1);
            F |= (uint32_t)f << j;
            cnt += (f && j < len) ? 1 : 0;
            d = m ? d + 1 : 0;
        }
        int total = 0;
        const int before = block_scan<WG>(cnt, scn, total);   // (barrier: all reads done)
        const int p0 = s - before + (fprev ? 1 : 0);
        // live positions of the segment: j is dead when j - 1 is counted
        const uint32_t live = ~((F << 1) | (fprev ? 1u : 0u)) & ((1u << len) - 1u);
        int p = p0;
        lmin = NO_RANK;
        uint32_t K[KMAX];
        uint32_t req = 0;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            K[j] = 0;
            if ((live >> j) & 1) {   // (else: the b of a counted (a, b), or past the segment)
                const bool fi = (F >> j) & 1;
                const uint32_t tv = fi ? c : T[j];
                const int nx = fi ? j + 2 : j + 1;
                uint32_t rv = NO_RANK;
                if (s + nx < n) {
                    const bool fn = (F >> nx) & 1;
                    const uint32_t tn = fi ? T[j + 2] : T[j + 1];
                    if (fi || fn) {
                        K[j] = (tv << 16) | (fn ? c : tn);
                        req |= 1u << j;
                    }
                    rv = R[j];
                }
                tok[p] = (uint16_t)tv;
                if (!((req >> j) & 1)) {
                    rk[p] = rv;
                    lmin = min(lmin, rv);
                }
                ++p;
            }
        }
        // the new pairs' rank words: one request per lane per round (its position: p0 + the live
        // positions before it)
        while (__ballot(req != 0)) {
            if (req) {
                const int j = __builtin_ctz(req);
                uint32_t key = 0;
#pragma unroll
                for (int jj = 0; jj < KMAX; ++jj)
                    if (jj == j) key = K[jj];
                const int pp = p0 + __builtin_popcount(live & ((1u << j) - 1u));
                const uint32_t rv = look(key);
                rk[pp] = rv;
                lmin = min(lmin, rv);
                req &= req - 1;
            }
        }
        n -= total;
        r = block_min<WG>(lmin, red);   // (barrier: the rewritten text visible)
        __syncthreads();
    }

    for (int i = tid; i < n; i += WG) out[base + i] = tok[i];
    if (tid == 0) {
        out_len[text] = n;
        if (steps) atomicAdd(steps_total, (unsigned long long)steps);
    }
}

// launch shapes (WG threads x KMAX tokens each), by text length: the smallest that holds the text,
// so the unrolled segment loops do little masked-off work
constexpr int N_SHAPES = 8;
constexpr int SHAPE_WG[N_SHAPES] = {64, 64, 64, 256, 256, 256, 1024, 1024};
constexpr int SHAPE_K[N_SHAPES] = {3, 5, 9, 5, 9, 17, 9, 17};

constexpr int shape_cap(int i) { return SHAPE_WG[i] * (SHAPE_K[i] - 1); }
constexpr size_t shape_lds(int i) { return (size_t)shape_cap(i) * 6; }
// The packed output of a call on the device: exclusive scan of the encoded lengths (one workgroup,
// 1024 lengths per round) and a gather of every text from its input offset to its output offset
// (one wave per text), so the host copies the result once, with no per-text loop.
// ooff[n + 1] receives the call's bad-id count (*err), so that one copy brings both back.
__global__ void __launch_bounds__(1024)
k_scan_lens(const int32_t *__restrict__ len, int64_t n, int64_t *__restrict__ ooff,
            const unsigned long long *__restrict__ err) {
    __shared__ int scn[16];
    long long carry = 0;
    for (int64_t b = 0; b < n; b += 1024) {
        const int64_t i = b + threadIdx.x;
        const int v = i < n ? len[i] : 0;
        int total = 0;
        const int before = block_scan<1024>(v, scn, total);
        if (i < n) ooff[i] = carry + before;
        carry += total;
        __syncthreads();   // (scn is reused next round)
    }
    if (threadIdx.x == 0) {
        ooff[n] = carry;
        ooff[n + 1] = (long long)*err;
    }
}

// Both in one workgroup, for a call of at most 1024 texts (the one-text-per-call shape): the scan,
// then one wave per text.
__global__ void __launch_bounds__(1024)
k_pack_small(const int32_t *__restrict__ src, const int64_t *__restrict__ in_off,
             const int32_t *__restrict__ len, int n, int64_t *__restrict__ ooff,
             const unsigned long long *__restrict__ err, int32_t *__restrict__ dst) {
    __shared__ int scn[16];
    __shared__ int start[1025];
    const int v = (int)threadIdx.x < n ? len[threadIdx.x] : 0;
    int total = 0;
    const int before = block_scan<1024>(v, scn, total);
    if ((int)threadIdx.x < n) {
        start[threadIdx.x] = before;
        ooff[threadIdx.x] = before;
    }
    if (threadIdx.x == 0) {
        ooff[n] = total;
        ooff[n + 1] = (long long)*err;
    }
    __syncthreads();
    for (int t = threadIdx.x >> 6; t < n; t += 16) {
        const int32_t *s = src + in_off[t];
        int32_t *d = dst + start[t];
        const int l = len[t];
        for (int i = threadIdx.x & 63; i < l; i += 64) d[i] = s[i];
    }
}

__global__ void __launch_bounds__(256)
k_gather(const int32_t *__restrict__ src, const int64_t *__restrict__ in_off,
         const int32_t *__restrict__ len, const int64_t *__restrict__ ooff, int64_t n,
         int32_t *__restrict__ dst) {
    const int64_t text = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (text >= n) return;
    const int32_t *s = src + in_off[text];
    int32_t *d = dst + ooff[text];
    const int l = len[text];
    for (int i = threadIdx.x & 63; i < l; i += 64) d[i] = s[i];
}

// shorter texts take the HBM table even in the few-texts form (the LDS copy costs more than its
// faster probes save over their few steps)
constexpr int LDS_TAB_MIN_TOKENS = 128;

}  // namespace

struct bpe_encoder {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // large calls in groups (encode_groups): copies on cstream, kernels on stream, two slots
    hipStream_t cstream = nullptr;
    hipEvent_t g_in[2] = {nullptr, nullptr}, g_k0[2] = {nullptr, nullptr}, g_k1[2] = {nullptr, nullptr};
    std::vector<int32_t> abc;                 // the merges, in rank order
    bool greedy_ok = true;                    // the rank-greedy form equals the replay (above)
    std::vector<uint8_t> is_input;            // ids used as a or b by the merges so far
    int32_t vocab = 0;                        // 1 + the largest id of the merges
    // rank table (host copy; uploaded when dirty)
    std::vector<unsigned long long> slots;
    uint32_t bits = 0;
    std::vector<uint16_t> c_of;               // rank -> c
    bool dirty = true;
    unsigned long long *d_slots = nullptr;
    size_t d_slots_n = 0;
    // the same merges as the LDS image (LdsTab), for calls of few texts
    std::vector<uint32_t> limg;
    uint32_t *d_limg = nullptr;
    size_t d_limg_n = 0;
    LdsTab lt{};
    unsigned long long *d_steps = nullptr;
    // staging: pinned host and device, grown as needed
    char *h_buf = nullptr, *d_buf = nullptr;
    size_t h_cap = 0, d_cap = 0;
    bpe_ctx *scratch = nullptr;               // the apply-pass route
    int32_t scratch_known = 0;
    bpe_encoder_stats st{};
};

namespace {

void table_insert(bpe_encoder *E, uint32_t key, uint32_t rank) {
    const uint32_t mask = (1u << E->bits) - 1, shift = 32 - E->bits;
    uint32_t h = rank_home(key, shift);
    for (;;) {
        unsigned long long &s = E->slots[h];
        if (s == ~0ull) {
            s = ((unsigned long long)key << 32) | (rank << 16) | E->c_of[rank];
            return;
        }
        if ((uint32_t)(s >> 32) == key) return;   // a repeated pair: its first rank wins (the
                                                  // later replaceAll finds nothing left)
        h = (h + 1) & mask;
    }
}

void table_rebuild(bpe_encoder *E, uint32_t bits) {
    E->bits = bits;
    E->slots.assign((size_t)1 << bits, ~0ull);
    const int64_t m = (int64_t)E->c_of.size();
    for (int64_t r = 0; r < m; ++r)
        table_insert(E, ((uint32_t)E->abc[3 * r] << 16) | (uint32_t)E->abc[3 * r + 1], (uint32_t)r);
}

template <typename T>
int grow_dev(T **p, size_t *have, size_t want) {
    if (*have >= want) return BPE_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    const size_t n = std::max<size_t>(want, 1) * 3 / 2 + 64;
    ENC_TRY(hipMalloc((void **)p, n * sizeof(T)));
    *have = n;
    return BPE_OK;
}

// the LDS image of the merges (LdsTab): keys, cs, slots
void build_lds_image(bpe_encoder *E) {
    const uint32_t m = (uint32_t)E->c_of.size();
    uint32_t bits = 1;
    while ((1u << bits) < 2 * m) ++bits;
    const uint32_t S = 1u << bits, m2 = (m + 1) & ~1u;
    E->limg.assign(m + m2 / 2 + S, 0u);
    uint32_t *keys = E->limg.data();
    uint16_t *cs = reinterpret_cast<uint16_t *>(keys + m);
    uint32_t *slot = keys + m + m2 / 2;
    for (uint32_t r = 0; r < m; ++r) {
        const uint32_t key = ((uint32_t)E->abc[3 * r] << 16) | (uint32_t)E->abc[3 * r + 1];
        keys[r] = key;
        cs[r] = E->c_of[r];
        uint32_t h = rank_home(key, 32 - bits);
        while (slot[h] && keys[(slot[h] & 0xFFFFu) - 1] != key) h = (h + 1) & (S - 1);
        if (!slot[h]) slot[h] = (fingerprint(key) << 16) | (r + 1);   // (a repeated pair keeps its first rank)
    }
    E->lt.words = (uint32_t)E->limg.size();
    E->lt.m = m;
    E->lt.mask = S - 1;
    E->lt.shift = 32 - bits;
}

int upload_table(bpe_encoder *E) {
    if (!E->dirty) return BPE_OK;
    int rc;
    if ((rc = grow_dev(&E->d_slots, &E->d_slots_n, E->slots.size()))) return rc;
    ENC_TRY(hipMemcpyAsync(E->d_slots, E->slots.data(), E->slots.size() * 8, hipMemcpyHostToDevice,
                           E->stream));
    build_lds_image(E);
    if ((rc = grow_dev(&E->d_limg, &E->d_limg_n, E->limg.size()))) return rc;
    ENC_TRY(hipMemcpyAsync(E->d_limg, E->limg.data(), E->limg.size() * 4, hipMemcpyHostToDevice,
                           E->stream));
    E->lt.img = E->d_limg;
    E->dirty = false;
    return BPE_OK;
}

// calls of at most this many id bytes go through the pinned staging buffer both ways
constexpr size_t SMALL_CALL_BYTES = 4u << 20;

// texts per call up to which each gets a CU of its own, so the LDS copy of the table pays
constexpr size_t LATENCY_TEXTS = 256;

template <int I, bool TAB_LDS>
hipError_t set_lds_attr() {
    return hipFuncSetAttribute((const void *)k_encode<SHAPE_WG[I], SHAPE_K[I], TAB_LDS>,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(TAB_LDS ? LDS_BYTES : shape_lds(I)));
}

template <int I>
hipError_t set_lds_attrs() {
    hipError_t e = set_lds_attr<I, true>();
    if (e == hipSuccess) e = set_lds_attr<I, false>();
    if constexpr (I + 1 < N_SHAPES) {
        if (e == hipSuccess) e = set_lds_attrs<I + 1>();
    }
    return e;
}

template <int I>
void launch_one(bpe_encoder *E, unsigned n, bool tab_lds, const int32_t *ids, const int64_t *off,
                const int32_t *which, int32_t *out, int32_t *len, unsigned long long *err) {
    constexpr int WG = SHAPE_WG[I], KM = SHAPE_K[I];
    const RankTab t{E->d_slots, (1u << E->bits) - 1, 32 - E->bits};
    if (tab_lds)
        k_encode<WG, KM, true><<<n, WG, shape_lds(I) + (size_t)E->lt.words * 4, E->stream>>>(
            ids, off, which, out, len, t, E->lt, E->d_steps, err);
    else
        k_encode<WG, KM, false><<<n, WG, shape_lds(I), E->stream>>>(ids, off, which, out, len, t,
                                                                    E->lt, E->d_steps, err);
}

template <int I = 0>
void launch_shape(int i, bpe_encoder *E, unsigned n, bool tab_lds, const int32_t *ids,
                  const int64_t *off, const int32_t *which, int32_t *out, int32_t *len,
                  unsigned long long *err) {
    if (i == I) return launch_one<I>(E, n, tab_lds, ids, off, which, out, len, err);
    if constexpr (I + 1 < N_SHAPES)
        launch_shape<I + 1>(i, E, n, tab_lds, ids, off, which, out, len, err);
}

// Staging buffers of a call: h_bytes of pinned host memory and d_bytes of device memory.  The
// pinned buffer holds only what a call stages through the host (a large call's ids go straight
// from and to the caller's buffers), and one larger than PINNED_KEEP is released at the end of
// the call that needed it (release_stage), so a rare huge call does not pin host memory for the
// encoder's lifetime.
constexpr size_t PINNED_KEEP = size_t(64) << 20;

int grow_stage(bpe_encoder *E, size_t h_bytes, size_t d_bytes) {
    if (E->h_cap < h_bytes) {
        if (E->h_buf) (void)hipHostFree(E->h_buf);
        E->h_buf = nullptr;
        E->h_cap = 0;
        const size_t n = h_bytes * 3 / 2 + 4096;
        ENC_TRY(hipHostMalloc((void **)&E->h_buf, n, hipHostMallocDefault));
        E->h_cap = n;
    }
    const size_t bytes = d_bytes;
    if (E->d_cap < bytes) {
        if (E->d_buf) (void)hipFree(E->d_buf);
        E->d_buf = nullptr;
        E->d_cap = 0;
        const size_t n = bytes * 3 / 2 + 4096;
        ENC_TRY(hipMalloc((void **)&E->d_buf, n));
        E->d_cap = n;
    }
    return BPE_OK;
}

void release_stage(bpe_encoder *E) {
    if (E->h_cap > PINNED_KEEP) {
        // (an early error return may leave a copy from it in flight)
        (void)hipStreamSynchronize(E->stream);
        (void)hipStreamSynchronize(E->cstream);
        (void)hipHostFree(E->h_buf);
        E->h_buf = nullptr;
        E->h_cap = 0;
    }
}

size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// the apply-pass route: every listed text as one sample of the scratch engine, all M merges
// replayed over them (one streaming pass per merge), the results back into out at the texts'
// own offsets (rel: offsets relative to off[0]) and their lengths into len
int encode_replay(bpe_encoder *E, const int32_t *ids, const int64_t *off, const std::vector<int64_t> &list,
                  int32_t *out, int64_t *len) {
    if (list.empty()) return BPE_OK;
    int rc;
    if (!E->scratch) {
        if ((rc = bpe_create(&E->scratch, E->device))) return rc;
        E->scratch_known = 0;
    }
    struct Clear {
        bpe_ctx *c;
        ~Clear() { bpe_clear_corpus(c); }
    } clear{E->scratch};
    if ((rc = bpe_clear_corpus(E->scratch))) return rc;
    int32_t vocab = E->vocab;
    for (int64_t k : list)
        for (int64_t i = off[k]; i < off[k + 1]; ++i) vocab = std::max(vocab, ids[i] + 1);
    // lengths only matter to the max_length filter of a find, which never runs here
    for (int32_t i = E->scratch_known; i < vocab; ++i)
        if ((rc = bpe_set_token_len16(E->scratch, i, 1))) return rc;
    E->scratch_known = std::max(E->scratch_known, vocab);
    for (int64_t k : list)
        if ((rc = bpe_add_sample(E->scratch, ids + off[k], off[k + 1] - off[k]))) return rc;
    const int64_t m = (int64_t)E->abc.size() / 3;
    if (m && (rc = bpe_apply_merges(E->scratch, E->abc.data(), m, nullptr, 0))) return rc;
    int64_t ns = 0, nt = 0;
    if ((rc = bpe_corpus_size(E->scratch, &ns, &nt))) return rc;
    std::vector<int32_t> got((size_t)std::max<int64_t>(nt, 1));
    std::vector<int64_t> goff((size_t)ns + 1);
    if ((rc = bpe_read_corpus(E->scratch, got.data(), (int64_t)got.size(), goff.data(), ns + 1))) return rc;
    for (size_t j = 0; j < list.size(); ++j) {
        const int64_t k = list[j], l = goff[j + 1] - goff[j];
        std::memcpy(out + (off[k] - off[0]), got.data() + goff[j], (size_t)l * 4);
        len[k] = l;
    }
    E->st.texts_replay += (int64_t)list.size();
    return BPE_OK;
}

// A large call (at least 2 x GROUP_TOKENS input tokens) whose texts all take the kernels, in a few
// groups (BPE_ENCODE_GROUPS, default 3) through two slots: the copy stream takes group g's ids up (a pageable copy: the host waits for
// it) while the kernel stream encodes group g - 1, and group g - 1's packed ids come down while
// group g encodes.  Each group is packed on its own; its ids land after the previous groups'.
constexpr int64_t GROUP_TOKENS = int64_t(1) << 23;

int encode_groups_run(bpe_encoder *E, const int32_t *ids, const int64_t *off, int64_t n_texts,
                      const std::vector<int32_t> &shape_of, int32_t *ids_out, int64_t *out_off) {
    // contiguous text ranges [g0, g1) of >= GROUP_TOKENS tokens (the last one whatever is left)
    // (few groups: each group's longest texts finish alone, so more groups cost kernel time)
    static const int64_t n_groups = [] {
        const char *v = getenv("BPE_ENCODE_GROUPS");
        return v && atoi(v) >= 2 ? (int64_t)atoi(v) : (int64_t)3;
    }();
    const int64_t gt = std::max<int64_t>(GROUP_TOKENS / 2,
                                          (off[n_texts] - off[0] + n_groups - 1) / n_groups);
    std::vector<int64_t> cut{0};
    for (int64_t k = 0; k < n_texts; ++k)
        if (off[k + 1] - off[cut.back()] >= gt && k + 1 < n_texts) cut.push_back(k + 1);
    cut.push_back(n_texts);
    const int ng = (int)cut.size() - 1;
    int64_t max_t = 0, max_n = 0;
    for (int g = 0; g < ng; ++g) {
        max_t = std::max(max_t, off[cut[g + 1]] - off[cut[g]]);
        max_n = std::max(max_n, cut[g + 1] - cut[g]);
    }
    // per slot, device: [ooff (n+2) | ids | off (n+2) | which | out | len]; pinned: [ooff | off | which]
    const size_t b_ids = align16((size_t)std::max<int64_t>(max_t, 1) * 4);
    const size_t b_off = align16((size_t)(max_n + 2) * 8);
    const size_t b_which = align16((size_t)max_n * 4);
    const size_t slot_d = b_off + b_ids + b_off + b_which + b_ids + b_which;
    const size_t slot_h = b_off + b_off + b_which;
    int rc;
    if ((rc = grow_stage(E, 2 * slot_h, 2 * slot_d))) return rc;
    hipStream_t ks = E->stream, cs = E->cstream;
    int64_t base = 0;
    out_off[0] = 0;
    int64_t n_checked = 0;
    // group g's texts come back: its offsets (small, pinned), then its packed ids
    auto finish = [&](int g) -> int {
        const int sl = g & 1;
        const int64_t k0 = cut[g], n = cut[g + 1] - k0;
        int64_t *h_ooff = reinterpret_cast<int64_t *>(E->h_buf + sl * slot_h);
        char *d = E->d_buf + sl * slot_d;
        ENC_TRY(hipStreamWaitEvent(cs, E->g_k1[sl], 0));
        ENC_TRY(hipMemcpyAsync(h_ooff, d, (size_t)(n + 2) * 8, hipMemcpyDeviceToHost, cs));
        ENC_TRY(hipStreamSynchronize(cs));
        if (h_ooff[n + 1]) return bpe_fail(BPE_ERR_VOCAB, "bpe native: token id out of range in text");
        const int64_t n_out = h_ooff[n];
        if (n_out < 0 || n_out > off[cut[g + 1]] - off[k0])
            return bpe_fail(BPE_ERR_STATE, "bpe native: bad packed length");
        if (n_out) {
            ENC_TRY(hipMemcpyAsync(ids_out + base, d + b_off, (size_t)n_out * 4, hipMemcpyDeviceToHost, cs));
            ENC_TRY(hipStreamSynchronize(cs));
        }
        for (int64_t k = 1; k <= n; ++k) out_off[k0 + k] = base + h_ooff[k];
        base += n_out;
        float ms = 0;
        ENC_TRY(hipEventElapsedTime(&ms, E->g_k0[sl], E->g_k1[sl]));
        E->st.kernel_ms += ms;
        n_checked = cut[g + 1];
        return BPE_OK;
    };
    for (int g = 0; g < ng; ++g) {
        const int sl = g & 1;
        const int64_t k0 = cut[g], n = cut[g + 1] - k0, t0 = off[k0], tn = off[cut[g + 1]] - t0;
        char *d = E->d_buf + sl * slot_d;
        char *h = E->h_buf + sl * slot_h;
        int64_t *d_ooff = reinterpret_cast<int64_t *>(d);
        int32_t *d_ids = reinterpret_cast<int32_t *>(d + b_off);
        int64_t *d_off = reinterpret_cast<int64_t *>(d + b_off + b_ids);
        int32_t *d_which = reinterpret_cast<int32_t *>(d + b_off + b_ids + b_off);
        int32_t *d_out = reinterpret_cast<int32_t *>(d + b_off + b_ids + b_off + b_which);
        int32_t *d_len = reinterpret_cast<int32_t *>(d + b_off + 2 * b_ids + b_off + b_which);
        unsigned long long *d_err = reinterpret_cast<unsigned long long *>(d_off + n + 1);
        int64_t *h_off = reinterpret_cast<int64_t *>(h + b_off);
        int32_t *h_which = reinterpret_cast<int32_t *>(h + b_off + b_off);
        // (slot sl's pinned staging was last read by group g - 2's upload, complete by now: its
        // kernels, which waited for it, were waited for by finish(g - 2))
        for (int64_t k = 0; k <= n; ++k) h_off[k] = off[k0 + k] - t0;
        h_off[n + 1] = 0;
        int64_t cnt[N_SHAPES] = {};
        for (int64_t k = 0; k < n; ++k) ++cnt[shape_of[k0 + k]];
        int64_t at[N_SHAPES];
        for (int i = 0, a = 0; i < N_SHAPES; a += (int)cnt[i], ++i) at[i] = a;
        int64_t fill[N_SHAPES];
        std::memcpy(fill, at, sizeof fill);
        for (int64_t k = 0; k < n; ++k) h_which[fill[shape_of[k0 + k]]++] = (int32_t)k;
        ENC_TRY(hipMemcpyAsync(d_ids, ids + t0, (size_t)tn * 4, hipMemcpyHostToDevice, cs));
        ENC_TRY(hipMemcpyAsync(d_off, h_off, b_off + (size_t)n * 4, hipMemcpyHostToDevice, cs));
        ENC_TRY(hipEventRecord(E->g_in[sl], cs));
        ENC_TRY(hipStreamWaitEvent(ks, E->g_in[sl], 0));
        ENC_TRY(hipEventRecord(E->g_k0[sl], ks));
        for (int i = 0; i < N_SHAPES; ++i)
            if (cnt[i])
                launch_shape(i, E, (unsigned)cnt[i], false, d_ids, d_off, d_which + at[i], d_out,
                             d_len, d_err);
        k_scan_lens<<<1, 1024, 0, ks>>>(d_len, n, d_ooff, d_err);
        k_gather<<<(unsigned)((n + 3) / 4), 256, 0, ks>>>(d_out, d_off, d_len, d_ooff, n, d_ids);
        ENC_TRY(hipGetLastError());
        ENC_TRY(hipEventRecord(E->g_k1[sl], ks));
        if (g > 0 && (rc = finish(g - 1))) return rc;
    }
    if ((rc = finish(ng - 1))) return rc;
    if (n_checked != n_texts) return bpe_fail(BPE_ERR_STATE, "bpe native: encode groups incomplete");
    E->st.texts_rank += n_texts;
    E->st.tokens_out += out_off[n_texts];
    return BPE_OK;
}

int encode_groups(bpe_encoder *E, const int32_t *ids, const int64_t *off, int64_t n_texts,
                  const std::vector<int32_t> &shape_of, int32_t *ids_out, int64_t *out_off) {
    // (nothing of an earlier call may still read the staging buffers; a refused call leaves
    // nothing in flight either)
    ENC_TRY(hipStreamSynchronize(E->stream));
    const int rc = encode_groups_run(E, ids, off, n_texts, shape_of, ids_out, out_off);
    // (every copy of the call is complete on success; a failed call drains both streams)
    (void)hipStreamSynchronize(E->cstream);
    (void)hipStreamSynchronize(E->stream);
    release_stage(E);
    return rc;
}

}  // namespace

extern "C" {

int bpe_encoder_create(bpe_encoder **out, int device) {
    if (!out) return bpe_fail(BPE_ERR_ARG, "bpe native: null argument");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return bpe_fail(BPE_ERR_HIP, "bpe native: no HIP device available (MI355X required)");
    if (device < 0 || device >= n) return bpe_fail(BPE_ERR_ARG, "bpe native: bad device index");
    bpe_encoder *E = new bpe_encoder();
    E->device = device;
    auto bail = [&](int rc) {
        bpe_encoder_destroy(E);
        return rc;
    };
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&E->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&E->ev0) != hipSuccess || hipEventCreate(&E->ev1) != hipSuccess ||
        hipStreamCreateWithFlags(&E->cstream, hipStreamNonBlocking) != hipSuccess)
        return bail(bpe_fail(BPE_ERR_HIP, "bpe native: encoder stream/events"));
    for (int i = 0; i < 2; ++i)
        if (hipEventCreateWithFlags(&E->g_in[i], hipEventDisableTiming) != hipSuccess ||
            hipEventCreate(&E->g_k0[i]) != hipSuccess || hipEventCreate(&E->g_k1[i]) != hipSuccess)
            return bail(bpe_fail(BPE_ERR_HIP, "bpe native: encoder stream/events"));
    if (hipMalloc((void **)&E->d_steps, 64) != hipSuccess ||
        hipMemset(E->d_steps, 0, 64) != hipSuccess)
        return bail(bpe_fail(BPE_ERR_OOM, "bpe native: encoder counters"));
    if (set_lds_attrs<0>() != hipSuccess)
        return bail(bpe_fail(BPE_ERR_HIP, "bpe native: encoder LDS attribute"));
    table_rebuild(E, 10);
    *out = E;
    return BPE_OK;
}

int bpe_encoder_destroy(bpe_encoder *E) {
    if (!E) return BPE_OK;
    (void)hipSetDevice(E->device);
    if (E->stream) (void)hipStreamSynchronize(E->stream);
    if (E->cstream) (void)hipStreamSynchronize(E->cstream);
    if (E->scratch) bpe_destroy(E->scratch);
    if (E->d_slots) (void)hipFree(E->d_slots);
    if (E->d_limg) (void)hipFree(E->d_limg);
    if (E->d_steps) (void)hipFree(E->d_steps);
    if (E->d_buf) (void)hipFree(E->d_buf);
    if (E->h_buf) (void)hipHostFree(E->h_buf);
    if (E->ev0) (void)hipEventDestroy(E->ev0);
    if (E->ev1) (void)hipEventDestroy(E->ev1);
    for (int i = 0; i < 2; ++i)
        for (hipEvent_t ev : {E->g_in[i], E->g_k0[i], E->g_k1[i]})
            if (ev) (void)hipEventDestroy(ev);
    if (E->cstream) (void)hipStreamDestroy(E->cstream);
    if (E->stream) (void)hipStreamDestroy(E->stream);
    delete E;
    return BPE_OK;
}

int bpe_encoder_clear(bpe_encoder *E) {
    if (!E) return bpe_fail(BPE_ERR_ARG, "bpe native: null encoder");
    E->abc.clear();
    E->c_of.clear();
    E->is_input.clear();
    E->greedy_ok = true;
    E->vocab = 0;
    table_rebuild(E, 10);
    E->dirty = true;
    return BPE_OK;
}

int bpe_encoder_add_merges(bpe_encoder *E, const int32_t *abc, int64_t n) {
    if (!E || n < 0 || (n && !abc)) return bpe_fail(BPE_ERR_ARG, "bpe native: bad add_merges arguments");
    for (int64_t i = 0; i < 3 * n; ++i)
        if (abc[i] < 0 || abc[i] >= BPE_MAX_VOCAB)
            return bpe_fail(BPE_ERR_VOCAB, "bpe native: merge token id out of range");
    if ((int64_t)E->c_of.size() + n > BPE_MAX_VOCAB)
        return bpe_fail(BPE_ERR_VOCAB, "bpe native: more merges than token ids");
    if (E->is_input.size() < (size_t)BPE_MAX_VOCAB) E->is_input.assign(BPE_MAX_VOCAB, 0);
    const size_t m = E->c_of.size() + (size_t)n;
    uint32_t bits = E->bits;
    while (((size_t)1 << bits) < 2 * m) ++bits;
    const bool rehash = bits != E->bits;
    for (int64_t i = 0; i < n; ++i) {
        const int32_t a = abc[3 * i], b = abc[3 * i + 1], c = abc[3 * i + 2];
        E->is_input[a] = E->is_input[b] = 1;
        // the greedy needs every new token to be new to the merges up to and including its own
        if (E->is_input[c]) E->greedy_ok = false;
        E->abc.push_back(a);
        E->abc.push_back(b);
        E->abc.push_back(c);
        E->c_of.push_back((uint16_t)c);
        E->vocab = std::max(E->vocab, std::max(a, std::max(b, c)) + 1);
        if (!rehash) table_insert(E, ((uint32_t)a << 16) | (uint32_t)b, (uint32_t)(E->c_of.size() - 1));
    }
    if (rehash) table_rebuild(E, bits);
    E->dirty = true;
    return BPE_OK;
}

int bpe_encoder_num_merges(bpe_encoder *E, int64_t *n) {
    if (!E || !n) return bpe_fail(BPE_ERR_ARG, "bpe native: null argument");
    *n = (int64_t)E->c_of.size();
    return BPE_OK;
}

int bpe_encode_batch(bpe_encoder *E, const int32_t *ids, const int64_t *off, int64_t n_texts,
                     int32_t *ids_out, int64_t *out_off) {
    if (!E || n_texts < 0 || (n_texts && (!off || !out_off)))
        return bpe_fail(BPE_ERR_ARG, "bpe native: bad encode_batch arguments");
    if (n_texts == 0) {
        if (out_off) out_off[0] = 0;
        return BPE_OK;
    }
    for (int64_t k = 0; k < n_texts; ++k)
        if (off[k + 1] < off[k]) return bpe_fail(BPE_ERR_ARG, "bpe native: text offsets must not decrease");
    const int64_t base = off[0], total = off[n_texts] - base;
    if (total && (!ids || !ids_out)) return bpe_fail(BPE_ERR_ARG, "bpe native: null id buffer");
    ENC_TRY(hipSetDevice(E->device));
    E->st.calls++;
    E->st.tokens_in += total;
    // launch shape of every text (the smallest that holds it), or the apply-pass route
    std::vector<int32_t> lists[N_SHAPES];
    std::vector<int64_t> replay;
    for (int64_t k = 0; k < n_texts; ++k) {
        const int64_t l = off[k + 1] - off[k];
        if (!E->greedy_ok || l > CAP_MAX) {
            replay.push_back(k);
        } else {
            int i = 0;
            while (shape_cap(i) < l) ++i;
            lists[i].push_back((int32_t)k);
        }
    }
    int64_t n_rank = 0;
    for (auto &L : lists) n_rank += (int64_t)L.size();
    int rc;
    if (!replay.empty()) {
        // (only the replay's host route checks ids on the host; the kernels count bad ids)
        for (int64_t k : replay)
            for (int64_t i = off[k]; i < off[k + 1]; ++i)
                if (ids[i] < 0 || ids[i] >= BPE_MAX_VOCAB)
                    return bpe_fail(BPE_ERR_VOCAB, "bpe native: token id out of range in text");
    }
    if ((rc = upload_table(E))) return rc;
    if (replay.empty() && total >= 2 * GROUP_TOKENS && !getenv("BPE_ENCODE_ONE_GROUP")) {
        std::vector<int32_t> shape_of((size_t)n_texts);
        for (int i = 0; i < N_SHAPES; ++i)
            for (int32_t k : lists[i]) shape_of[k] = i;
        return encode_groups(E, ids, off, n_texts, shape_of, ids_out, out_off);
    }
    // device: [ooff (n+2) | ids, then the packed output | off (n+2) | which | out | len].  A small
    // call's pinned host buffer mirrors [ooff | ids | off | which], so it moves [ids | off | which]
    // up in one copy and [ooff | packed ids] down in one; a large call copies its ids straight from
    // and to the caller's buffers and pins only [ooff | off | which].  off[n+1] = 0 is the bad-id
    // counter (zeroed by the upload), which the pack kernel copies to ooff[n+1].
    const size_t b_ids = align16((size_t)std::max<int64_t>(total, 1) * 4);
    const size_t b_off = align16((size_t)(n_texts + 2) * 8);
    const size_t b_which = align16((size_t)std::max<int64_t>(n_rank, 1) * 4);
    const size_t b_len = align16((size_t)n_texts * 4);
    const size_t bytes = b_off + b_ids + b_off + b_which + b_ids + b_len;
    // Large calls copy the ids straight from the caller's buffer (no host staging pass); small ones
    // through the pinned buffer (a pageable copy costs tens of microseconds of fixed overhead)
    const bool small = (size_t)total * 4 <= SMALL_CALL_BYTES;
    const size_t h_ids_bytes = small ? b_ids : 0;
    if ((rc = grow_stage(E, b_off + h_ids_bytes + b_off + b_which, bytes))) return rc;
    struct Release {
        bpe_encoder *e;
        ~Release() { release_stage(e); }
    } release{E};
    char *h = E->h_buf, *d = E->d_buf;
    int64_t *d_ooff = reinterpret_cast<int64_t *>(d);
    int32_t *d_ids = reinterpret_cast<int32_t *>(d + b_off);
    int64_t *d_off = reinterpret_cast<int64_t *>(d + b_off + b_ids);
    int32_t *d_which = reinterpret_cast<int32_t *>(d + b_off + b_ids + b_off);
    int32_t *d_out = reinterpret_cast<int32_t *>(d + b_off + b_ids + b_off + b_which);
    int32_t *d_len = reinterpret_cast<int32_t *>(d + b_off + 2 * b_ids + b_off + b_which);
    unsigned long long *d_err = reinterpret_cast<unsigned long long *>(d_off + n_texts + 1);
    int64_t *h_ooff = reinterpret_cast<int64_t *>(h);
    int32_t *h_ids = reinterpret_cast<int32_t *>(h + b_off);   // (small calls only)
    int64_t *h_off = reinterpret_cast<int64_t *>(h + b_off + h_ids_bytes);
    int32_t *h_which = reinterpret_cast<int32_t *>(h + b_off + h_ids_bytes + b_off);
    for (int64_t k = 0; k <= n_texts; ++k) h_off[k] = off[k] - base;
    h_off[n_texts + 1] = 0;
    size_t at = 0;
    for (auto &L : lists) {
        std::memcpy(h_which + at, L.data(), L.size() * 4);
        at += L.size();
    }
    if (small) {
        if (total) std::memcpy(h_ids, ids + base, (size_t)total * 4);
        ENC_TRY(hipMemcpyAsync(d_ids, h_ids, b_ids + b_off + (size_t)n_rank * 4, hipMemcpyHostToDevice,
                               E->stream));
    } else {
        ENC_TRY(hipMemcpyAsync(d_ids, ids + base, (size_t)total * 4, hipMemcpyHostToDevice, E->stream));
        ENC_TRY(hipMemcpyAsync(d_off, h_off, b_off + (size_t)n_rank * 4, hipMemcpyHostToDevice, E->stream));
    }
    // replay texts keep length 0 on the device; they are written on the host below
    if (!replay.empty()) ENC_TRY(hipMemsetAsync(d_len, 0, (size_t)n_texts * 4, E->stream));
    // few texts: each has a CU to itself, and the table is read from LDS (when it fits)
    const size_t tab = (size_t)E->lt.words * 4;
    const bool few = (size_t)n_rank <= LATENCY_TEXTS;
    ENC_TRY(hipEventRecord(E->ev0, E->stream));
    at = 0;
    for (int i = 0; i < N_SHAPES; ++i) {
        if (lists[i].empty()) continue;
        const bool tab_lds = few && shape_cap(i) > LDS_TAB_MIN_TOKENS && shape_lds(i) + tab <= LDS_BYTES;
        launch_shape(i, E, (unsigned)lists[i].size(), tab_lds, d_ids, d_off, d_which + at, d_out, d_len,
                     d_err);
        at += lists[i].size();
    }
    ENC_TRY(hipGetLastError());
    ENC_TRY(hipEventRecord(E->ev1, E->stream));
    if (replay.empty()) {
        // packed on the device, into the ids buffer (read by the kernels above, free now)
        if (n_texts <= 1024 && total <= (1 << 18)) {   // (one workgroup copies it all)
            k_pack_small<<<1, 1024, 0, E->stream>>>(d_out, d_off, d_len, (int)n_texts, d_ooff, d_err, d_ids);
        } else {
            k_scan_lens<<<1, 1024, 0, E->stream>>>(d_len, n_texts, d_ooff, d_err);
            k_gather<<<(unsigned)((n_texts + 3) / 4), 256, 0, E->stream>>>(d_out, d_off, d_len, d_ooff,
                                                                            n_texts, d_ids);
        }
        ENC_TRY(hipGetLastError());
        if (small) {
            ENC_TRY(hipMemcpyAsync(h_ooff, d_ooff, b_off + (size_t)total * 4, hipMemcpyDeviceToHost,
                                   E->stream));
            ENC_TRY(hipStreamSynchronize(E->stream));
            if (h_ooff[n_texts + 1]) return bpe_fail(BPE_ERR_VOCAB, "bpe native: token id out of range in text");
            std::memcpy(out_off, h_ooff, (size_t)(n_texts + 1) * 8);
            if (h_ooff[n_texts]) std::memcpy(ids_out, h_ids, (size_t)h_ooff[n_texts] * 4);
        } else {
            // the offsets first, then only the packed ids (merges shrink a batch: 5x on zipf words)
            ENC_TRY(hipMemcpyAsync(h_ooff, d_ooff, (size_t)(n_texts + 2) * 8, hipMemcpyDeviceToHost, E->stream));
            ENC_TRY(hipStreamSynchronize(E->stream));
            if (h_ooff[n_texts + 1]) return bpe_fail(BPE_ERR_VOCAB, "bpe native: token id out of range in text");
            const int64_t n_out = h_ooff[n_texts];
            if (n_out < 0 || n_out > total) return bpe_fail(BPE_ERR_STATE, "bpe native: bad packed length");
            if (n_out) {
                ENC_TRY(hipMemcpyAsync(ids_out, d_ids, (size_t)n_out * 4, hipMemcpyDeviceToHost, E->stream));
                ENC_TRY(hipStreamSynchronize(E->stream));
            }
            std::memcpy(out_off, h_ooff, (size_t)(n_texts + 1) * 8);
        }
    } else {
        // host assembly: the kernels' texts come back at their input offsets, the replayed ones
        // from the scratch engine (into the same host buffer: after the copies have landed)
        std::vector<int64_t> len((size_t)n_texts, 0);
        std::vector<int32_t> out((size_t)std::max<int64_t>(total, 1));
        std::vector<int32_t> lens((size_t)n_texts);
        unsigned long long err = 0;
        ENC_TRY(hipMemcpyAsync(out.data(), d_out, (size_t)total * 4, hipMemcpyDeviceToHost, E->stream));
        ENC_TRY(hipMemcpyAsync(lens.data(), d_len, (size_t)n_texts * 4, hipMemcpyDeviceToHost, E->stream));
        ENC_TRY(hipMemcpyAsync(&err, d_err, 8, hipMemcpyDeviceToHost, E->stream));
        ENC_TRY(hipStreamSynchronize(E->stream));
        if (err) return bpe_fail(BPE_ERR_VOCAB, "bpe native: token id out of range in text");
        if ((rc = encode_replay(E, ids, off, replay, out.data(), len.data()))) return rc;
        for (auto &L : lists)
            for (int32_t k : L) len[k] = lens[k];
        int64_t o = 0;
        out_off[0] = 0;
        for (int64_t k = 0; k < n_texts; ++k) {
            if (len[k]) std::memcpy(ids_out + o, out.data() + (off[k] - base), (size_t)len[k] * 4);
            o += len[k];
            out_off[k + 1] = o;
        }
    }
    float ms = 0;
    ENC_TRY(hipEventElapsedTime(&ms, E->ev0, E->ev1));
    E->st.kernel_ms += ms;
    E->st.texts_rank += n_rank;
    E->st.tokens_out += out_off[n_texts];
    return BPE_OK;
}

int bpe_encoder_get_stats(bpe_encoder *E, bpe_encoder_stats *out) {
    if (!E || !out) return bpe_fail(BPE_ERR_ARG, "bpe native: null argument");
    ENC_TRY(hipSetDevice(E->device));
    unsigned long long steps[8] = {};
    ENC_TRY(hipMemcpy(steps, E->d_steps, 64, hipMemcpyDeviceToHost));
    E->st.steps = (int64_t)steps[0];
    *out = E->st;
    return BPE_OK;
}

int bpe_encoder_reset_stats(bpe_encoder *E) {
    if (!E) return bpe_fail(BPE_ERR_ARG, "bpe native: null argument");
    ENC_TRY(hipSetDevice(E->device));
    ENC_TRY(hipMemset(E->d_steps, 0, 64));
    E->st = bpe_encoder_stats{};
    return BPE_OK;
}

}  // extern "C"
