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
#include <cstring>
#include <string>
#include <vector>

#include "bpe.h"
#include "bpe_multi.h"   // bpe_fail

namespace {

constexpr uint32_t NO_RANK = 0xFFFFu;
// tokens per workgroup buffer of each launch shape (LDS: 9 bytes per token)
constexpr int CAP_64 = 512;       //   4.5 KiB, one wave
constexpr int CAP_256 = 4096;     //  36 KiB
constexpr int CAP_1024 = 16384;   // 144 KiB of the CU's 160 KiB

#define ENC_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return bpe_fail(e_ == hipErrorOutOfMemory ? BPE_ERR_OOM : BPE_ERR_HIP,         \
                            (std::string("bpe native: ") + #expr + ": " +                   \
                             hipGetErrorString(e_)).c_str());                              \
    } while (0)

struct RankTab {
    const unsigned long long *slots;   // (a << 16 | b) << 32 | rank; empty = ~0
    uint32_t mask;
    uint32_t shift;                    // 32 - log2(slots)
    const uint16_t *c_of;              // rank -> new token id
};

__host__ __device__ __forceinline__ uint32_t rank_home(uint32_t key, uint32_t shift) {
    return (key * 0x9E3779B1u) >> shift;
}

__device__ __forceinline__ uint32_t rank_of(const RankTab &t, uint32_t x, uint32_t y) {
    const uint32_t key = (x << 16) | y;
    uint32_t h = rank_home(key, t.shift);
    for (;;) {
        const unsigned long long e = t.slots[h];
        if ((uint32_t)(e >> 32) == key) return (uint32_t)e & 0xFFFFu;
        if (e == ~0ull) return NO_RANK;
        h = (h + 1) & t.mask;
    }
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, d));
    return v;
}

__device__ __forceinline__ int wave_incl(int v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(v, d);
        if (lane >= d) v += o;
    }
    return v;
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
        total = __shfl(incl, 63);
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

// One text per workgroup: which[blockIdx.x] indexes the texts of this launch shape.  Output at the
// text's own input offsets (never longer than the input) plus its length.
template <int WG>
__global__ void __launch_bounds__(WG)
k_encode(const int32_t *__restrict__ in, const int64_t *__restrict__ off,
         const int32_t *__restrict__ which, int32_t *__restrict__ out, int32_t *__restrict__ out_len,
         RankTab t, int cap, unsigned long long *__restrict__ steps_total) {
    extern __shared__ uint16_t lds16[];
    __shared__ uint32_t red[WG / 64];
    __shared__ int scn[WG / 64];
    uint16_t *tok = lds16, *rk = lds16 + cap, *tok2 = lds16 + 2 * cap, *rk2 = lds16 + 3 * cap;
    uint8_t *fl = reinterpret_cast<uint8_t *>(lds16 + 4 * cap);

    const int text = which[blockIdx.x];
    const int64_t base = off[text];
    int n = (int)(off[text + 1] - base);
    const int tid = threadIdx.x;

    for (int i = tid; i < n; i += WG) tok[i] = (uint16_t)in[base + i];
    __syncthreads();
    uint32_t lmin = NO_RANK;
    for (int i = tid; i < n; i += WG) {
        const uint32_t r = i + 1 < n ? rank_of(t, tok[i], tok[i + 1]) : NO_RANK;
        rk[i] = (uint16_t)r;
        lmin = min(lmin, r);
    }
    uint32_t r = block_min<WG>(lmin, red);
    if (WG == 64) __syncthreads();
    int steps = 0;

    while (r != NO_RANK) {   // (uniform: every thread holds the same r)
        ++steps;
        const uint32_t c = t.c_of[r];
        const int k = (n + WG - 1) / WG;
        const int s = min(n, tid * k), e = min(n, s + k);
        // 1. counted occurrences of rank r in [s, e): even offsets inside an r-chain (x == y runs;
        //    for x != y a chain has length 1)
        int cnt = 0;
        {
            int d = 0;
            if (s < e)
                for (int j = s - 1; j >= 0 && rk[j] == r; --j) ++d;
            for (int i = s; i < e; ++i) {
                const bool m = rk[i] == r;
                const bool f = m && !(d & 1);
                fl[i] = f;
                cnt += f;
                d = m ? d + 1 : 0;
            }
        }
        // 2. destination of the segment: i - #counted in [0, i - 1) for its first live position
        int total = 0;
        const int before = block_scan<WG>(cnt, scn, total);   // (barrier: flags visible)
        int p = s - before + (s > 0 && s < e ? fl[s - 1] : 0);
        // 3. compacted rewrite; pairs touching c get their rank again
        lmin = NO_RANK;
        for (int i = s; i < e; ++i) {
            if (i > 0 && fl[i - 1]) continue;   // the b of a counted (a, b)
            const bool fi = fl[i];
            const uint32_t tv = fi ? c : tok[i];
            const int nx = fi ? i + 2 : i + 1;
            uint32_t rv = NO_RANK;
            if (nx < n) {
                const bool fn = fl[nx];
                rv = (fi || fn) ? rank_of(t, tv, fn ? c : tok[nx]) : rk[i];
            }
            tok2[p] = (uint16_t)tv;
            rk2[p] = (uint16_t)rv;
            ++p;
            lmin = min(lmin, rv);
        }
        n -= total;
        uint16_t *x = tok;
        tok = tok2;
        tok2 = x;
        x = rk;
        rk = rk2;
        rk2 = x;
        r = block_min<WG>(lmin, red);   // (barrier: the new buffer visible, the old one free)
        if (WG == 64) __syncthreads();
    }

    for (int i = tid; i < n; i += WG) out[base + i] = tok[i];
    if (tid == 0) {
        out_len[text] = n;
        if (steps_total && steps) atomicAdd(steps_total, (unsigned long long)steps);
    }
}

template <int WG>
constexpr int cap_of() {
    return WG == 64 ? CAP_64 : WG == 256 ? CAP_256 : CAP_1024;
}

template <int WG>
constexpr size_t lds_of() {
    return (size_t)cap_of<WG>() * 9;
}

}  // namespace

struct bpe_encoder {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::vector<int32_t> abc;                 // the merges, in rank order
    bool greedy_ok = true;                    // the rank-greedy form equals the replay (above)
    std::vector<uint8_t> is_input;            // ids used as a or b by the merges so far
    int32_t vocab = 0;                        // 1 + the largest id of the merges
    // rank table (host copy; uploaded when dirty)
    std::vector<unsigned long long> slots;
    uint32_t bits = 0;
    std::vector<uint16_t> c_of;
    bool dirty = true;
    unsigned long long *d_slots = nullptr;
    size_t d_slots_n = 0;
    uint16_t *d_c = nullptr;
    size_t d_c_n = 0;
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
            s = ((unsigned long long)key << 32) | rank;
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

int upload_table(bpe_encoder *E) {
    if (!E->dirty) return BPE_OK;
    int rc;
    if ((rc = grow_dev(&E->d_slots, &E->d_slots_n, E->slots.size()))) return rc;
    if ((rc = grow_dev(&E->d_c, &E->d_c_n, std::max<size_t>(E->c_of.size(), 1)))) return rc;
    ENC_TRY(hipMemcpyAsync(E->d_slots, E->slots.data(), E->slots.size() * 8, hipMemcpyHostToDevice,
                           E->stream));
    if (!E->c_of.empty())
        ENC_TRY(hipMemcpyAsync(E->d_c, E->c_of.data(), E->c_of.size() * 2, hipMemcpyHostToDevice,
                               E->stream));
    E->dirty = false;
    return BPE_OK;
}

int grow_stage(bpe_encoder *E, size_t bytes) {
    if (E->h_cap < bytes) {
        if (E->h_buf) (void)hipHostFree(E->h_buf);
        E->h_buf = nullptr;
        E->h_cap = 0;
        const size_t n = bytes * 3 / 2 + 4096;
        ENC_TRY(hipHostMalloc((void **)&E->h_buf, n, hipHostMallocDefault));
        E->h_cap = n;
    }
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
        hipEventCreate(&E->ev0) != hipSuccess || hipEventCreate(&E->ev1) != hipSuccess)
        return bail(bpe_fail(BPE_ERR_HIP, "bpe native: encoder stream/events"));
    if (hipMalloc((void **)&E->d_steps, 8) != hipSuccess ||
        hipMemset(E->d_steps, 0, 8) != hipSuccess)
        return bail(bpe_fail(BPE_ERR_OOM, "bpe native: encoder counters"));
    if (hipFuncSetAttribute((const void *)k_encode<1024>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds_of<1024>()) != hipSuccess ||
        hipFuncSetAttribute((const void *)k_encode<256>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds_of<256>()) != hipSuccess)
        return bail(bpe_fail(BPE_ERR_HIP, "bpe native: encoder LDS attribute"));
    table_rebuild(E, 10);
    *out = E;
    return BPE_OK;
}

int bpe_encoder_destroy(bpe_encoder *E) {
    if (!E) return BPE_OK;
    (void)hipSetDevice(E->device);
    if (E->stream) (void)hipStreamSynchronize(E->stream);
    if (E->scratch) bpe_destroy(E->scratch);
    if (E->d_slots) (void)hipFree(E->d_slots);
    if (E->d_c) (void)hipFree(E->d_c);
    if (E->d_steps) (void)hipFree(E->d_steps);
    if (E->d_buf) (void)hipFree(E->d_buf);
    if (E->h_buf) (void)hipHostFree(E->h_buf);
    if (E->ev0) (void)hipEventDestroy(E->ev0);
    if (E->ev1) (void)hipEventDestroy(E->ev1);
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
    for (int64_t i = 0; i < total; ++i)
        if (ids[base + i] < 0 || ids[base + i] >= BPE_MAX_VOCAB)
            return bpe_fail(BPE_ERR_VOCAB, "bpe native: token id out of range in text");
    ENC_TRY(hipSetDevice(E->device));
    E->st.calls++;
    E->st.tokens_in += total;
    std::vector<int64_t> len((size_t)n_texts);
    std::vector<int32_t> out((size_t)std::max<int64_t>(total, 1));
    const int64_t m = (int64_t)E->c_of.size();
    // launch shape of every text: 0/1/2 = k_encode<64/256/1024>, 3 = the apply-pass route
    std::vector<int32_t> lists[3];
    std::vector<int64_t> replay;
    for (int64_t k = 0; k < n_texts; ++k) {
        const int64_t l = off[k + 1] - off[k];
        if (m == 0 || l < 2) {
            std::memcpy(out.data() + (off[k] - base), ids + off[k], (size_t)l * 4);
            len[k] = l;
        } else if (!E->greedy_ok || l > CAP_1024) {
            replay.push_back(k);
        } else {
            lists[l <= CAP_64 ? 0 : l <= CAP_256 ? 1 : 2].push_back((int32_t)k);
        }
    }
    const int64_t n_rank = (int64_t)(lists[0].size() + lists[1].size() + lists[2].size());
    int rc;
    if (n_rank) {
        if ((rc = upload_table(E))) return rc;
        // staging: [ids | off (relative) | which lists] up, [out | len] down
        const size_t b_ids = align16((size_t)total * 4), b_off = align16((size_t)(n_texts + 1) * 8);
        const size_t b_which = align16((size_t)n_rank * 4), b_len = align16((size_t)n_texts * 4);
        const size_t up = b_ids + b_off + b_which, bytes = up + b_ids + b_len;
        if ((rc = grow_stage(E, bytes))) return rc;
        char *h = E->h_buf, *d = E->d_buf;
        std::memcpy(h, ids + base, (size_t)total * 4);
        int64_t *h_off = reinterpret_cast<int64_t *>(h + b_ids);
        for (int64_t k = 0; k <= n_texts; ++k) h_off[k] = off[k] - base;
        int32_t *h_which = reinterpret_cast<int32_t *>(h + b_ids + b_off);
        size_t at = 0;
        for (auto &L : lists) {
            std::memcpy(h_which + at, L.data(), L.size() * 4);
            at += L.size();
        }
        ENC_TRY(hipMemcpyAsync(d, h, up, hipMemcpyHostToDevice, E->stream));
        const int32_t *d_ids = reinterpret_cast<const int32_t *>(d);
        const int64_t *d_off = reinterpret_cast<const int64_t *>(d + b_ids);
        const int32_t *d_which = reinterpret_cast<const int32_t *>(d + b_ids + b_off);
        int32_t *d_out = reinterpret_cast<int32_t *>(d + up);
        int32_t *d_len = reinterpret_cast<int32_t *>(d + up + b_ids);
        RankTab t{E->d_slots, (1u << E->bits) - 1, 32 - E->bits, E->d_c};
        ENC_TRY(hipEventRecord(E->ev0, E->stream));
        at = 0;
        if (!lists[0].empty())
            k_encode<64><<<(unsigned)lists[0].size(), 64, lds_of<64>(), E->stream>>>(
                d_ids, d_off, d_which + at, d_out, d_len, t, CAP_64, E->d_steps);
        at += lists[0].size();
        if (!lists[1].empty())
            k_encode<256><<<(unsigned)lists[1].size(), 256, lds_of<256>(), E->stream>>>(
                d_ids, d_off, d_which + at, d_out, d_len, t, CAP_256, E->d_steps);
        at += lists[1].size();
        if (!lists[2].empty())
            k_encode<1024><<<(unsigned)lists[2].size(), 1024, lds_of<1024>(), E->stream>>>(
                d_ids, d_off, d_which + at, d_out, d_len, t, CAP_1024, E->d_steps);
        ENC_TRY(hipGetLastError());
        ENC_TRY(hipEventRecord(E->ev1, E->stream));
        ENC_TRY(hipMemcpyAsync(h + up, d + up, b_ids + b_len, hipMemcpyDeviceToHost, E->stream));
        // the long texts replay on the scratch engine's own stream meanwhile
        if ((rc = encode_replay(E, ids, off, replay, out.data(), len.data()))) return rc;
        ENC_TRY(hipStreamSynchronize(E->stream));
        float ms = 0;
        ENC_TRY(hipEventElapsedTime(&ms, E->ev0, E->ev1));
        E->st.kernel_ms += ms;
        E->st.texts_rank += n_rank;
        const int32_t *h_out = reinterpret_cast<const int32_t *>(h + up);
        const int32_t *h_len = reinterpret_cast<const int32_t *>(h + up + b_ids);
        for (auto &L : lists)
            for (int32_t k : L) {
                len[k] = h_len[k];
                std::memcpy(out.data() + (off[k] - base), h_out + (off[k] - base), (size_t)h_len[k] * 4);
            }
    } else if ((rc = encode_replay(E, ids, off, replay, out.data(), len.data()))) {
        return rc;
    }
    int64_t o = 0;
    out_off[0] = 0;
    for (int64_t k = 0; k < n_texts; ++k) {
        if (len[k]) std::memcpy(ids_out + o, out.data() + (off[k] - base), (size_t)len[k] * 4);
        o += len[k];
        out_off[k + 1] = o;
    }
    E->st.tokens_out += o;
    return BPE_OK;
}

int bpe_encoder_get_stats(bpe_encoder *E, bpe_encoder_stats *out) {
    if (!E || !out) return bpe_fail(BPE_ERR_ARG, "bpe native: null argument");
    ENC_TRY(hipSetDevice(E->device));
    unsigned long long steps = 0;
    ENC_TRY(hipMemcpy(&steps, E->d_steps, 8, hipMemcpyDeviceToHost));
    E->st.steps = (int64_t)steps;
    *out = E->st;
    return BPE_OK;
}

int bpe_encoder_reset_stats(bpe_encoder *E) {
    if (!E) return bpe_fail(BPE_ERR_ARG, "bpe native: null argument");
    ENC_TRY(hipSetDevice(E->device));
    ENC_TRY(hipMemset(E->d_steps, 0, 8));
    E->st = bpe_encoder_stats{};
    return BPE_OK;
}

}  // extern "C"
