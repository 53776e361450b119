// bpe_multi.cpp — one corpus sharded over several HIP devices behind ONE bpe_ctx
// (bpe_create_multi, include/bpe.h): the drop-in's BPE_NUM_GPUS, so that `new BPETokenizer()`
// (core.ts:77) and every corpus-touching method keep their surface while the corpus spans the
// GPUs of the node.
//
// Layout.  Shard r is an ordinary single-device context holding a contiguous run of whole
// samples, in corpus order: pairs never cross samples (core.ts:265-267), so each shard counts
// and rewrites its samples alone, and rule R3's "earliest last occurrence" compares
// (shard, shard-local position) lexicographically.  Samples added before the first pass over the
// corpus are staged on the host and then cut into n runs of about equal token counts; samples
// added later go to the last shard (corpus order is kept).
//
// Exchange per merge iteration (the device-resident rank loop of every shard, bpe_rank_loop_*):
//   all-reduce(SUM) of the 81920-bin pair table -> selection on every shard from the same global
//   table -> all-reduce(MAX) of the tied candidates' (shard << 40 | last position) -> decision ->
//   the fused apply + count pass of every shard.
// The all-reduces run over RCCL (one communicator per device, ncclCommInitAll, grouped calls on
// the shards' streams) or, for shards sharing a device (tests), as host copies.  An iteration the
// rank loop cannot finish (heavy sketch buckets, many tied pairs) takes the host protocol: global
// table, exact counts of the heavy cold pairs on every shard, global selection, tie positions.
#include "bpe_multi.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

extern "C" int bpe_leave_global(bpe_ctx *c);

namespace {

constexpr int64_t RANK_SHIFT = 40;   // as sharded.py / k_tie_export: rank << 40 | position

struct Rccl {
    void *so = nullptr;
    ncclResult_t (*init_all)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*all_reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t,
                               ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
};

}  // namespace

struct bpe_multi {
    int n = 0;
    int reduce = BPE_REDUCE_HOST;
    std::vector<int> dev;
    std::vector<bpe_ctx *> sh;
    std::vector<hipStream_t> st;
    std::vector<unsigned long long *> d_table, d_tie;   // per shard, on its device
    std::vector<unsigned long long *> d_xchg;            // per shard: the rank loop's exchange
    std::vector<uint32_t *> d_keys;                      // per shard: exact cold-pair lists
    std::vector<unsigned long long *> d_counts;
    int64_t cold_cap = 0;
    unsigned long long *h_buf = nullptr, *h_sum = nullptr;   // pinned, BPE_XCHG_WORDS each
    std::vector<std::vector<int32_t>> staged;            // samples not yet on a device
    bool distributed = false;
    // the maintained state (every shard holds the global tables, bpe_set_global_counts), and the
    // host-protocol iterations in a row that needed exact cold counts (two: enter that state)
    bool maintained = false;
    int heavy_streak = 0;
    // the incremental mode (bpe_set_mode): the global state lives in every shard's position
    // index, entered at the first batch; entries counts them (one index build each), and a run
    // whose batches keep handing over goes on in the streaming mode (pix_off)
    bool pix = false, pix_off = false;
    // (since the last bpe_set_mode: index entries, merges made; fallbacks: times pix_off was set)
    int64_t pix_entries = 0, pix_merged = 0, pix_fallbacks = 0;
    // the streaming mode went on in the incremental mode past AUTO_PIX_VOCAB token ids (round 5)
    bool pix_auto = false;
    // the caller chose a mode (bpe_set_mode): the automatic switch to the incremental mode past
    // AUTO_PIX_VOCAB ids then leaves it alone
    bool mode_explicit = false;
    std::vector<ncclComm_t> comms;
    Rccl rccl;
    // shards sharing one device (the one-GPU test box, BPE_REDUCE_HOST): the exchange is a device
    // kernel on shard 0's stream, ordered by events, with no host copies or syncs
    bool one_device = false;
    std::vector<hipEvent_t> ev;
    hipEvent_t ev_done = nullptr;
};

namespace {

#define MHIP(expr)                                                                         \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return bpe_fail(e_ == hipErrorOutOfMemory ? BPE_ERR_OOM : BPE_ERR_HIP,        \
                            (std::string("bpe native: ") + #expr + ": " +                 \
                             hipGetErrorString(e_)).c_str());                              \
    } while (0)

#define MTRY(expr)                 \
    do {                           \
        int rc_ = (expr);          \
        if (rc_ < 0) return rc_;   \
    } while (0)

// RCCL has to run on the same HIP runtime as libbpe.  A process can hold two: PyTorch's wheel
// bundles libamdhip64 and librccl under the same sonames as /opt/rocm/lib, and when libbpe is
// loaded before `import torch` both runtimes end up in the process.  A plain dlopen("librccl.so.1")
// would then return torch's RCCL (already loaded, same soname), whose HIP runtime finds no device
// ("ncclCommInitAll: unhandled cuda error").  So the RCCL in the directory of libbpe's own
// libamdhip64 comes first, by path.
int load_rccl(Rccl &r) {
    Dl_info info{};
    if (dladdr(reinterpret_cast<void *>(&hipGetDeviceCount), &info) && info.dli_fname) {
        std::string dir(info.dli_fname);
        const size_t slash = dir.rfind('/');
        if (slash != std::string::npos) {
            dir.resize(slash + 1);
            for (const char *nm : {"librccl.so.1", "librccl.so"})
                if ((r.so = dlopen((dir + nm).c_str(), RTLD_NOW | RTLD_LOCAL))) break;
        }
    }
    const char *names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char *nm : names)
        if (!r.so && (r.so = dlopen(nm, RTLD_NOW | RTLD_LOCAL))) break;
    if (!r.so) return bpe_fail(BPE_ERR_HIP, "bpe native: RCCL (librccl.so) not found");
    r.init_all = (decltype(r.init_all))dlsym(r.so, "ncclCommInitAll");
    r.all_reduce = (decltype(r.all_reduce))dlsym(r.so, "ncclAllReduce");
    r.group_start = (decltype(r.group_start))dlsym(r.so, "ncclGroupStart");
    r.group_end = (decltype(r.group_end))dlsym(r.so, "ncclGroupEnd");
    r.destroy = (decltype(r.destroy))dlsym(r.so, "ncclCommDestroy");
    r.error_string = (decltype(r.error_string))dlsym(r.so, "ncclGetErrorString");
    r.get_unique_id = (decltype(r.get_unique_id))dlsym(r.so, "ncclGetUniqueId");
    r.init_rank = (decltype(r.init_rank))dlsym(r.so, "ncclCommInitRank");
    if (!r.init_all || !r.all_reduce || !r.group_start || !r.group_end || !r.destroy)
        return bpe_fail(BPE_ERR_HIP, "bpe native: RCCL symbols missing");
    return BPE_OK;
}

int nccl_check(bpe_multi *m, ncclResult_t r, const char *what) {
    if (r == ncclSuccess) return BPE_OK;
    std::string msg = std::string("bpe native: ") + what + ": " +
                      (m->rccl.error_string ? m->rccl.error_string(r) : "RCCL error");
    return bpe_fail(BPE_ERR_HIP, msg.c_str());
}

// In-place all-reduce of count u64 per shard (SUM or MAX), ordered on the shards' streams.
int all_reduce(bpe_multi *m, std::vector<unsigned long long *> &buf, size_t count, bool max) {
    // (one shard: nothing to add, but an RCCL context still makes the call, so that the RCCL leg
    // of the rank loop runs on a one-GPU box as it does on eight)
    if (m->n == 1 && m->reduce != BPE_REDUCE_RCCL) return BPE_OK;
    if (m->reduce == BPE_REDUCE_RCCL) {
        MTRY(nccl_check(m, m->rccl.group_start(), "ncclGroupStart"));
        for (int r = 0; r < m->n; ++r) {
            ncclResult_t e = m->rccl.all_reduce(buf[r], buf[r], count, ncclUint64,
                                                max ? ncclMax : ncclSum, m->comms[r], m->st[r]);
            if (e != ncclSuccess) {
                m->rccl.group_end();
                return nccl_check(m, e, "ncclAllReduce");
            }
        }
        return nccl_check(m, m->rccl.group_end(), "ncclGroupEnd");
    }
    if (m->one_device) {
        MHIP(hipSetDevice(m->dev[0]));
        for (int r = 0; r < m->n; ++r) {
            MHIP(hipEventRecord(m->ev[r], m->st[r]));
            MHIP(hipStreamWaitEvent(m->st[0], m->ev[r], 0));
        }
        MTRY(bpe_sum_shards(buf.data(), m->n, count, max ? 1 : 0, m->st[0]));
        MHIP(hipEventRecord(m->ev_done, m->st[0]));
        for (int r = 1; r < m->n; ++r) MHIP(hipStreamWaitEvent(m->st[r], m->ev_done, 0));
        return BPE_OK;
    }
    // host copies (shards on several devices without RCCL): after each shard's stream has
    // produced its part
    for (int r = 0; r < m->n; ++r) {
        MHIP(hipSetDevice(m->dev[r]));
        MHIP(hipMemcpyAsync(m->h_buf, buf[r], count * 8, hipMemcpyDeviceToHost, m->st[r]));
        MHIP(hipStreamSynchronize(m->st[r]));
        static const bool dbg = getenv("BPE_DEBUG_GLOBAL") != nullptr;
        if (dbg && !max)
            for (size_t i = 0; i < count; ++i)
                if (m->h_buf[i] >> 32)
                    fprintf(stderr, "[bpe debug] all-reduce: shard %d word %zu (other %lld row %lld) = %llu = 0x%llx\n",
                            r, i, (long long)((i - 8) / 6), (long long)((i - 8) % 6), m->h_buf[i], m->h_buf[i]);
        if (r == 0) {
            std::memcpy(m->h_sum, m->h_buf, count * 8);
        } else if (max) {
            for (size_t i = 0; i < count; ++i) m->h_sum[i] = std::max(m->h_sum[i], m->h_buf[i]);
        } else {
            for (size_t i = 0; i < count; ++i) m->h_sum[i] += m->h_buf[i];
        }
    }
    for (int r = 0; r < m->n; ++r) {
        MHIP(hipSetDevice(m->dev[r]));
        MHIP(hipMemcpyAsync(buf[r], m->h_sum, count * 8, hipMemcpyHostToDevice, m->st[r]));
        MHIP(hipStreamSynchronize(m->st[r]));   // (h_sum is reused by the next reduction)
    }
    return BPE_OK;
}

// ---- the batch enqueued by one host thread per shard ---------------------------------------------
// (round 5) Each iteration of the rank loop enqueues about eight launches per shard plus the two
// exchanges; from one host thread, eight shards' enqueues bounded the one-process driver.  Each
// shard's thread enqueues its own kernels on its own stream.  The RCCL exchange needs no host
// coordination (one communicator per thread, as NCCL's one-thread-per-GPU use); the device-kernel
// exchange of shards sharing a device meets at a spin barrier twice per all-reduce (every shard's
// event recorded, then shard 0's sum kernel enqueued behind them and its event recorded).
struct SpinBarrier {
    explicit SpinBarrier(int n) : n(n) {}
    int n;
    std::atomic<int> count{0}, gen{0};
    std::atomic<bool> abort{false};
    bool wait() {
        const int g = gen.load(std::memory_order_acquire);
        if (count.fetch_add(1, std::memory_order_acq_rel) == n - 1) {
            count.store(0, std::memory_order_relaxed);
            gen.fetch_add(1, std::memory_order_release);
            return !abort.load(std::memory_order_relaxed);
        }
        for (int spin = 0; gen.load(std::memory_order_acquire) == g; ++spin) {
            if (abort.load(std::memory_order_relaxed)) return false;
            if (spin > 4096) std::this_thread::yield();
        }
        return !abort.load(std::memory_order_relaxed);
    }
};

constexpr int ABORTED = -1000;   // (another shard's thread failed: this one stops, no message)
constexpr int32_t AUTO_PIX_VOCAB = 18432;   // (INCR_RLIM, bpe_kernels.hip.h)

int shard_all_reduce(bpe_multi *m, int r, SpinBarrier &bar, std::vector<unsigned long long *> &buf,
                     size_t count, bool max) {
    if (m->reduce == BPE_REDUCE_RCCL) {
        const ncclResult_t e = m->rccl.all_reduce(buf[r], buf[r], count, ncclUint64,
                                                  max ? ncclMax : ncclSum, m->comms[r], m->st[r]);
        return nccl_check(m, e, "ncclAllReduce");
    }
    // one device: every shard's part, then the sum on shard 0's stream, then every shard after it
    MHIP(hipEventRecord(m->ev[r], m->st[r]));
    if (!bar.wait()) return ABORTED;
    if (r == 0) {
        for (int q = 0; q < m->n; ++q) MHIP(hipStreamWaitEvent(m->st[0], m->ev[q], 0));
        MTRY(bpe_sum_shards(buf.data(), m->n, count, max ? 1 : 0, m->st[0]));
        MHIP(hipEventRecord(m->ev_done, m->st[0]));
    }
    if (!bar.wait()) return ABORTED;
    if (r != 0) MHIP(hipStreamWaitEvent(m->st[r], m->ev_done, 0));
    return BPE_OK;
}

// `want` iterations of every shard's rank loop (bpe_rank_loop_begin done on every shard), nw words
// of exchange per iteration.
int enqueue_batch(bpe_multi *m, int64_t want, size_t nw) {
    static const bool one_thread = getenv("BPE_MULTI_ONE_THREAD") != nullptr;   // (A/B knob)
    if (m->n == 1 || one_thread || (m->reduce != BPE_REDUCE_RCCL && !m->one_device)) {
        for (int64_t i = 0; i < want; ++i) {
            MTRY(all_reduce(m, m->d_xchg, nw, false));
            for (auto s : m->sh) MTRY(bpe_rank_loop_select(s));
            MTRY(all_reduce(m, m->d_tie, BPE_TIE_WORDS, true));
            for (auto s : m->sh) MTRY(bpe_rank_loop_decide(s));
            for (auto s : m->sh) MTRY(bpe_rank_loop_count(s));
        }
        return BPE_OK;
    }
    SpinBarrier bar(m->n);
    std::vector<int> rcs(m->n, BPE_OK);
    std::vector<std::string> msgs(m->n);
    auto work = [&](int r) {
        auto run = [&]() -> int {
            MHIP(hipSetDevice(m->dev[r]));
            for (int64_t i = 0; i < want; ++i) {
                MTRY(shard_all_reduce(m, r, bar, m->d_xchg, nw, false));
                MTRY(bpe_rank_loop_select(m->sh[r]));
                MTRY(shard_all_reduce(m, r, bar, m->d_tie, BPE_TIE_WORDS, true));
                MTRY(bpe_rank_loop_decide(m->sh[r]));
                MTRY(bpe_rank_loop_count(m->sh[r]));
            }
            return BPE_OK;
        };
        rcs[r] = run();
        if (rcs[r] < 0 && rcs[r] != ABORTED) {
            char buf[512];
            bpe_last_error(buf, sizeof buf);   // (this thread's message: republished by the caller)
            msgs[r] = buf;
            bar.abort.store(true);
        }
    };
    std::vector<std::thread> th;
    for (int r = 1; r < m->n; ++r) th.emplace_back(work, r);
    work(0);
    for (auto &t : th) t.join();
    for (int r = 0; r < m->n; ++r)
        if (rcs[r] < 0 && rcs[r] != ABORTED) return bpe_fail(rcs[r], msgs[r].c_str());
    return BPE_OK;
}

// The staged samples, cut into n contiguous runs of about equal token counts.
int distribute(bpe_multi *m) {
    if (m->distributed) return BPE_OK;
    m->distributed = true;
    int64_t total = 0;
    for (auto &s : m->staged) total += (int64_t)s.size();
    int64_t acc = 0;
    for (auto &s : m->staged) {
        const int64_t len = (int64_t)s.size();
        int r = total ? (int)std::min<int64_t>(m->n - 1, (acc + len / 2) * m->n / total) : 0;
        MTRY(bpe_add_sample(m->sh[r], s.data(), len));
        acc += len;
        std::vector<int32_t>().swap(s);
    }
    m->staged.clear();
    return BPE_OK;
}

int ensure_cold_bufs(bpe_multi *m, int64_t need) {
    if (need <= m->cold_cap) return BPE_OK;
    int64_t cap = std::max<int64_t>(need, std::max<int64_t>(1 << 16, 2 * m->cold_cap));
    for (int r = 0; r < m->n; ++r) {
        MHIP(hipSetDevice(m->dev[r]));
        if (m->d_keys[r]) (void)hipFree(m->d_keys[r]);
        if (m->d_counts[r]) (void)hipFree(m->d_counts[r]);
        m->d_keys[r] = nullptr;
        m->d_counts[r] = nullptr;
        MHIP(hipMalloc((void **)&m->d_keys[r], cap * sizeof(uint32_t)));
        MHIP(hipMalloc((void **)&m->d_counts[r], cap * sizeof(unsigned long long)));
    }
    m->cold_cap = cap;
    return BPE_OK;
}

}  // namespace

// ---- lifecycle -----------------------------------------------------------------------------------
int multi_create(bpe_multi **out, int n, const int *devices, int reduce) {
    *out = nullptr;
    if (n < 1 || (reduce != BPE_REDUCE_RCCL && reduce != BPE_REDUCE_HOST))
        return bpe_fail(BPE_ERR_ARG, "bpe native: bad multi-device arguments");
    int n_dev = 0;
    if (hipGetDeviceCount(&n_dev) != hipSuccess || n_dev == 0)
        return bpe_fail(BPE_ERR_HIP, "bpe native: no HIP device available (MI355X required)");
    bpe_multi *m = new bpe_multi();
    m->n = n;
    m->reduce = reduce;
    for (int r = 0; r < n; ++r) m->dev.push_back(devices ? devices[r] : r);
    auto bail = [&](int rc) {
        multi_destroy(m);
        return rc;
    };
    for (int r = 0; r < n; ++r) {
        if (m->dev[r] < 0 || m->dev[r] >= n_dev)
            return bail(bpe_fail(BPE_ERR_ARG, "bpe native: bad device index"));
        for (int q = 0; q < r; ++q)
            if (m->dev[q] == m->dev[r] && reduce == BPE_REDUCE_RCCL)
                return bail(bpe_fail(BPE_ERR_ARG, "bpe native: RCCL needs one shard per device "
                                                  "(use BPE_REDUCE_HOST for shared devices)"));
    }
    m->sh.assign(n, nullptr);
    m->st.assign(n, nullptr);
    m->d_table.assign(n, nullptr);
    m->d_tie.assign(n, nullptr);
    m->d_xchg.assign(n, nullptr);
    m->d_keys.assign(n, nullptr);
    m->d_counts.assign(n, nullptr);
    for (int r = 0; r < n; ++r) {
        int rc = bpe_create(&m->sh[r], m->dev[r]);
        if (rc) return bail(rc);
        void *s = nullptr;
        bpe_get_stream(m->sh[r], &s);
        m->st[r] = (hipStream_t)s;
        if (hipSetDevice(m->dev[r]) != hipSuccess ||
            hipMalloc((void **)&m->d_table[r], BPE_TABLE_BINS * 8) != hipSuccess ||
            hipMalloc((void **)&m->d_xchg[r], BPE_XCHG_WORDS * 8) != hipSuccess ||
            hipMalloc((void **)&m->d_tie[r], BPE_TIE_WORDS * 8) != hipSuccess)
            return bail(bpe_fail(BPE_ERR_OOM, "bpe native: multi-device buffers"));
        // the rank loop owes the caller nothing about these buffers' contents (bpe.h): a poison
        // pattern makes any reliance on zeroed memory fail the same way on every run
        if (hipMemset(m->d_xchg[r], 0xA5, BPE_XCHG_WORDS * 8) != hipSuccess ||
            hipMemset(m->d_tie[r], 0xA5, BPE_TIE_WORDS * 8) != hipSuccess)
            return bail(bpe_fail(BPE_ERR_OOM, "bpe native: multi-device buffers"));
    }
    m->one_device = reduce == BPE_REDUCE_HOST && n <= BPE_MAX_SHARDS_ONE_DEVICE &&
                    std::all_of(m->dev.begin(), m->dev.end(), [&](int d) { return d == m->dev[0]; }) &&
                    !getenv("BPE_HOST_EXCHANGE");   // (A/B knob: the host-copy exchange)
    if (m->one_device) {
        (void)hipSetDevice(m->dev[0]);
        m->ev.assign(n, nullptr);
        for (int r = 0; r < n; ++r)
            if (hipEventCreateWithFlags(&m->ev[r], hipEventDisableTiming) != hipSuccess)
                return bail(bpe_fail(BPE_ERR_HIP, "bpe native: hipEventCreate failed"));
        if (hipEventCreateWithFlags(&m->ev_done, hipEventDisableTiming) != hipSuccess)
            return bail(bpe_fail(BPE_ERR_HIP, "bpe native: hipEventCreate failed"));
    }
    if (hipHostMalloc((void **)&m->h_buf, BPE_XCHG_WORDS * 8, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void **)&m->h_sum, BPE_XCHG_WORDS * 8, hipHostMallocDefault) != hipSuccess)
        return bail(bpe_fail(BPE_ERR_OOM, "bpe native: pinned host buffers"));
    if (reduce == BPE_REDUCE_RCCL) {   // (one device too: a 1-rank communicator)
        int rc = load_rccl(m->rccl);
        if (rc) return bail(rc);
        m->comms.assign(n, nullptr);
        rc = nccl_check(m, m->rccl.init_all(m->comms.data(), n, m->dev.data()), "ncclCommInitAll");
        if (rc) {
            m->comms.clear();
            return bail(rc);
        }
    }
    *out = m;
    return BPE_OK;
}

int multi_destroy(bpe_multi *m) {
    if (!m) return BPE_OK;
    for (auto c : m->comms)
        if (c && m->rccl.destroy) m->rccl.destroy(c);
    for (int r = 0; r < (int)m->sh.size(); ++r) {
        (void)hipSetDevice(m->dev[r]);
        if (m->sh[r]) bpe_destroy(m->sh[r]);
        void *ptrs[] = {m->d_table[r], m->d_tie[r], m->d_xchg[r], m->d_keys[r], m->d_counts[r]};
        for (void *p : ptrs)
            if (p) (void)hipFree(p);
    }
    for (auto e : m->ev)
        if (e) (void)hipEventDestroy(e);
    if (m->ev_done) (void)hipEventDestroy(m->ev_done);
    if (m->h_buf) (void)hipHostFree(m->h_buf);
    if (m->h_sum) (void)hipHostFree(m->h_sum);
    if (m->rccl.so) dlclose(m->rccl.so);
    delete m;
    return BPE_OK;
}

int multi_shard_count(bpe_multi *m, int *n) {
    *n = m->n;
    return BPE_OK;
}

int multi_set_mode(bpe_multi *m, int mode, bool explicit_choice) {
    for (auto s : m->sh) MTRY(bpe_set_mode(s, mode));
    if (explicit_choice) m->mode_explicit = true;
    m->pix = mode == BPE_MODE_INCREMENTAL;
    m->pix_auto = false;
    m->pix_off = false;
    m->pix_entries = m->pix_merged = 0;
    m->maintained = false;   // (the next batch enters the mode's own global state)
    m->heavy_streak = 0;
    for (auto s : m->sh) MTRY(bpe_leave_global(s));
    return BPE_OK;
}

// ---- vocabulary and corpus ------------------------------------------------------------------------
int multi_set_token_len16(bpe_multi *m, int32_t id, int32_t len16) {
    for (auto s : m->sh) MTRY(bpe_set_token_len16(s, id, len16));
    return BPE_OK;
}

int check_vocab(bpe_multi *m, int32_t *n_tokens);

// A sample added to the last shard reseals only that shard, which drops its replicated global
// tables (the maintained state).  Every shard must leave that state alike, or the next batch's
// exchange sizes differ between shards: the next batch then starts from the table state.
int drop_global(bpe_multi *m) {
    m->maintained = false;
    m->heavy_streak = 0;
    for (auto s : m->sh) MTRY(bpe_leave_global(s));
    return BPE_OK;
}

int multi_num_tokens(bpe_multi *m, int32_t *n) { return bpe_num_tokens(m->sh[0], n); }

int multi_add_sample(bpe_multi *m, const int32_t *ids, int64_t n) {
    for (int64_t i = 0; i < n; ++i)
        if (ids[i] < 0 || ids[i] >= BPE_MAX_VOCAB)
            return bpe_fail(BPE_ERR_ARG, "bpe native: token id out of range in sample");
    // every shard knows every token before any shard sees it: a new id grows the vocabulary of
    // all of them alike, so the next merge numbers its token the same on every shard
    int32_t mx = -1;
    for (int64_t i = 0; i < n; ++i) mx = std::max(mx, ids[i]);
    int32_t nt = 0;
    MTRY(bpe_num_tokens(m->sh[0], &nt));
    for (int32_t id = nt; id <= mx; ++id) MTRY(multi_set_token_len16(m, id, 1));
    if (m->distributed) {
        MTRY(bpe_add_sample(m->sh.back(), ids, n));   // (corpus order kept)
        return drop_global(m);
    }
    m->staged.emplace_back(ids, ids + n);
    return BPE_OK;
}

// The shards' vocabularies must agree (every new id is numbered by the vocabulary size).
int check_vocab(bpe_multi *m, int32_t *n_tokens) {
    int32_t n0 = 0;
    MTRY(bpe_num_tokens(m->sh[0], &n0));
    for (int r = 1; r < m->n; ++r) {
        int32_t nr = 0;
        MTRY(bpe_num_tokens(m->sh[r], &nr));
        if (nr != n0) return bpe_fail(BPE_ERR_STATE, "bpe native: shards disagree on the vocabulary size");
    }
    if (n_tokens) *n_tokens = n0;
    return BPE_OK;
}

int multi_add_latin1(bpe_multi *m, const uint8_t *bytes, int64_t n, int64_t sample_bytes,
                     int32_t char_to_id[256], int32_t *n_tokens_io, int64_t char_hist[256]) {
    const int32_t nt0 = *n_tokens_io;
    if (m->distributed || !m->staged.empty() || n == 0) {
        // after other samples: all of it to the end of the corpus
        MTRY(distribute(m));
        MTRY(bpe_add_latin1(m->sh.back(), bytes, n, sample_bytes, char_to_id, n_tokens_io,
                            char_hist));
    } else {
        // a fresh corpus: whole samples cut into n contiguous parts, in order (the char map is
        // threaded through the parts, so ids follow the corpus-wide first appearance)
        if (sample_bytes == 0 || sample_bytes > n) sample_bytes = n;
        const int64_t n_smp = (n + sample_bytes - 1) / sample_bytes;
        int64_t hist[256] = {0}, part[256];
        int64_t s0 = 0;
        for (int r = 0; r < m->n; ++r) {
            const int64_t s1 = r == m->n - 1 ? n_smp : n_smp * (r + 1) / m->n;
            const int64_t b0 = s0 * sample_bytes, b1 = std::min(n, s1 * sample_bytes);
            if (b1 > b0) {
                MTRY(bpe_add_latin1(m->sh[r], bytes + b0, b1 - b0, sample_bytes, char_to_id,
                                    n_tokens_io, part));
                for (int ch = 0; ch < 256; ++ch) hist[ch] += part[ch];
            }
            s0 = s1;
        }
        m->distributed = true;
        if (char_hist) std::memcpy(char_hist, hist, sizeof hist);
    }
    // every shard knows every token (new ids are numbered by the vocabulary size)
    for (int32_t id = nt0; id < *n_tokens_io; ++id) MTRY(multi_set_token_len16(m, id, 1));
    return drop_global(m);
}

int multi_clear_corpus(bpe_multi *m) {
    m->staged.clear();
    m->distributed = false;
    m->maintained = false;
    m->heavy_streak = 0;
    for (auto s : m->sh) MTRY(bpe_clear_corpus(s));
    return BPE_OK;
}

int multi_corpus_size(bpe_multi *m, int64_t *n_samples, int64_t *n_tokens) {
    int64_t ns = 0, nt = 0;
    for (auto s : m->sh) {
        int64_t a = 0, b = 0;
        MTRY(bpe_corpus_size(s, &a, &b));
        ns += a;
        nt += b;
    }
    for (auto &s : m->staged) {
        ns += 1;
        nt += (int64_t)s.size();
    }
    if (n_samples) *n_samples = ns;
    if (n_tokens) *n_tokens = nt;
    return BPE_OK;
}

int multi_read_corpus(bpe_multi *m, int32_t *ids_out, int64_t ids_cap, int64_t *sample_off,
                      int64_t off_cap) {
    MTRY(distribute(m));
    int64_t ns = 0, nt = 0;
    MTRY(multi_corpus_size(m, &ns, &nt));
    if (ids_cap < nt || off_cap < ns + 1 || (nt && !ids_out) || !sample_off)
        return bpe_fail(BPE_ERR_ARG, "bpe native: read_corpus buffers too small");
    int64_t o = 0, k = 0;
    sample_off[0] = 0;
    for (auto s : m->sh) {
        int64_t a = 0, b = 0;
        MTRY(bpe_corpus_size(s, &a, &b));
        std::vector<int64_t> off(a + 1);
        MTRY(bpe_read_corpus(s, ids_out ? ids_out + o : nullptr, b, off.data(), a + 1));
        for (int64_t i = 1; i <= a; ++i) sample_off[++k] = o + off[i];
        o += b;
    }
    return BPE_OK;
}

// Per-sample lengths and sample reads: the shards hold consecutive runs of samples, so sample i
// of the corpus is sample i - first[r] of the shard r whose run contains it.
int multi_sample_lengths(bpe_multi *m, int64_t *lens, int64_t cap) {
    MTRY(distribute(m));
    int64_t ns = 0;
    MTRY(multi_corpus_size(m, &ns, nullptr));
    if (cap < ns || (ns && !lens)) return bpe_fail(BPE_ERR_ARG, "bpe native: sample_lengths buffer too small");
    int64_t k = 0;
    for (auto s : m->sh) {
        int64_t a = 0;
        MTRY(bpe_corpus_size(s, &a, nullptr));
        MTRY(bpe_sample_lengths(s, lens + k, a));
        k += a;
    }
    return BPE_OK;
}

int multi_read_samples(bpe_multi *m, const int64_t *idx, int64_t n, int32_t *ids_out,
                       int64_t ids_cap, int64_t *off) {
    MTRY(distribute(m));
    if (n < 0 || (n && !idx) || !off) return bpe_fail(BPE_ERR_ARG, "bpe native: bad read_samples arguments");
    std::vector<int64_t> first(m->n + 1, 0);
    for (int r = 0; r < m->n; ++r) {
        int64_t a = 0;
        MTRY(bpe_corpus_size(m->sh[r], &a, nullptr));
        first[r + 1] = first[r] + a;
    }
    // per shard: its requested samples (local indices) and where each goes in the answer
    std::vector<std::vector<int64_t>> local(m->n), slot(m->n);
    for (int64_t k = 0; k < n; ++k) {
        if (idx[k] < 0 || idx[k] >= first[m->n])
            return bpe_fail(BPE_ERR_ARG, "bpe native: sample index out of range");
        const int r = (int)(std::upper_bound(first.begin(), first.end(), idx[k]) - first.begin()) - 1;
        local[r].push_back(idx[k] - first[r]);
        slot[r].push_back(k);
    }
    std::vector<std::vector<int32_t>> ids(m->n);
    std::vector<std::vector<int64_t>> offs(m->n);
    std::vector<int64_t> len(n);
    for (int r = 0; r < m->n; ++r) {
        if (local[r].empty()) continue;
        const int64_t q = (int64_t)local[r].size();
        std::vector<int64_t> lens(first[r + 1] - first[r]);
        MTRY(bpe_sample_lengths(m->sh[r], lens.data(), (int64_t)lens.size()));
        int64_t need = 0;
        for (int64_t i : local[r]) need += lens[i];
        ids[r].resize(need);
        offs[r].resize(q + 1);
        MTRY(bpe_read_samples(m->sh[r], local[r].data(), q, ids[r].data(), need, offs[r].data()));
        for (int64_t j = 0; j < q; ++j) len[slot[r][j]] = offs[r][j + 1] - offs[r][j];
    }
    off[0] = 0;
    for (int64_t k = 0; k < n; ++k) off[k + 1] = off[k] + len[k];
    if (ids_cap < off[n] || (off[n] && !ids_out))
        return bpe_fail(BPE_ERR_ARG, "bpe native: read_samples buffer too small");
    for (int r = 0; r < m->n; ++r)
        for (size_t j = 0; j < slot[r].size(); ++j) {
            const int64_t k = slot[r][j];
            std::copy(ids[r].begin() + offs[r][j], ids[r].begin() + offs[r][j + 1], ids_out + off[k]);
        }
    return BPE_OK;
}

// ---- the hot path -----------------------------------------------------------------------------------
// findNextMerge over the shards (core.ts:247-326): the host protocol (sharded.py
// exchange_and_select, in C++).
int find_next_merge_host(bpe_multi *m, int64_t max_length, int64_t min_weight, int32_t *a,
                         int32_t *b, int64_t *w, bool *heavy_out);

int multi_find_next_merge(bpe_multi *m, int64_t max_length, int64_t min_weight, int32_t *a,
                          int32_t *b, int64_t *w) {
    bool heavy = false;
    return find_next_merge_host(m, max_length, min_weight, a, b, w, &heavy);
}

// The host protocol of one iteration; *heavy_out: some sketch bucket needed exact cold counts.
int find_next_merge_host(bpe_multi *m, int64_t max_length, int64_t min_weight, int32_t *a,
                         int32_t *b, int64_t *w, bool *heavy_out) {
    MTRY(distribute(m));
    m->maintained = false;   // (the shards recount their own tables below)
    for (int r = 0; r < m->n; ++r) MTRY(bpe_export_counts(m->sh[r], (uint64_t *)m->d_table[r]));
    MTRY(all_reduce(m, m->d_table, BPE_TABLE_BINS, false));
    // exact counts of the cold pairs whose global sketch bucket could still win (every shard
    // decides alike whether any bucket qualifies)
    std::map<uint32_t, uint64_t> cold;
    bool heavy = false;
    for (int r = 0; r < m->n; ++r) {
        int64_t nc = 0;
        int rc = bpe_heavy_counts(m->sh[r], (uint64_t *)m->d_table[r], max_length, m->d_keys[r],
                                  (uint64_t *)m->d_counts[r], m->cold_cap, &nc);
        if (rc < 0 && nc > m->cold_cap) {
            MTRY(ensure_cold_bufs(m, nc));
            rc = bpe_heavy_counts(m->sh[r], (uint64_t *)m->d_table[r], max_length, m->d_keys[r],
                                  (uint64_t *)m->d_counts[r], m->cold_cap, &nc);
        }
        if (rc < 0) return rc;
        if (nc < 0) continue;
        heavy = true;
        *heavy_out = true;
        if (nc == 0) continue;
        std::vector<uint32_t> k(nc);
        std::vector<uint64_t> v(nc);
        MHIP(hipSetDevice(m->dev[r]));
        MHIP(hipMemcpy(k.data(), m->d_keys[r], nc * 4, hipMemcpyDeviceToHost));
        MHIP(hipMemcpy(v.data(), m->d_counts[r], nc * 8, hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < nc; ++i)
            if (v[i]) cold[k[i]] += v[i];   // (holes: count 0)
    }
    int64_t n_cold = 0;
    if (heavy && !cold.empty()) {
        MTRY(ensure_cold_bufs(m, (int64_t)cold.size()));
        std::vector<uint32_t> k;
        std::vector<uint64_t> v;
        for (auto &kv : cold) {
            k.push_back(kv.first);
            v.push_back(kv.second);
        }
        n_cold = (int64_t)k.size();
        MHIP(hipSetDevice(m->dev[0]));
        MHIP(hipMemcpy(m->d_keys[0], k.data(), n_cold * 4, hipMemcpyHostToDevice));
        MHIP(hipMemcpy(m->d_counts[0], v.data(), n_cold * 8, hipMemcpyHostToDevice));
    }
    constexpr int64_t CAP = 4096;
    std::vector<int32_t> cand(2 * CAP);
    int64_t n_cand = 0, W = 0;
    int rc = bpe_select_counts(m->sh[0], (uint64_t *)m->d_table[0], m->d_keys[0],
                               (uint64_t *)m->d_counts[0], n_cold, max_length, min_weight,
                               cand.data(), CAP, &n_cand, &W);
    if (rc) return rc;   // BPE_NO_MERGE or an error
    if (n_cand > CAP) return bpe_fail(BPE_ERR_STATE, "bpe native: more than 4096 tied pairs");
    int64_t best = 0;
    if (n_cand > 1) {
        // R3: the candidate whose last counted occurrence is earliest in corpus order
        std::vector<uint64_t> glob(n_cand, 0), last(n_cand);
        for (int r = 0; r < m->n; ++r) {
            MTRY(bpe_tie_positions(m->sh[r], cand.data(), n_cand, last.data()));
            for (int64_t j = 0; j < n_cand; ++j)
                if (last[j]) glob[j] = std::max<uint64_t>(glob[j], ((uint64_t)r << RANK_SHIFT) | last[j]);
        }
        uint64_t bp = ~0ull;
        best = -1;
        for (int64_t j = 0; j < n_cand; ++j)
            if (glob[j] && glob[j] < bp) {
                bp = glob[j];
                best = j;
            }
        if (best < 0) return bpe_fail(BPE_ERR_STATE, "bpe native: tie pass found no occurrence");
    }
    *a = cand[2 * best];
    *b = cand[2 * best + 1];
    *w = W;
    return BPE_OK;
}

int multi_apply_merge(bpe_multi *m, int32_t a, int32_t b, int32_t c, int64_t *replaced) {
    MTRY(distribute(m));
    m->maintained = false;
    int64_t tot = 0;
    for (auto s : m->sh) {
        int64_t r = 0;
        MTRY(bpe_apply_merge(s, a, b, c, &r));
        tot += r;
    }
    if (replaced) *replaced = tot;
    return BPE_OK;
}

int multi_apply_merges(bpe_multi *m, const int32_t *abc, int64_t n, int64_t *replaced,
                       int count_after) {
    MTRY(distribute(m));
    m->maintained = false;
    std::vector<int64_t> rep(std::max<int64_t>(n, 1));
    if (replaced) std::fill(replaced, replaced + n, 0);
    for (auto s : m->sh) {
        MTRY(bpe_apply_merges(s, abc, n, rep.data(), count_after));
        if (replaced)
            for (int64_t i = 0; i < n; ++i) replaced[i] += rep[i];
    }
    return BPE_OK;
}

int debug_compare_global(bpe_multi *m, int64_t merges_so_far);

// The maintained state over the shards: the global table (all-reduced) and every shard's exact
// cold-pair list, gathered through the host, loaded into every shard (bpe_set_global_counts).
int enter_maintained(bpe_multi *m) {
    for (int r = 0; r < m->n; ++r) MTRY(bpe_export_counts(m->sh[r], (uint64_t *)m->d_table[r]));
    MTRY(all_reduce(m, m->d_table, BPE_TABLE_BINS, false));
    std::vector<int64_t> cnt(m->n, 0);
    int64_t total = 0;
    for (int r = 0; r < m->n; ++r) {
        MTRY(bpe_cold_counts(m->sh[r], nullptr, nullptr, 0, &cnt[r]));   // (the pass; kept)
        total += cnt[r];
    }
    MTRY(ensure_cold_bufs(m, std::max<int64_t>(total, 1)));
    std::vector<uint32_t> keys(total);
    std::vector<uint64_t> vals(total);
    int64_t o = 0;
    for (int r = 0; r < m->n; ++r) {
        int64_t nr = 0;
        MTRY(bpe_cold_counts(m->sh[r], m->d_keys[r], (uint64_t *)m->d_counts[r], m->cold_cap, &nr));
        if (nr != cnt[r]) return bpe_fail(BPE_ERR_STATE, "bpe native: cold list changed size");
        if (nr) {
            MHIP(hipSetDevice(m->dev[r]));
            MHIP(hipMemcpy(keys.data() + o, m->d_keys[r], nr * 4, hipMemcpyDeviceToHost));
            MHIP(hipMemcpy(vals.data() + o, m->d_counts[r], nr * 8, hipMemcpyDeviceToHost));
        }
        o += nr;
    }
    for (int r = 0; r < m->n; ++r) {
        if (total) {
            MHIP(hipSetDevice(m->dev[r]));
            MHIP(hipMemcpy(m->d_keys[r], keys.data(), total * 4, hipMemcpyHostToDevice));
            MHIP(hipMemcpy(m->d_counts[r], vals.data(), total * 8, hipMemcpyHostToDevice));
        }
        MTRY(bpe_set_global_counts(m->sh[r], (const uint64_t *)m->d_table[r], m->d_keys[r],
                                   (const uint64_t *)m->d_counts[r], total));
    }
    m->maintained = true;
    m->heavy_streak = 0;
    static const bool dbg = getenv("BPE_DEBUG_GLOBAL") != nullptr;
    if (dbg && !m->pix) MTRY(debug_compare_global(m, -1));
    return BPE_OK;
}

extern "C" int bpe_debug_tables(bpe_ctx *c, uint64_t *hot, uint32_t *keys, uint64_t *counts,
                                int64_t cap, int64_t *n);

// (debug: BPE_DEBUG_GLOBAL=1) every shard's copy of the global tables must be the same: the hot
// bins, and the cold pairs with a count (holes and dead claims aside)
int debug_compare_global(bpe_multi *m, int64_t merges_so_far) {
    std::vector<uint64_t> hot0(BPE_HOT_BINS), hot(BPE_HOT_BINS);
    std::map<uint32_t, uint64_t> cold0;
    for (int r = 0; r < m->n; ++r) {
        int64_t nu = 0;
        MTRY(bpe_debug_tables(m->sh[r], hot.data(), nullptr, nullptr, 0, &nu));
        std::vector<uint32_t> k(nu);
        std::vector<uint64_t> v(nu);
        MTRY(bpe_debug_tables(m->sh[r], hot.data(), k.data(), v.data(), nu, &nu));
        std::map<uint32_t, uint64_t> cold;
        for (int64_t i = 0; i < nu; ++i)
            if (v[i] && k[i] != 0xFFFFFFFFu) cold[k[i]] += v[i];
        if (r == 0) {
            hot0 = hot;
            cold0 = cold;
            continue;
        }
        for (int b = 0; b < BPE_HOT_BINS; ++b)
            if (hot[b] != hot0[b]) {
                fprintf(stderr, "[bpe debug] after %lld merges: shard %d hot bin (%d, %d) = %llu, shard 0: %llu\n",
                        (long long)merges_so_far, r, b & 255, b >> 8, (unsigned long long)hot[b],
                        (unsigned long long)hot0[b]);
                return bpe_fail(BPE_ERR_STATE, "bpe debug: global hot tables differ");
            }
        if (cold != cold0) {
            for (auto &kv : cold0)
                if (cold[kv.first] != kv.second) {
                    fprintf(stderr, "[bpe debug] after %lld merges: shard %d cold (%u, %u) = %llu, shard 0: %llu\n",
                            (long long)merges_so_far, r, kv.first >> 16, kv.first & 0xFFFF,
                            (unsigned long long)cold[kv.first], (unsigned long long)kv.second);
                    break;
                }
            return bpe_fail(BPE_ERR_STATE, "bpe debug: global cold tables differ");
        }
    }
    // no count may exceed the corpus (a count of 2^32 and more here is garbage)
    for (int b = 0; b < BPE_HOT_BINS; ++b)
        if (hot0[b] >> 32) {
            fprintf(stderr, "[bpe debug] after %lld merges: hot bin (%d, %d) = %llu\n", (long long)merges_so_far,
                    b & 255, b >> 8, (unsigned long long)hot0[b]);
            return bpe_fail(BPE_ERR_STATE, "bpe debug: garbage hot count");
        }
    for (auto &kv : cold0)
        if (kv.second >> 32) {
            fprintf(stderr, "[bpe debug] after %lld merges: cold (%u, %u) = %llu\n", (long long)merges_so_far,
                    kv.first >> 16, kv.first & 0xFFFF, (unsigned long long)kv.second);
            return bpe_fail(BPE_ERR_STATE, "bpe debug: garbage cold count");
        }
    fprintf(stderr, "[bpe debug] after %lld merges: %d shards agree (%zu cold pairs)\n",
            (long long)merges_so_far, m->n, cold0.size());
    return BPE_OK;
}

// mergeUntil (core.ts:365-383) over the shards: batches of the device-resident rank loop, the
// host protocol for the iterations it hands back.  Two host iterations in a row that needed exact
// cold counts (the cold pairs outgrow the sketch: skewed corpora, large vocabularies) move the
// shards to the maintained state, where the batches keep the global tables with delta rows.
int multi_merge_until(bpe_multi *m, int64_t max_length, int64_t min_weight,
                      int64_t max_iterations, int64_t *out_abw, int64_t cap, int64_t *n_merges) {
    MTRY(distribute(m));
    int64_t n = 0, batch = BPE_LOOP_BATCH;
    std::vector<std::vector<int64_t>> log(m->n, std::vector<int64_t>(4 * BPE_LOOP_BATCH));
    auto put = [&](int32_t a, int32_t b, int64_t w) {
        if (n < cap) {
            out_abw[3 * n] = a;
            out_abw[3 * n + 1] = b;
            out_abw[3 * n + 2] = w;
        }
        ++n;
    };
    while (!max_iterations || n < max_iterations) {
        int32_t nt = 0;
        MTRY(check_vocab(m, &nt));
        // Past AUTO_PIX_VOCAB token ids the streaming mode's maintained state outgrows its design:
        // the merge pass's LDS rows index the other token of a pair below 18432 (INCR_RLIM), and
        // every merge scans all the claimed cold pairs (their invalidation; the selection's block
        // maxima fall back to full scans past 2^16 blocks), whose number grows with the vocabulary
        // (8 shards of 512 MiB: 1.0 ms/merge at 4k merges, 5.1 ms/merge at 32k; profiles/
        // r05_kernel_stats_multi8_32k_stream.csv).  So the shards go on in the incremental mode,
        // whose merges and counts are the same.  A mode the caller set
        // (bpe_set_mode) is kept; BPE_STREAM_ONLY=1 keeps the stream for every context.
        static const bool stream_only = getenv("BPE_STREAM_ONLY") != nullptr;
        // (BPE_AUTO_PIX_VOCAB=n, tests: switch at n token ids; read per batch)
        const char *av = getenv("BPE_AUTO_PIX_VOCAB");
        const int32_t auto_vocab = av ? (int32_t)atoi(av) : AUTO_PIX_VOCAB;
        if (!m->pix && !m->mode_explicit && !stream_only && nt >= auto_vocab) {
            MTRY(multi_set_mode(m, BPE_MODE_INCREMENTAL, false));
            m->pix_auto = true;
        }
        int64_t want = std::min<int64_t>(batch, BPE_MAX_VOCAB - (int64_t)nt);
        if (max_iterations) want = std::min<int64_t>(want, max_iterations - n);
        int status = 2;
        bool batch_maintained = false;
        if (want > 0) {
            // (the incremental mode enters its global state, the shards' position indexes, at
            // once; the streaming mode when the cold pairs outgrow the sketch)
            const bool pix = m->pix && !m->pix_off;
            if (!m->maintained && (m->heavy_streak >= 2 || pix)) {
                // (more than 64 entries since the mode was set, at least one per 16 merges made:
                // the index keeps handing over here, and the stream goes on)
                if (pix && ++m->pix_entries > 64 && m->pix_entries > (m->pix_merged + n) / 16) {
                    m->pix_off = true;
                    ++m->pix_fallbacks;
                    for (auto s : m->sh) MTRY(bpe_set_mode(s, BPE_MODE_STREAM));
                }
                int erc = enter_maintained(m);
                if (erc == BPE_ERR_NOFIT && pix && m->pix_auto) {
                    // (the automatic switch: the shards' indexes do not fit beside their corpora,
                    // e.g. 2 GiB shards sharing one device; the stream goes on.  Only on that code:
                    // any other error, a HIP fault or a table overflow, is the caller's)
                    m->pix_off = true;
                    ++m->pix_fallbacks;
                    for (auto s : m->sh) MTRY(bpe_set_mode(s, BPE_MODE_STREAM));
                    for (auto s : m->sh) MTRY(bpe_leave_global(s));
                    erc = enter_maintained(m);
                }
                MTRY(erc);
            }
            batch_maintained = m->maintained;
            int64_t nw = -1;
            for (int r = 0; r < m->n; ++r) {
                int64_t w_r = 0;
                MTRY(bpe_rank_loop_begin(m->sh[r], max_length, min_weight, (uint64_t *)m->d_xchg[r],
                                         (uint64_t *)m->d_tie[r], r, m->n, &w_r));
                if (nw >= 0 && w_r != nw) return bpe_fail(BPE_ERR_STATE, "bpe native: shards disagree on the exchange");
                nw = w_r;
            }
            MTRY(enqueue_batch(m, want, (size_t)nw));
            int64_t nd = -1;
            for (int r = 0; r < m->n; ++r) {
                int64_t k = 0;
                int st = 0;
                MTRY(bpe_rank_loop_end(m->sh[r], log[r].data(), BPE_LOOP_BATCH, &k, &st));
                bool same = nd < 0 || (k == nd && st == status);
                for (int64_t i = 0; same && r > 0 && i < k; ++i)
                    same = std::equal(log[r].begin() + 4 * i, log[r].begin() + 4 * i + 3,
                                      log[0].begin() + 4 * i);
                if (!same) return bpe_fail(BPE_ERR_STATE, "bpe native: shards disagree on the merges");
                nd = k;
                status = st;
            }
            for (int64_t i = 0; i < nd; ++i) {
                // every merge: the shards' replacement counts sum to W (core.ts:356-359)
                int64_t tot = 0;
                for (int r = 0; r < m->n; ++r) tot += log[r][4 * i + 3];
                if (tot != log[0][4 * i + 2]) return bpe_fail(BPE_ERR_STATE, "bpe native: replacement count != W");
                put((int32_t)log[0][4 * i], (int32_t)log[0][4 * i + 1], log[0][4 * i + 2]);
            }
            static const bool dbg = getenv("BPE_DEBUG_GLOBAL") != nullptr;
            if (dbg && batch_maintained && status == 0 && !m->pix) MTRY(debug_compare_global(m, n));
            if (status != 0) m->maintained = false;   // (the shards left the global state)
            if (status == 1) break;                                        // no pair qualifies
            if (status == 0) {
                batch = std::min<int64_t>(BPE_LOOP_BATCH, 2 * batch);
                static const int dbg_batch = getenv("BPE_DEBUG_BATCH") ? atoi(getenv("BPE_DEBUG_BATCH")) : 0;
                if (dbg_batch > 0 && m->maintained) batch = std::min<int64_t>(batch, dbg_batch);
                continue;
            }
            batch = std::max<int64_t>(1, std::min<int64_t>(BPE_LOOP_BATCH, 2 * nd));
            if (max_iterations && n >= max_iterations) break;
        }
        // the host protocol for this iteration (or the vocabulary limit, reported by the apply).
        // After a maintained batch hands over, one more iteration with exact counts re-enters it.
        const bool was_maintained = batch_maintained && status == 2;
        int32_t a, b;
        int64_t w;
        bool heavy = false;
        int rc = find_next_merge_host(m, max_length, min_weight, &a, &b, &w, &heavy);
        if (rc == BPE_NO_MERGE) break;
        if (rc) return rc;
        m->heavy_streak = heavy ? std::max(m->heavy_streak + 1, was_maintained ? 2 : 1) : 0;
        MTRY(check_vocab(m, &nt));
        int64_t rep = 0;
        MTRY(multi_apply_merge(m, a, b, nt, &rep));
        if (rep != w) return bpe_fail(BPE_ERR_STATE, "bpe native: replacement count != W");
        put(a, b, w);
    }
    if (m->pix) m->pix_merged += n;
    *n_merges = n;
    return BPE_OK;
}

// ---- measurement -------------------------------------------------------------------------------------
int multi_stats_enable(bpe_multi *m, int on) {
    for (auto s : m->sh) MTRY(bpe_stats_enable(s, on));
    return BPE_OK;
}

int multi_get_stats(bpe_multi *m, bpe_stats *out) {
    // counters summed over the shards; times: the slowest shard's
    bpe_stats acc;
    std::memset(&acc, 0, sizeof acc);
    for (auto s : m->sh) {
        bpe_stats x;
        MTRY(bpe_get_stats(s, &x));
        acc.step_ms = std::max(acc.step_ms, x.step_ms);
        acc.select_ms = std::max(acc.select_ms, x.select_ms);
        acc.step_launches += x.step_launches;
        acc.step_slots += x.step_slots;
        acc.step_live += x.step_live;
        acc.tie_passes += x.tie_passes;
        acc.iterations = std::max(acc.iterations, x.iterations);
        acc.live_tokens += x.live_tokens;
        acc.compactions += x.compactions;
        acc.exact_passes += x.exact_passes;
        acc.step_timed = std::max(acc.step_timed, x.step_timed);
        acc.tie_tail += x.tie_tail;
        acc.tie_lone += x.tie_lone;
        acc.loop_host = std::max(acc.loop_host, x.loop_host);
        acc.fused_passes += x.fused_passes;
        acc.pix_builds += x.pix_builds;
        acc.pix_merges += x.pix_merges;
        acc.pix_host = std::max(acc.pix_host, x.pix_host);
        acc.pix_build_ms = std::max(acc.pix_build_ms, x.pix_build_ms);
        acc.xchg_bytes += x.xchg_bytes;
        acc.cold_rebuilds += x.cold_rebuilds;
        acc.incr_ms = std::max(acc.incr_ms, x.incr_ms);
        acc.incr_timed = std::max(acc.incr_timed, x.incr_timed);
        acc.incr_launches += x.incr_launches;
        acc.incr_live += x.incr_live;
        acc.unscreened_passes += x.unscreened_passes;
        acc.xchg_iters = std::max(acc.xchg_iters, x.xchg_iters);
    }
    acc.pix_fallbacks = m->pix_fallbacks;
    *out = acc;
    return BPE_OK;
}

int multi_reset_stats(bpe_multi *m) {
    for (auto s : m->sh) MTRY(bpe_reset_stats(s));
    return BPE_OK;
}

int multi_get_stream(bpe_multi *m, void **stream) { return bpe_get_stream(m->sh[0], stream); }

// ---- one rank of a sharded corpus per process: the rank loop's collectives from C++ ---------------
// (include/bpe.h bpe_rank_rccl_*): one RCCL communicator per context, its all-reduces issued on the
// context's own stream between the rank loop's kernels, so a batch of iterations is enqueued by
// one call with no host round trip and no cross-stream event per collective.
namespace {
// (one RCCL library for every rank communicator and for ncclGetUniqueId: loaded once, kept for
// the process's lifetime, so no communicator outlives the library it came from)
Rccl &id_rccl() {
    static Rccl r;
    return r;
}
struct RankComm {
    const Rccl *rccl = nullptr;
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1;
};
std::map<bpe_ctx *, RankComm> &rank_comms() {
    static std::map<bpe_ctx *, RankComm> m;
    return m;
}
}  // namespace

// (internal, bpe_engine.hip bpe_destroy) a context going away frees its communicator
void rank_rccl_forget(bpe_ctx *ctx) {
    auto &m = rank_comms();
    auto it = m.find(ctx);
    if (it == m.end()) return;
    if (it->second.comm && it->second.rccl && it->second.rccl->destroy)
        it->second.rccl->destroy(it->second.comm);
    m.erase(it);
}

extern "C" {

int bpe_rccl_unique_id(void *id, size_t cap) {
    if (!id || cap < sizeof(ncclUniqueId)) return bpe_fail(BPE_ERR_ARG, "bpe native: unique id buffer too small");
    Rccl &r = id_rccl();
    if (!r.so) MTRY(load_rccl(r));
    if (!r.get_unique_id) return bpe_fail(BPE_ERR_HIP, "bpe native: RCCL symbols missing");
    ncclUniqueId u;
    const ncclResult_t e = r.get_unique_id(&u);
    if (e != ncclSuccess)
        return bpe_fail(BPE_ERR_HIP, (std::string("bpe native: ncclGetUniqueId: ") +
                                      (r.error_string ? r.error_string(e) : "RCCL error")).c_str());
    std::memcpy(id, &u, sizeof u);
    return BPE_OK;
}

int bpe_rank_rccl_init(bpe_ctx *ctx, const void *id, int rank, int world) {
    if (!ctx || !id || world < 1 || rank < 0 || rank >= world)
        return bpe_fail(BPE_ERR_ARG, "bpe native: bad rank communicator arguments");
    int n_shards = 0;
    MTRY(bpe_shard_count(ctx, &n_shards));
    if (n_shards != 1) return bpe_fail(BPE_ERR_STATE, "bpe native: a rank communicator needs a single-device context");
    rank_rccl_forget(ctx);
    Rccl &lib = id_rccl();
    if (!lib.so) MTRY(load_rccl(lib));
    RankComm rc;
    rc.rccl = &lib;
    if (!lib.init_rank) return bpe_fail(BPE_ERR_HIP, "bpe native: RCCL symbols missing");
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    // (the communicator belongs to the context's device, whatever device the caller has current)
    void *s = nullptr;
    MTRY(bpe_get_stream(ctx, &s));
    hipDevice_t dev = 0;
    MHIP(hipStreamGetDevice((hipStream_t)s, &dev));
    MHIP(hipSetDevice(dev));
    const ncclResult_t e = lib.init_rank(&rc.comm, world, u, rank);
    if (e != ncclSuccess)
        return bpe_fail(BPE_ERR_HIP, (std::string("bpe native: ncclCommInitRank: ") +
                                      (lib.error_string ? lib.error_string(e) : "RCCL error")).c_str());
    rc.rank = rank;
    rc.world = world;
    rank_comms()[ctx] = rc;
    return BPE_OK;
}

int bpe_rank_loop_rccl(bpe_ctx *ctx, uint64_t *xchg, int64_t xchg_words, uint64_t *tie, int iterations) {
    auto it = rank_comms().find(ctx);
    if (it == rank_comms().end())
        return bpe_fail(BPE_ERR_STATE, "bpe native: no rank communicator (bpe_rank_rccl_init)");
    if (!xchg || !tie || xchg_words < 1 || iterations < 0)
        return bpe_fail(BPE_ERR_ARG, "bpe native: bad rank loop arguments");
    // the all-reduces must cover exactly the buffers the batch's kernels use (bpe_rank_loop_begin)
    unsigned long long *bx = nullptr, *bt = nullptr;
    int64_t bw = 0;
    MTRY(rank_loop_buffers(ctx, &bx, &bt, &bw));
    if ((void *)bx != (void *)xchg || (void *)bt != (void *)tie || xchg_words != bw)
        return bpe_fail(BPE_ERR_ARG, "bpe native: the exchange / tie buffers or the word count differ "
                                     "from the batch's (bpe_rank_loop_begin)");
    RankComm &rc = it->second;
    void *sp = nullptr;
    MTRY(bpe_get_stream(ctx, &sp));
    hipStream_t st = (hipStream_t)sp;
    auto ar = [&](uint64_t *buf, size_t count, ncclRedOp_t op, const char *what) -> int {
        const ncclResult_t e = rc.rccl->all_reduce(buf, buf, count, ncclUint64, op, rc.comm, st);
        if (e == ncclSuccess) return BPE_OK;
        return bpe_fail(BPE_ERR_HIP, (std::string("bpe native: ") + what + ": " +
                                      (rc.rccl->error_string ? rc.rccl->error_string(e) : "RCCL error")).c_str());
    };
    for (int i = 0; i < iterations; ++i) {
        MTRY(ar(xchg, (size_t)xchg_words, ncclSum, "ncclAllReduce(exchange)"));
        MTRY(bpe_rank_loop_select(ctx));
        MTRY(ar(tie, BPE_TIE_WORDS, ncclMax, "ncclAllReduce(tie)"));
        MTRY(bpe_rank_loop_decide(ctx));
        MTRY(bpe_rank_loop_count(ctx));
    }
    return BPE_OK;
}

int bpe_rank_rccl_destroy(bpe_ctx *ctx) {
    rank_rccl_forget(ctx);
    return BPE_OK;
}

}  // extern "C"
