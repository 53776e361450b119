// bpe_napi.cc — Node N-API addon: the thin binding core.js uses to reach the C ABI of libbpe
// (include/bpe.h).  Every function maps 1:1 onto a bpe_* entry point; errors become JS
// `Error('bpe native: ...')` carrying bpe_last_error().
#define NAPI_VERSION 6
#include <node_api.h>

#include <cstdint>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "bpe.h"

namespace {

napi_value throw_native(napi_env env, const char *what) {
    char buf[1024];
    bpe_last_error(buf, sizeof buf);
    std::string msg = buf[0] ? std::string(buf) : std::string("bpe native: ") + what + " failed";
    napi_throw_error(env, nullptr, msg.c_str());
    return nullptr;
}

napi_value throw_arg(napi_env env, const char *msg) {
    napi_throw_type_error(env, nullptr, msg);
    return nullptr;
}

bool get_args(napi_env env, napi_callback_info info, size_t want, napi_value *argv) {
    size_t argc = want;
    if (napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr) != napi_ok) return false;
    return argc >= want;
}

// An engine handle: the context behind a JS external.  destroyEngine() frees the context (its
// device memory) at once; the holder itself goes with the external's finalizer.
struct Holder {
    bpe_ctx *c = nullptr;
};

void finalize_ctx(napi_env, void *data, void *) {
    Holder *h = static_cast<Holder *>(data);
    if (!h) return;
    if (h->c) bpe_destroy(h->c);
    delete h;
}

bpe_ctx *get_ctx(napi_env env, napi_value v) {
    void *p = nullptr;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) return nullptr;
    return static_cast<Holder *>(p)->c;   // (null after destroyEngine: every call then fails)
}

int64_t get_i64(napi_env env, napi_value v) {
    int64_t x = 0;
    napi_get_value_int64(env, v, &x);
    return x;
}

napi_value num(napi_env env, double x) {
    napi_value v;
    napi_create_double(env, x, &v);
    return v;
}

// createEngine(device[, Int32Array devices, reduce]) -> external handle (bpe_create, core.ts:77
// `new BPETokenizer()`); with a device list, one corpus sharded over those devices
// (bpe_create_multi, reduce = BPE_REDUCE_RCCL 0 / BPE_REDUCE_HOST 1)
napi_value CreateEngine(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    int device = 0;
    size_t argc = 3;
    napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
    if (argc >= 1) device = (int)get_i64(env, argv[0]);
    bpe_ctx *ctx = nullptr;
    napi_valuetype t = napi_undefined;
    if (argc >= 2) napi_typeof(env, argv[1], &t);
    if (argc >= 2 && t == napi_object) {
        napi_typedarray_type type;
        size_t n = 0, off = 0;
        void *data = nullptr;
        napi_value ab;
        if (napi_get_typedarray_info(env, argv[1], &type, &n, &data, &ab, &off) != napi_ok ||
            type != napi_int32_array || n == 0)
            return throw_arg(env, "createEngine expects an Int32Array of device indices");
        const int reduce = argc >= 3 ? (int)get_i64(env, argv[2]) : BPE_REDUCE_RCCL;
        if (bpe_create_multi(&ctx, (int)n, static_cast<const int *>(data), reduce) != BPE_OK)
            return throw_native(env, "bpe_create_multi");
    } else if (bpe_create(&ctx, device) != BPE_OK) {
        return throw_native(env, "bpe_create");
    }
    napi_value ext;
    Holder *h = new Holder();
    h->c = ctx;
    napi_create_external(env, h, finalize_ctx, nullptr, &ext);
    return ext;
}

// destroyEngine(h): frees the context and its device memory now, not at garbage collection
napi_value DestroyEngine(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return throw_arg(env, "destroyEngine(h)");
    void *p = nullptr;
    if (napi_get_value_external(env, argv[0], &p) != napi_ok || !p)
        return throw_arg(env, "destroyEngine expects an engine handle");
    Holder *h = static_cast<Holder *>(p);
    if (h->c) bpe_destroy(h->c);
    h->c = nullptr;
    return nullptr;
}

// deviceCount() -> number of HIP devices
napi_value DeviceCount(napi_env env, napi_callback_info) {
    int n = 0;
    bpe_device_count(&n);
    return num(env, n);
}

// setTokenLen16(h, id, len16)
napi_value SetTokenLen16(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return throw_arg(env, "setTokenLen16(h, id, len16)");
    bpe_ctx *ctx = get_ctx(env, argv[0]);
    if (bpe_set_token_len16(ctx, (int32_t)get_i64(env, argv[1]), (int32_t)get_i64(env, argv[2])) < 0)
        return throw_native(env, "bpe_set_token_len16");
    return nullptr;
}

// addSample(h, Int32Array ids)  (addToCorpus / restoreToCorpus)
napi_value AddSample(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return throw_arg(env, "addSample(h, Int32Array)");
    bpe_ctx *ctx = get_ctx(env, argv[0]);
    napi_typedarray_type type;
    size_t length = 0, offset = 0;
    void *data = nullptr;
    napi_value ab;
    if (napi_get_typedarray_info(env, argv[1], &type, &length, &data, &ab, &offset) != napi_ok ||
        type != napi_int32_array)
        return throw_arg(env, "addSample expects an Int32Array");
    if (bpe_add_sample(ctx, static_cast<const int32_t *>(data), (int64_t)length) < 0)
        return throw_native(env, "bpe_add_sample");
    return nullptr;
}

// addLatin1(h, Buffer bytes, sampleBytes, Int32Array charToId[256], nTokens) -> [nTokens, hist]
napi_value AddLatin1(napi_env env, napi_callback_info info) {
    napi_value argv[5];
    if (!get_args(env, info, 5, argv)) return throw_arg(env, "addLatin1(h, buf, sampleBytes, map, n)");
    bpe_ctx *ctx = get_ctx(env, argv[0]);
    void *bytes = nullptr;
    size_t n = 0;
    if (napi_get_buffer_info(env, argv[1], &bytes, &n) != napi_ok)
        return throw_arg(env, "addLatin1 expects a Buffer");
    napi_typedarray_type type;
    size_t mlen = 0, off = 0;
    void *map = nullptr;
    napi_value ab;
    if (napi_get_typedarray_info(env, argv[3], &type, &mlen, &map, &ab, &off) != napi_ok ||
        type != napi_int32_array || mlen != 256)
        return throw_arg(env, "addLatin1 expects an Int32Array(256) char map");
    int32_t nt = (int32_t)get_i64(env, argv[4]);
    int64_t hist[256];
    if (bpe_add_latin1(ctx, static_cast<const uint8_t *>(bytes), (int64_t)n, get_i64(env, argv[2]),
                       static_cast<int32_t *>(map), &nt, hist) < 0)
        return throw_native(env, "bpe_add_latin1");
    napi_value out, h;
    napi_create_array_with_length(env, 2, &out);
    napi_set_element(env, out, 0, num(env, nt));
    napi_create_array_with_length(env, 256, &h);
    for (int i = 0; i < 256; ++i) napi_set_element(env, h, i, num(env, (double)hist[i]));
    napi_set_element(env, out, 1, h);
    return out;
}

// clearCorpus(h)   (corpus_in_code = [])
napi_value ClearCorpus(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return throw_arg(env, "clearCorpus(h)");
    if (bpe_clear_corpus(get_ctx(env, argv[0])) < 0) return throw_native(env, "bpe_clear_corpus");
    return nullptr;
}

// corpusSize(h) -> [samples, tokens]
napi_value CorpusSize(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return throw_arg(env, "corpusSize(h)");
    int64_t s = 0, t = 0;
    if (bpe_corpus_size(get_ctx(env, argv[0]), &s, &t) < 0) return throw_native(env, "bpe_corpus_size");
    napi_value out;
    napi_create_array_with_length(env, 2, &out);
    napi_set_element(env, out, 0, num(env, (double)s));
    napi_set_element(env, out, 1, num(env, (double)t));
    return out;
}

// readCorpus(h) -> [Int32Array ids, Float64Array offsets]   (materialises corpus_in_code)
napi_value ReadCorpus(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return throw_arg(env, "readCorpus(h)");
    bpe_ctx *ctx = get_ctx(env, argv[0]);
    int64_t ns = 0, nt = 0;
    if (bpe_corpus_size(ctx, &ns, &nt) < 0) return throw_native(env, "bpe_corpus_size");
    void *ids_data = nullptr, *off_data = nullptr;
    napi_value ids_ab, off_ab, ids, offs;
    napi_create_arraybuffer(env, (size_t)std::max<int64_t>(nt, 1) * 4, &ids_data, &ids_ab);
    napi_create_arraybuffer(env, (size_t)(ns + 1) * 8, &off_data, &off_ab);
    std::vector<int64_t> off(ns + 1);
    if (bpe_read_corpus(ctx, static_cast<int32_t *>(ids_data), std::max<int64_t>(nt, 1), off.data(),
                        ns + 1) < 0)
        return throw_native(env, "bpe_read_corpus");
    double *od = static_cast<double *>(off_data);
    for (int64_t i = 0; i <= ns; ++i) od[i] = (double)off[i];
    napi_create_typedarray(env, napi_int32_array, (size_t)nt, ids_ab, 0, &ids);
    napi_create_typedarray(env, napi_float64_array, (size_t)(ns + 1), off_ab, 0, &offs);
    napi_value out;
    napi_create_array_with_length(env, 2, &out);
    napi_set_element(env, out, 0, ids);
    napi_set_element(env, out, 1, offs);
    return out;
}

// sampleLengths(h) -> Float64Array: live tokens per sample (bpe_sample_lengths; the db twin's
// changed-row test, db/core.ts:399-413)
napi_value SampleLengths(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return throw_arg(env, "sampleLengths(h)");
    bpe_ctx *ctx = get_ctx(env, argv[0]);
    int64_t ns = 0;
    if (bpe_corpus_size(ctx, &ns, nullptr) < 0) return throw_native(env, "bpe_corpus_size");
    std::vector<int64_t> lens(std::max<int64_t>(ns, 1));
    if (bpe_sample_lengths(ctx, lens.data(), (int64_t)lens.size()) < 0)
        return throw_native(env, "bpe_sample_lengths");
    void *data = nullptr;
    napi_value ab, out;
    napi_create_arraybuffer(env, (size_t)std::max<int64_t>(ns, 1) * 8, &data, &ab);
    double *d = static_cast<double *>(data);
    for (int64_t i = 0; i < ns; ++i) d[i] = (double)lens[i];
    napi_create_typedarray(env, napi_float64_array, (size_t)ns, ab, 0, &out);
    return out;
}

// readSamples(h, Float64Array idx) -> [Int32Array ids, Float64Array offsets] of those samples, in
// that order (bpe_read_samples; the db twin's row write-back, db/core.ts:414-417)
napi_value ReadSamples(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return throw_arg(env, "readSamples(h, Float64Array)");
    bpe_ctx *ctx = get_ctx(env, argv[0]);
    napi_typedarray_type type;
    size_t n = 0, o = 0;
    void *data = nullptr;
    napi_value ab;
    if (napi_get_typedarray_info(env, argv[1], &type, &n, &data, &ab, &o) != napi_ok ||
        type != napi_float64_array)
        return throw_arg(env, "readSamples expects a Float64Array of sample indices");
    std::vector<int64_t> idx(n);
    for (size_t k = 0; k < n; ++k) idx[k] = (int64_t) static_cast<const double *>(data)[k];
    int64_t ns = 0;
    if (bpe_corpus_size(ctx, &ns, nullptr) < 0) return throw_native(env, "bpe_corpus_size");
    std::vector<int64_t> lens(std::max<int64_t>(ns, 1));
    if (bpe_sample_lengths(ctx, lens.data(), (int64_t)lens.size()) < 0)
        return throw_native(env, "bpe_sample_lengths");
    int64_t need = 0;
    for (int64_t i : idx) {
        if (i < 0 || i >= ns) return throw_arg(env, "readSamples: sample index out of range");
        need += lens[i];
    }
    void *ids_data = nullptr, *off_data = nullptr;
    napi_value ids_ab, off_ab, ids, offs;
    napi_create_arraybuffer(env, (size_t)std::max<int64_t>(need, 1) * 4, &ids_data, &ids_ab);
    napi_create_arraybuffer(env, (n + 1) * 8, &off_data, &off_ab);
    std::vector<int64_t> off(n + 1);
    if (bpe_read_samples(ctx, idx.data(), (int64_t)n, static_cast<int32_t *>(ids_data),
                         std::max<int64_t>(need, 1), off.data()) < 0)
        return throw_native(env, "bpe_read_samples");
    double *od = static_cast<double *>(off_data);
    for (size_t k = 0; k <= n; ++k) od[k] = (double)off[k];
    napi_create_typedarray(env, napi_int32_array, (size_t)need, ids_ab, 0, &ids);
    napi_create_typedarray(env, napi_float64_array, n + 1, off_ab, 0, &offs);
    napi_value out;
    napi_create_array_with_length(env, 2, &out);
    napi_set_element(env, out, 0, ids);
    napi_set_element(env, out, 1, offs);
    return out;
}

// findNextMerge(h, maxLength, minWeight) -> [a, b, W] | null   (core.ts:247-326)
napi_value FindNextMerge(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return throw_arg(env, "findNextMerge(h, maxLength, minWeight)");
    int32_t a = 0, b = 0;
    int64_t w = 0;
    int rc = bpe_find_next_merge(get_ctx(env, argv[0]), get_i64(env, argv[1]), get_i64(env, argv[2]),
                                 &a, &b, &w);
    if (rc < 0) return throw_native(env, "bpe_find_next_merge");
    napi_value out;
    if (rc == BPE_NO_MERGE) {
        napi_get_null(env, &out);
        return out;
    }
    napi_create_array_with_length(env, 3, &out);
    napi_set_element(env, out, 0, num(env, a));
    napi_set_element(env, out, 1, num(env, b));
    napi_set_element(env, out, 2, num(env, (double)w));
    return out;
}

// applyMerge(h, a, b, c) -> replaced   (core.ts:356-359)
napi_value ApplyMerge(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (!get_args(env, info, 4, argv)) return throw_arg(env, "applyMerge(h, a, b, c)");
    int64_t rep = 0;
    if (bpe_apply_merge(get_ctx(env, argv[0]), (int32_t)get_i64(env, argv[1]),
                        (int32_t)get_i64(env, argv[2]), (int32_t)get_i64(env, argv[3]), &rep) < 0)
        return throw_native(env, "bpe_apply_merge");
    return num(env, (double)rep);
}

// applyMerges(h, Int32Array abc, countAfter): a run of (a, b, c) rewrites (bpe_apply_merges)
napi_value ApplyMerges(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return throw_arg(env, "applyMerges(h, Int32Array, countAfter)");
    bpe_ctx *ctx = get_ctx(env, argv[0]);
    napi_typedarray_type type;
    size_t length = 0, offset = 0;
    void *data = nullptr;
    napi_value ab;
    if (napi_get_typedarray_info(env, argv[1], &type, &length, &data, &ab, &offset) != napi_ok ||
        type != napi_int32_array || length % 3 != 0)
        return throw_arg(env, "applyMerges expects an Int32Array of (a, b, c) triples");
    if (bpe_apply_merges(ctx, static_cast<const int32_t *>(data), (int64_t)(length / 3), nullptr,
                         (int)get_i64(env, argv[2])) < 0)
        return throw_native(env, "bpe_apply_merges");
    return nullptr;
}

// mergeUntil(h, maxLength, minWeight, maxIterations) -> Float64Array of (a, b, W) triples
// (bpe_merge_until: the device-resident loop, core.ts:365-383; new ids follow bpe_num_tokens)
napi_value MergeUntil(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (!get_args(env, info, 4, argv))
        return throw_arg(env, "mergeUntil(h, maxLength, minWeight, maxIterations)");
    bpe_ctx *ctx = get_ctx(env, argv[0]);
    int32_t nt = 0;
    if (bpe_num_tokens(ctx, &nt) < 0) return throw_native(env, "bpe_num_tokens");
    const int64_t max_it = get_i64(env, argv[3]);
    // every merge adds a token below the vocabulary limit (bpe.h BPE_MAX_VOCAB)
    int64_t cap = BPE_MAX_VOCAB - (int64_t)nt;
    if (max_it > 0 && max_it < cap) cap = max_it;
    if (cap < 1) cap = 1;
    std::vector<int64_t> abw(3 * cap);
    int64_t n = 0;
    if (bpe_merge_until(ctx, get_i64(env, argv[1]), get_i64(env, argv[2]), max_it, abw.data(), cap,
                        &n) < 0)
        return throw_native(env, "bpe_merge_until");
    if (n > cap) n = cap;
    void *data = nullptr;
    napi_value ab, out;
    napi_create_arraybuffer(env, (size_t)std::max<int64_t>(1, 3 * n) * 8, &data, &ab);
    double *d = static_cast<double *>(data);
    for (int64_t i = 0; i < 3 * n; ++i) d[i] = (double)abw[i];
    napi_create_typedarray(env, napi_float64_array, (size_t)(3 * n), ab, 0, &out);
    return out;
}

// An encoder handle (bpe_encoder_*: the merge list as a rank table on the device, encodeToCode
// core.ts:392-409) behind a JS external, freed by its finalizer.  Each tokenizer holds its own, so
// worker_threads environments never share one.
void finalize_encoder(napi_env, void *data, void *) {
    if (data) bpe_encoder_destroy(static_cast<bpe_encoder *>(data));
}

bpe_encoder *get_encoder(napi_env env, napi_value v) {
    void *p = nullptr;
    if (napi_get_value_external(env, v, &p) != napi_ok) return nullptr;
    return static_cast<bpe_encoder *>(p);
}

// createEncoder([device]) -> external handle
napi_value CreateEncoder(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    size_t argc = 1;
    napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
    const int device = argc >= 1 ? (int)get_i64(env, argv[0]) : 0;
    bpe_encoder *enc = nullptr;
    if (bpe_encoder_create(&enc, device) != BPE_OK) return throw_native(env, "bpe_encoder_create");
    napi_value ext;
    napi_create_external(env, enc, finalize_encoder, nullptr, &ext);
    return ext;
}

// encoderAddMerges(enc, Int32Array abc): appends (a, b, c) triples in merge_codes order
napi_value EncoderAddMerges(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return throw_arg(env, "encoderAddMerges(enc, Int32Array)");
    napi_typedarray_type t;
    size_t n = 0, o = 0;
    void *abc = nullptr;
    napi_value ab;
    if (napi_get_typedarray_info(env, argv[1], &t, &n, &abc, &ab, &o) != napi_ok ||
        t != napi_int32_array || n % 3 != 0)
        return throw_arg(env, "encoderAddMerges expects (a, b, c) triples in an Int32Array");
    if (bpe_encoder_add_merges(get_encoder(env, argv[0]), static_cast<const int32_t *>(abc),
                               (int64_t)(n / 3)) < 0)
        return throw_native(env, "bpe_encoder_add_merges");
    return nullptr;
}

// encoderClear(enc)
napi_value EncoderClear(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return throw_arg(env, "encoderClear(enc)");
    if (bpe_encoder_clear(get_encoder(env, argv[0])) < 0) return throw_native(env, "bpe_encoder_clear");
    return nullptr;
}

// encodeBatch(enc, Int32Array ids, Float64Array offsets) -> [Int32Array ids, Float64Array offsets]
// (bpe_encode_batch: text k = ids[offsets[k] .. offsets[k+1]))
napi_value EncodeBatch(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return throw_arg(env, "encodeBatch(enc, Int32Array, Float64Array)");
    napi_typedarray_type t1, t2;
    size_t n1 = 0, n2 = 0, o1 = 0, o2 = 0;
    void *ids = nullptr, *offd = nullptr;
    napi_value ab1, ab2;
    if (napi_get_typedarray_info(env, argv[1], &t1, &n1, &ids, &ab1, &o1) != napi_ok ||
        t1 != napi_int32_array ||
        napi_get_typedarray_info(env, argv[2], &t2, &n2, &offd, &ab2, &o2) != napi_ok ||
        t2 != napi_float64_array || n2 < 1)
        return throw_arg(env, "encodeBatch expects Int32Array ids and Float64Array offsets");
    const int64_t n_texts = (int64_t)n2 - 1;
    std::vector<int64_t> off(n2);
    const double *od = static_cast<const double *>(offd);
    for (size_t k = 0; k < n2; ++k) {
        off[k] = (int64_t)od[k];
        if (off[k] < 0 || (size_t)off[k] > n1) return throw_arg(env, "encodeBatch: offset out of range");
    }
    const int64_t total = off[n_texts] - off[0];
    void *out_data = nullptr, *oo_data = nullptr;
    napi_value out_ab, oo_ab, out, oo, pair;
    napi_create_arraybuffer(env, (size_t)std::max<int64_t>(total, 1) * 4, &out_data, &out_ab);
    std::vector<int64_t> out_off(n2);
    if (bpe_encode_batch(get_encoder(env, argv[0]), static_cast<const int32_t *>(ids), off.data(),
                         n_texts, static_cast<int32_t *>(out_data), out_off.data()) < 0)
        return throw_native(env, "bpe_encode_batch");
    napi_create_typedarray(env, napi_int32_array, (size_t)out_off[n_texts], out_ab, 0, &out);
    napi_create_arraybuffer(env, n2 * 8, &oo_data, &oo_ab);
    double *ood = static_cast<double *>(oo_data);
    for (size_t k = 0; k < n2; ++k) ood[k] = (double)out_off[k];
    napi_create_typedarray(env, napi_float64_array, n2, oo_ab, 0, &oo);
    napi_create_array_with_length(env, 2, &pair);
    napi_set_element(env, pair, 0, out);
    napi_set_element(env, pair, 1, oo);
    return pair;
}

napi_value Init(napi_env env, napi_value exports) {
    struct {
        const char *name;
        napi_callback cb;
    } fns[] = {
        {"createEngine", CreateEngine}, {"destroyEngine", DestroyEngine},
        {"deviceCount", DeviceCount},
        {"setTokenLen16", SetTokenLen16}, {"addSample", AddSample},
        {"addLatin1", AddLatin1}, {"clearCorpus", ClearCorpus},
        {"corpusSize", CorpusSize}, {"readCorpus", ReadCorpus},
        {"findNextMerge", FindNextMerge}, {"applyMerge", ApplyMerge},
        {"applyMerges", ApplyMerges}, {"mergeUntil", MergeUntil},
        {"sampleLengths", SampleLengths}, {"readSamples", ReadSamples},
        {"createEncoder", CreateEncoder}, {"encoderAddMerges", EncoderAddMerges},
        {"encoderClear", EncoderClear}, {"encodeBatch", EncodeBatch},
    };
    for (auto &f : fns) {
        napi_value fn;
        napi_create_function(env, f.name, NAPI_AUTO_LENGTH, f.cb, nullptr, &fn);
        napi_set_named_property(env, exports, f.name, fn);
    }
    return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
