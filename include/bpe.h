/*
 * bpe.h — C ABI of libbpe: the MI355X (gfx950) engine for the BPE merge-training hot path of
 * beenotung/bpe-tokenizer (reference: /root/reference/core.ts, v2.2.0).
 *
 * The reference has no FFI layer: its drop-in boundary is the public `BPETokenizer` class
 * (core.ts:77).  These entry points are exactly what that class's corpus-touching methods need;
 * the host side (bpe-tokenizer_amd/js/core.js over the N-API addon, or any ctypes/cgo binding —
 * see INTEGRATION.md) keeps the token table, codes, JSON and encode/decode bookkeeping and calls
 * down here for every pass over the corpus.
 *
 * Conventions
 *   - Every function returns an int status: BPE_OK (0), BPE_NO_MERGE (1, "findNextMerge returned
 *     null"), or a negative error code; bpe_last_error() returns the message of the last error
 *     raised on the calling thread.
 *   - Token ids are the reference's `token.index` (code point of `token.code` minus one,
 *     core.ts:149,189,316,485).  Ids must stay below BPE_MAX_VOCAB (55 296): above it the
 *     reference's codes become lone UTF-16 surrogates (hard part 8).
 *   - Caller-owned host buffers are copied in/out; the library never retains host pointers.
 *   - A context owns one HIP device, one stream and all device memory of one corpus shard.
 *   - There is no CPU fallback: without a usable HIP device bpe_create() fails with BPE_ERR_HIP.
 */
#ifndef BPE_H
#define BPE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BPE_OK 0
#define BPE_NO_MERGE 1
#define BPE_ERR_ARG (-1)
#define BPE_ERR_HIP (-2)
#define BPE_ERR_OOM (-3)
#define BPE_ERR_STATE (-4)
#define BPE_ERR_VOCAB (-5)
/* The incremental mode's position index does not fit beside this shard's corpus in device memory
 * (bpe_set_global_counts on a shard in BPE_MODE_INCREMENTAL).  Nothing was changed: the streaming
 * mode, which needs no index, can go on.  Drivers fall back to it on this code only. */
#define BPE_ERR_NOFIT (-6)

#define BPE_MAX_VOCAB 55296

typedef struct bpe_ctx bpe_ctx;

/* Library version (major*10000 + minor*100 + patch). */
int bpe_version(void);

/* Copies the last error message of this thread (NUL-terminated, truncated to cap). */
int bpe_last_error(char *buf, size_t cap);

/* Number of visible HIP devices (0 when none). */
int bpe_device_count(int *n);

/* `new BPETokenizer()` (core.ts:77-106): an empty corpus shard on HIP device `device`. */
int bpe_create(bpe_ctx **out, int device);
int bpe_destroy(bpe_ctx *ctx);

/* One corpus sharded over n_shards HIP devices behind one context (the drop-in's BPE_NUM_GPUS;
 * SURVEY.md §5, §8(e)).  devices: n_shards device indices (NULL: 0 .. n_shards-1).  Every entry
 * point below works on it as on a single-device context, with identical results: the shards hold
 * contiguous runs of whole samples (pairs never cross samples, core.ts:265-267), samples added
 * before the first pass are cut into runs of about equal size, later ones go to the last shard.
 * Per merge iteration the shards all-reduce their pair tables and tie positions:
 *   BPE_REDUCE_RCCL — RCCL communicators over the devices (ncclCommInitAll, grouped calls on the
 *                     shards' streams; one shard per device);
 *   BPE_REDUCE_HOST — host copies (any placement, e.g. several shards on one device: tests).
 * The per-shard entry points (bpe_export_counts ... bpe_rank_loop_*, bpe_recount) refuse a
 * multi-device context. */
#define BPE_REDUCE_RCCL 0
#define BPE_REDUCE_HOST 1
int bpe_create_multi(bpe_ctx **out, int n_shards, const int *devices, int reduce);
int bpe_shard_count(bpe_ctx *ctx, int *n_shards);

/* ---- vocabulary ------------------------------------------------------------------------------
 * Registers token `id` with the UTF-16 length of its chars (`token.chars.length`, used by the
 * max_length filter, core.ts:270-273).  Grows the table when id >= current size.  Called by the
 * host for every new char token (core.ts:186-199) and on fromJSON (core.ts:147-162); merged tokens
 * are registered by bpe_apply_merge itself (len16[c] = len16[a] + len16[b], core.ts:318). */
int bpe_set_token_len16(bpe_ctx *ctx, int32_t id, int32_t len16);
int bpe_num_tokens(bpe_ctx *ctx, int32_t *n_tokens);

/* ---- corpus ----------------------------------------------------------------------------------
 * addToCorpus (core.ts:182-207) / restoreToCorpus (core.ts:213-216): appends ONE sample whose
 * chars the host has already mapped to token ids.  n may be 0 (an empty sample). */
int bpe_add_sample(bpe_ctx *ctx, const int32_t *ids, int64_t n);

/* Bulk native ingest for corpora JS strings cannot hold: `n` latin1 bytes
 * (byte b == code point b), split into samples of `sample_bytes` (last one shorter; 0 = one
 * sample).  char_to_id[256] is in/out: -1 marks an unseen char; unseen chars get ids
 * *n_tokens_io, *n_tokens_io+1, ... in first-appearance order (core.ts:186-199).  char_hist[256]
 * receives the per-char occurrence counts of this call (the weight/original_weight increments of
 * core.ts:192-202).  Each new char is registered with len16 = 1. */
int bpe_add_latin1(bpe_ctx *ctx, const uint8_t *bytes, int64_t n, int64_t sample_bytes,
                   int32_t char_to_id[256], int32_t *n_tokens_io, int64_t char_hist[256]);

/* `corpus_in_code = []` (example/import-merge-log-to-ram.ts:21-22): drops every sample. */
int bpe_clear_corpus(bpe_ctx *ctx);

/* Sample count and live token count (excluding sample separators). */
int bpe_corpus_size(bpe_ctx *ctx, int64_t *n_samples, int64_t *n_tokens);

/* Materialises `corpus_in_code` (core.ts:106): all samples' ids back to back into ids_out
 * (capacity ids_cap) and n_samples+1 offsets into sample_off (capacity off_cap). */
int bpe_read_corpus(bpe_ctx *ctx, int32_t *ids_out, int64_t ids_cap, int64_t *sample_off,
                    int64_t off_cap);

/* Live token count of every sample, in corpus order (cap >= n_samples).  A merge shortens
 * exactly the samples it rewrites, so comparing lengths before and after finds the rows
 * BPETokenizerDB.applyMerge selects and updates (db/core.ts:399-417: `like '%from_code%'` +
 * `update corpus`).  Two reads of the corpus on the device; n_samples x 8 B come back. */
int bpe_sample_lengths(bpe_ctx *ctx, int64_t *lens, int64_t cap);

/* Reads back the samples idx[0..n) (any order, repeats allowed): their ids packed in that order
 * into ids_out (capacity ids_cap), sample k at [sample_off[k], sample_off[k+1]) (n+1 offsets).
 * The db twin's row write-back (db/core.ts:414-417) without materialising the whole corpus. */
int bpe_read_samples(bpe_ctx *ctx, const int64_t *idx, int64_t n, int32_t *ids_out, int64_t ids_cap,
                     int64_t *sample_off);

/* ---- hot path ----------------------------------------------------------------------------------
 * findNextMerge (core.ts:247-326).  max_length: 0 = falsy = unlimited (core.ts:255,272);
 * min_weight: 0 = falsy = 2 (core.ts:256).  On BPE_OK writes the chosen pair (a, b) and its count
 * W (== c.weight == c.original_weight, core.ts:317-323); BPE_NO_MERGE when the reference returns
 * null (core.ts:312-313).  The selection is bit-identical to the reference's running argmax
 * (max W, then min a+b, then earliest W-th counted occurrence — SURVEY.md Appendix A). */
int bpe_find_next_merge(bpe_ctx *ctx, int64_t max_length, int64_t min_weight, int32_t *a,
                        int32_t *b, int64_t *w);

/* applyMerge corpus rewrite (core.ts:356-359, `replaceAll(a.code+b.code, c.code)`): every
 * leftmost non-overlapping occurrence of (a, b) becomes c.  Also registers c (len16 sum).
 * `replaced` (may be NULL) receives the replacement count (== W for a merge from findNextMerge). */
int bpe_apply_merge(bpe_ctx *ctx, int32_t a, int32_t b, int32_t c, int64_t *replaced);

/* A run of applyMerge rewrites without counting pairs: restoreMerge replay (core.ts:477-494,
 * `example/import-merge-log-to-ram.ts`) and batch encoding of a corpus with a trained merge list
 * (encodeToCode, core.ts:392-409, applies the merges in order with replaceAll).  abc holds n
 * triples (a, b, c), applied in order, each registering c as bpe_apply_merge does.  One
 * apply-only streaming pass per merge.  count_after != 0: the last merge is applied by the fused
 * apply + count pass, so a findNextMerge that follows streams nothing extra.  replaced (may be
 * NULL) receives n replacement counts. */
int bpe_apply_merges(bpe_ctx *ctx, const int32_t *abc, int64_t n, int64_t *replaced,
                     int count_after);

/* mergeUntil (core.ts:365-383).  max_iterations 0 = unlimited.  New tokens get ids
 * bpe_num_tokens(), bpe_num_tokens()+1, ...  (core.ts:315).  Writes (a, b, W) int64 triples into
 * out_abw (capacity `cap` triples) and the number of merges into *n_merges. */
int bpe_merge_until(bpe_ctx *ctx, int64_t max_length, int64_t min_weight, int64_t max_iterations,
                    int64_t *out_abw, int64_t cap, int64_t *n_merges);

/* ---- sharded corpus (one process per GPU) ------------------------------------------------------
 * Pairs never cross samples (core.ts:265-267), so a corpus split at sample boundaries is counted
 * shard by shard; the caller sums the shards' tables (all-reduce / all-gather over RCCL) and
 * selects from the global table.  All table pointers below are DEVICE pointers on this context's
 * device (e.g. torch tensors); host pointers are marked.
 *
 * The pair-count table has BPE_TABLE_BINS u64 entries: [0, 65536) exact counts of the pairs with
 * both ids < 256 at b*256+a, [65536, 81920) a count sketch of every other pair (bucket =
 * ((b * 0x19B1 + a / 2) mod 8192) * 2 + (a & 1)): an upper bound of each such pair's count. */
#define BPE_HOT_BINS 65536
#define BPE_TABLE_BINS 81920

/* This shard's table for the current corpus (one streaming pass if none is cached). */
int bpe_export_counts(bpe_ctx *ctx, uint64_t *table);

/* Given the GLOBAL (summed) table: the cold pairs whose sketch bucket reaches the best hot count
 * (the only ones that can still win) are counted exactly on this shard (one streaming pass) and
 * written as cold_keys[i] = a<<16|b (u32), cold_counts[i] (u64).  *n_cold = entries; -1 (and no
 * pass) when no bucket qualifies, a decision every rank reaches alike from the same global table,
 * so the cold-list exchange can be skipped; when *n_cold > cap nothing is written and
 * BPE_ERR_ARG is returned (retry with a bigger buffer). */
int bpe_heavy_counts(bpe_ctx *ctx, const uint64_t *table, int64_t max_length, uint32_t *cold_keys,
                     uint64_t *cold_counts, int64_t cap, int64_t *n_cold);

/* findNextMerge's selection (core.ts:294-313) over the GLOBAL table's exact hot bins plus the
 * GLOBAL exact cold entries (distinct keys).  Writes W and the candidate pairs sharing the best
 * (W, a+b) as host int32 (a, b) pairs into cand (capacity cap pairs); *n_cand may exceed cap
 * (then only cap written).  BPE_NO_MERGE when the reference would return null. */
int bpe_select_counts(bpe_ctx *ctx, const uint64_t *table, const uint32_t *cold_keys,
                      const uint64_t *cold_counts, int64_t n_cold, int64_t max_length,
                      int64_t min_weight, int32_t *cand, int64_t cap, int64_t *n_cand,
                      int64_t *w);

/* Rule R3 on this shard: for each host (a, b) pair in cand, the shard-local position + 1 of its
 * last counted occurrence (0 when none) into host last[n].  Positions grow in corpus order. */
int bpe_tie_positions(bpe_ctx *ctx, const int32_t *cand, int64_t n, uint64_t *last);

/* ---- the device-resident loop on one rank of a sharded corpus ---------------------------------
 * mergeUntil (core.ts:365-383) over shards with no host sync per iteration.  `xchg`
 * (BPE_XCHG_WORDS u64) and `tie` (BPE_TIE_WORDS u64) are DEVICE buffers the caller all-reduces IN
 * ORDER on this context's stream (bpe_get_stream; e.g. RCCL on that stream).  Per iteration:
 *   all-reduce(SUM, xchg[0 .. *xchg_words)); bpe_rank_loop_select;
 *   all-reduce(MAX, tie[0 .. BPE_TIE_WORDS)); bpe_rank_loop_decide; bpe_rank_loop_count
 * at most BPE_LOOP_BATCH times between bpe_rank_loop_begin and bpe_rank_loop_end.  Every rank takes
 * the same decisions from the same global tables, so all ranks run the same collectives; an
 * iteration after the batch has ended is a no-op (its collectives still run).
 * The exchange holds a header (BPE_XCHG_HDR words; word 0: this shard's replacement count of the
 * merge just applied, so that the sum checked against W covers every shard) and either
 *   - this shard's pair table (BPE_TABLE_BINS words), summed into the global table, or
 *   - after bpe_set_global_counts (the maintained state: every rank holds the GLOBAL hot and cold
 *     tables and keeps them merge by merge), BPE_DELTA_ROWS delta rows per token id: this shard's
 *     recount of every pair the merge (a, b) -> c touched, at HDR + 6 * other + row, rows
 *     (a, .) (b, .) (., a) (., b) (c, .) (., c) in this order of precedence.  In the
 *     incremental mode (bpe_set_mode) the global state lives in the shard's position index instead
 *     (every pair's global count beside this shard's own lists) and the exchange carries each
 *     merge's count CHANGES: 16 words for the pairs of two of {a, b, c} (signed, two's complement
 *     u64), then per token id and side the sites with that neighbour (left: (x, a) -> (x, c);
 *     right: (b, y) -> (c, y)) in unsigned lanes as wide as the last merge's count, packed in the
 *     u64 words (their u64 sum adds the lanes without carries).  *xchg_words is
 *     then 8 + 16 + 2 ceil(ids / lanes per word) for the batch's ids.
 *     A tie there takes one iteration of its own: the scan's positions cross in `tie`, and the
 *     next iteration commits the winner, so a batch may merge fewer times than it iterates.
 * tie: the tied candidates' last positions (rank << 40 | position, rule R3: rank r's occurrences
 * come after rank r-1's) in words 0..15, and word 16 this rank's vote for the host path (facts of
 * its own copy of the maintained tables: fill, dead claims, room).  A tie between pairs X Y is
 * decided from the corpus tail, which only the last rank (world - 1) scans.
 * bpe_rank_loop_begin writes this shard's part of the first exchange and *xchg_words (the words to
 * all-reduce per iteration of this batch: the same on every rank).  bpe_rank_loop_end syncs and
 * writes the batch's merges as (a, b, W, this shard's replacement count) quadruples into host
 * out_abwr (capacity cap quadruples; sum the counts over the shards: == W), *status:
 * 0 = every enqueued iteration merged, 1 = no pair qualifies (stop), 2 = the next iteration needs
 * the host protocol (heavy sketch buckets, more than BPE_MAX_CAND tied pairs, a vote: export /
 * heavy / select / tie_positions above).  A batch of the maintained state that ran to its end
 * leaves its last merge's delta rows in xchg for the next batch's first exchange: pass the same
 * buffer again. */
#define BPE_MAX_CAND 16
#define BPE_LOOP_BATCH 64
#define BPE_XCHG_HDR 8
#define BPE_DELTA_ROWS 6
#define BPE_XCHG_WORDS (BPE_XCHG_HDR + BPE_DELTA_ROWS * BPE_MAX_VOCAB)
#define BPE_TIE_WORDS 32
int bpe_rank_loop_begin(bpe_ctx *ctx, int64_t max_length, int64_t min_weight, uint64_t *xchg,
                        uint64_t *tie, int rank, int world, int64_t *xchg_words);
int bpe_rank_loop_select(bpe_ctx *ctx);
int bpe_rank_loop_decide(bpe_ctx *ctx);
int bpe_rank_loop_count(bpe_ctx *ctx);
int bpe_rank_loop_end(bpe_ctx *ctx, int64_t *out_abwr, int64_t cap, int64_t *n_merges, int *status);

/* The maintained state of a sharded corpus (skewed corpora, large vocabularies: the cold pairs
 * outgrow the sketch).  Every rank: bpe_cold_counts (its exact count of every pair with an id >=
 * 256, one streaming pass; *n > cap: nothing written, call again with room, no second pass), then
 * the lists of ALL ranks gathered (e.g. all-gather) and bpe_set_global_counts with the global table
 * (all-reduced bpe_export_counts) and the gathered lists (device pointers; duplicate keys summed).
 * The next rank loop batches keep those global tables up to date with delta rows (above); any
 * per-shard entry point (find/apply/export/...) drops the state.  In the incremental mode
 * bpe_set_global_counts builds the shard's position index and loads the global counts into it
 * (enter at once: a driver need not wait for the cold pairs to outgrow the sketch). */
int bpe_cold_counts(bpe_ctx *ctx, uint32_t *keys, uint64_t *counts, int64_t cap, int64_t *n);

/* The rank loop's collectives from C++ (one process per GPU): an RCCL
 * communicator per context, and a batch's iterations enqueued by one call.  Rank 0 makes the id
 * (bpe_rccl_unique_id, 128 bytes: NCCL_UNIQUE_ID_BYTES), the caller broadcasts it (e.g.
 * torch.distributed), then every rank calls bpe_rank_rccl_init (collective).  Between
 * bpe_rank_loop_begin and bpe_rank_loop_end, bpe_rank_loop_rccl(ctx, xchg, xchg_words, tie, k) runs
 * k iterations of: ncclAllReduce(SUM, xchg[0 .. xchg_words)); bpe_rank_loop_select;
 * ncclAllReduce(MAX, tie); bpe_rank_loop_decide; bpe_rank_loop_count — all on the context's
 * stream (no host sync, no cross-stream events).  The RCCL is the one beside the HIP runtime libbpe
 * runs on.  bpe_destroy frees the communicator; bpe_rank_rccl_destroy frees it earlier. */
int bpe_rccl_unique_id(void *id, size_t cap);
int bpe_rank_rccl_init(bpe_ctx *ctx, const void *id, int rank, int world);
int bpe_rank_loop_rccl(bpe_ctx *ctx, uint64_t *xchg, int64_t xchg_words, uint64_t *tie, int iterations);
int bpe_rank_rccl_destroy(bpe_ctx *ctx);
int bpe_set_global_counts(bpe_ctx *ctx, const uint64_t *table, const uint32_t *keys,
                          const uint64_t *counts, int64_t n);

/* ---- modes -------------------------------------------------------------------------------------
 * BPE_MODE_STREAM (default): every merge is one fused streaming pass over the corpus (apply the
 * merge, recount every pair): the reference's own full recount (core.ts:265-310), at HBM rate.
 * BPE_MODE_INCREMENTAL: bpe_merge_until works on a position index: per
 * merge only the W match sites and their neighbours are touched, O(W) instead of O(N).  Same
 * merges, counts and corpus; it changes what pair-scans/s measures, so it is reported apart.
 * Built per call by a hand-written counting scatter of the corpus's positions into per-pair lists
 * (one count pass, one exclusive scan, two fill passes; no sort); 32-bit positions, so up to
 * 0xFFFF0000 live slots per context or shard.  Env BPE_PIX=1 selects it for new contexts.  On a
 * multi-device context (bpe_create_multi) the mode applies to every shard: each shard indexes its
 * own samples inside the rank loop (above). */
#define BPE_MODE_STREAM 0
#define BPE_MODE_INCREMENTAL 1
int bpe_set_mode(bpe_ctx *ctx, int mode);

/* ---- measurement -------------------------------------------------------------------------------
 * HIP-event timings of the kernels, recorded on the context's own stream. */
typedef struct {
    double step_ms;           /* fused streaming pass (K1 count + K4 apply of the pending merge) */
    int64_t step_launches;
    int64_t step_slots;       /* int32 slots streamed by those passes (live + dead) */
    int64_t step_live;        /* live corpus tokens at those passes (pair-scans) */
    double select_ms;         /* boundary stitch + reduce + argmax + collect + R3 tie passes */
    int64_t tie_passes;       /* R3 tie-break passes */
    int64_t iterations;       /* findNextMerge calls */
    int64_t live_tokens;      /* sum over those calls of live corpus tokens (pair-scans) */
    int64_t compactions;      /* dead-slot compactions */
    int64_t exact_passes;     /* extra streaming passes for cold pairs whose sketch bucket could win */
    int64_t step_timed;       /* streaming passes whose duration step_ms sums (the device loop times
                                 every SPAN_EVERY-th iteration, all of its spans; select_ms covers
                                 those same iterations) */
    int64_t tie_tail;         /* device loop: R3 ties decided from the corpus-tail window alone */
    int64_t tie_lone;         /* ... of which the lone candidate missing from the window won */
    int64_t loop_host;        /* device loop: iterations handed to the host path (heavy sketch
                                 buckets, > BPE_MAX_CAND tied pairs, >= 2 tied pairs missing from
                                 the tail window, the vocabulary limit) */
    int64_t fused_passes;     /* merge passes that also refreshed the maintained cold-pair table */
    int64_t pix_builds;       /* incremental mode: position-index builds (one counting scatter of
                                 the corpus's positions) */
    int64_t pix_merges;       /* incremental mode: merges made on the index (O(W) each) */
    int64_t pix_host;         /* incremental mode: iterations the index handed to the stream */
    double pix_build_ms;      /* incremental mode: wall time of those builds (host clock, synced) */
    int64_t cold_used;        /* maintained state: claimed entries of the cold-pair table (largest seen) */
    int64_t sel_blocks;       /* maintained state: block maxima recomputed by incremental selections
                                 (cumulative since the context was made) */
    int64_t xchg_bytes;       /* rank loop: bytes of the per-iteration exchange all-reduced (SUM leg;
                                 the table, or the maintained state's delta rows), summed over the
                                 iterations (a multi-device context: over its shards) */
    int64_t xchg_iters;       /* rank loop: iterations those bytes cover */
    int64_t pix_fallbacks;    /* multi-device context, incremental mode: times the shards' index kept
                                 handing over and the run went on in the streaming mode */
    int64_t cold_rebuilds;    /* maintained state: cold pair tables rebuilt from their own live
                                 claims (instead of an exact pass over the corpus) */
    double incr_ms;           /* the device loop's maintained-state passes (k_step_loop<MODE_INCR>)
                                 among the timed step spans: their durations, */
    int64_t incr_timed;       /* ... their number, */
    int64_t incr_launches;    /* ... all such passes, */
    int64_t incr_live;        /* ... and the live corpus tokens summed over them (pair-scans) */
    int64_t unscreened_passes;/* device loop, table state: merge passes whose LDS adds return nothing
                                 and skip the overflow screen (no counter can reach 16 bits: the
                                 largest table bin + 2 W < 2^16) */
} bpe_stats;

int bpe_stats_enable(bpe_ctx *ctx, int on);
int bpe_get_stats(bpe_ctx *ctx, bpe_stats *out);
int bpe_reset_stats(bpe_ctx *ctx);

/* Raw device pointer of the context's HIP stream (hipStream_t), for callers that order their own
 * work (collectives, events) against the engine. */
int bpe_get_stream(bpe_ctx *ctx, void **stream);

/* ---- encoding ----------------------------------------------------------------------------------
 * encodeToCode (core.ts:392-409) for a batch of texts with a trained merge list, apart from any
 * corpus: `for (let [from_code, to_code] of this.merge_codes) content_in_code =
 * content_in_code.replaceAll(from_code, to_code)` (core.ts:404-406) on every text.  An encoder
 * holds the merge list as a rank table on one device.  A text of up to
 * BPE_ENCODE_LDS_TOKENS tokens is encoded by one workgroup in LDS: the lowest-ranked merge present is rewritten
 * (all its leftmost non-overlapping occurrences) until none is, which equals the in-order replay
 * whenever no merge's new token c is an input (a or b) of itself or an earlier merge — every list
 * the reference makes (c is a fresh index, core.ts:315,484).  Longer texts, and lists that break
 * that rule (checked as merges are added), are replayed merge by merge by apply-only streaming
 * passes (bpe_apply_merges on a scratch engine of the encoder).  Output is identical either way. */
#define BPE_ENCODE_LDS_TOKENS 16384
typedef struct bpe_encoder bpe_encoder;
typedef struct {
    double kernel_ms;         /* HIP-event time of the merge-rank kernels (per call: launch to end) */
    int64_t calls;            /* bpe_encode_batch calls */
    int64_t texts_rank;       /* texts encoded by the merge-rank kernels */
    int64_t texts_replay;     /* texts replayed by apply-only passes (long, or a non-greedy list) */
    int64_t tokens_in;        /* ids in */
    int64_t tokens_out;       /* ids out */
    int64_t steps;            /* merge-rank kernels: greedy steps (ranks rewritten), all texts */
} bpe_encoder_stats;

/* An encoder with no merges on HIP device `device` (fails with BPE_ERR_HIP without one). */
int bpe_encoder_create(bpe_encoder **out, int device);
int bpe_encoder_destroy(bpe_encoder *enc);
/* Appends n merges (a, b, c) in list order (`merge_codes`, core.ts:91,352; restoreMerge
 * core.ts:477-494 and fromJSON core.ts:163-169 append the same way).  Ids < BPE_MAX_VOCAB. */
int bpe_encoder_add_merges(bpe_encoder *enc, const int32_t *abc, int64_t n);
/* Drops every merge (fromJSON of another tokenizer, core.ts:140-145). */
int bpe_encoder_clear(bpe_encoder *enc);
int bpe_encoder_num_merges(bpe_encoder *enc, int64_t *n);
/* Encodes n_texts texts: text k = ids[off[k] .. off[k+1]) (token ids, `token.index`).  Writes the
 * encoded texts back to back into ids_out (capacity off[n_texts] - off[0]: a text never grows) and
 * n_texts + 1 offsets into out_off (out_off[0] = 0). */
int bpe_encode_batch(bpe_encoder *enc, const int32_t *ids, const int64_t *off, int64_t n_texts,
                     int32_t *ids_out, int64_t *out_off);
int bpe_encoder_get_stats(bpe_encoder *enc, bpe_encoder_stats *out);
int bpe_encoder_reset_stats(bpe_encoder *enc);

#ifdef __cplusplus
}
#endif
#endif /* BPE_H */
