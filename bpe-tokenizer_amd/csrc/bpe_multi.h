// bpe_multi.h — internal: one corpus sharded over several HIP devices behind one bpe_ctx
// (bpe_create_multi, include/bpe.h).  bpe_engine.hip forwards every C-ABI call made on such a
// context here; the shards are ordinary single-device contexts driven through the same C ABI.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "bpe.h"

struct bpe_multi;

int multi_create(bpe_multi **out, int n_shards, const int *devices, int reduce);
int multi_destroy(bpe_multi *m);
int multi_set_token_len16(bpe_multi *m, int32_t id, int32_t len16);
int multi_num_tokens(bpe_multi *m, int32_t *n);
int multi_add_sample(bpe_multi *m, const int32_t *ids, int64_t n);
int multi_add_latin1(bpe_multi *m, const uint8_t *bytes, int64_t n, int64_t sample_bytes,
                     int32_t char_to_id[256], int32_t *n_tokens_io, int64_t char_hist[256]);
int multi_clear_corpus(bpe_multi *m);
int multi_corpus_size(bpe_multi *m, int64_t *n_samples, int64_t *n_tokens);
int multi_read_corpus(bpe_multi *m, int32_t *ids_out, int64_t ids_cap, int64_t *sample_off,
                      int64_t off_cap);
int multi_sample_lengths(bpe_multi *m, int64_t *lens, int64_t cap);
int multi_read_samples(bpe_multi *m, const int64_t *idx, int64_t n, int32_t *ids_out,
                       int64_t ids_cap, int64_t *off);
int multi_find_next_merge(bpe_multi *m, int64_t max_length, int64_t min_weight, int32_t *a,
                          int32_t *b, int64_t *w);
int multi_apply_merge(bpe_multi *m, int32_t a, int32_t b, int32_t c, int64_t *replaced);
int multi_apply_merges(bpe_multi *m, const int32_t *abc, int64_t n, int64_t *replaced,
                       int count_after);
int multi_merge_until(bpe_multi *m, int64_t max_length, int64_t min_weight,
                      int64_t max_iterations, int64_t *out_abw, int64_t cap, int64_t *n_merges);
int multi_stats_enable(bpe_multi *m, int on);
int multi_get_stats(bpe_multi *m, bpe_stats *out);
int multi_reset_stats(bpe_multi *m);
int multi_get_stream(bpe_multi *m, void **stream);
int multi_shard_count(bpe_multi *m, int *n);
// explicit_choice: the caller's bpe_set_mode (false: the automatic switch past AUTO_PIX_VOCAB ids)
int multi_set_mode(bpe_multi *m, int mode, bool explicit_choice = true);

// shards that share one device exchange through a device kernel (bpe_engine.hip)
constexpr int BPE_MAX_SHARDS_ONE_DEVICE = 16;
extern "C" int bpe_sum_shards(unsigned long long *const *bufs, int n, size_t count, int take_max,
                              void *stream);

// (bpe_multi.cpp) a context going away frees its rank communicator (bpe_rank_rccl_init)
void rank_rccl_forget(bpe_ctx *ctx);

// (bpe_engine.hip) the exchange and tie buffers and the exchange's word count of the context's
// open rank-loop batch (bpe_rank_loop_begin); BPE_ERR_STATE when no batch is open
int rank_loop_buffers(bpe_ctx *c, unsigned long long **xchg, unsigned long long **tie, int64_t *words);

// error reporting shared with bpe_engine.hip
int bpe_fail(int code, const char *msg);
