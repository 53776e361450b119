/*
 * bpe_tools.h — benchmark/test utilities exported by libbpe (not part of the reference boundary).
 */
#ifndef BPE_TOOLS_H
#define BPE_TOOLS_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Synthetic corpus of SURVEY.md §8(d): xorshift32 (x ^= x<<13; x ^= x>>17; x ^= x<<5) from
 * `seed`, skipping the first `skip` outputs (GF(2) jump-ahead, so a shard can be generated
 * without its prefix), byte = base + floor(x * A / 2^32).  Writes n bytes. */
int bpe_synth_latin1(uint32_t seed, uint32_t A, uint32_t base, uint64_t skip, uint8_t *out,
                     int64_t n);

/* Skewed variant of the synthetic corpus (Zipf s=1.1 words, the worst case for
 * counter contention and for pairs of merged tokens): a list of n_words words, word w of 2..8
 * letters a-z from its own xorshift32 stream; each sample of sample_bytes bytes is a stream of
 * words drawn with P(rank r) ∝ r^-s, each followed by '\n' (1 in 16) or ' ', cut at the sample
 * end.  Sample k depends only on (seed, k), so a shard starting at sample `first_sample` is
 * generated without its prefix.  Writes n bytes (samples first_sample, first_sample + 1, ...). */
int bpe_synth_zipf(uint32_t seed, double s, uint32_t n_words, uint64_t first_sample,
                   int64_t sample_bytes, uint8_t *out, int64_t n);

/* Forces one plain streaming count pass over the current corpus (no merge applied): what
 * findNextMerge does when no counts are cached.  For measuring K1 alone. */
struct bpe_ctx;
int bpe_recount(struct bpe_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif
