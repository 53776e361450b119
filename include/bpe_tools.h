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

/* Forces one plain streaming count pass over the current corpus (no merge applied): what
 * findNextMerge does when no counts are cached.  For measuring K1 alone. */
struct bpe_ctx;
int bpe_recount(struct bpe_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif
