// bpe_pixlib.h — internal: hipCUB primitives for the position index (csrc/bpe_pixlib.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

hipError_t pixlib_sort_pairs(void *tmp, size_t &bytes, const uint32_t *kin, uint32_t *kout,
                             const uint32_t *vin, uint32_t *vout, uint32_t n, hipStream_t s);
hipError_t pixlib_max_scan(void *tmp, size_t &bytes, const int32_t *in, int32_t *out, uint32_t n,
                           hipStream_t s);
hipError_t pixlib_reduce_by_key(void *tmp, size_t &bytes, const uint32_t *keys, uint32_t *uniq,
                                const uint32_t *vals, uint32_t *sums, uint32_t *n_runs, uint32_t n,
                                hipStream_t s);
hipError_t pixlib_run_lengths(void *tmp, size_t &bytes, const uint32_t *keys, uint32_t *uniq,
                              uint32_t *lens, uint32_t *n_runs, uint32_t n, hipStream_t s);
hipError_t pixlib_exclusive_sum(void *tmp, size_t &bytes, const uint32_t *in, uint32_t *out,
                                uint32_t n, hipStream_t s);
hipError_t pixlib_select_flagged(void *tmp, size_t &bytes, const int32_t *in, const uint8_t *flags,
                                 int32_t *out, uint32_t *n_sel, uint32_t n, hipStream_t s);
