// bpe_pixlib.hip — the library primitives the position index is built from (radix sort, scans,
// reduce-by-key, run-length encoding, selection), from hipCUB/rocPRIM, in a translation unit of
// their own so that the engine does not recompile them.  Each wrapper follows hipCUB's two-call
// convention: tmp == nullptr only reports the temp storage it needs in bytes.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>

#include "bpe_pixlib.h"

hipError_t pixlib_sort_pairs(void *tmp, size_t &bytes, const uint32_t *kin, uint32_t *kout,
                             const uint32_t *vin, uint32_t *vout, uint32_t n, hipStream_t s) {
    return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, kin, kout, vin, vout, n, 0, 32, s);
}

hipError_t pixlib_max_scan(void *tmp, size_t &bytes, const int32_t *in, int32_t *out, uint32_t n,
                           hipStream_t s) {
    return hipcub::DeviceScan::InclusiveScan(tmp, bytes, in, out, hipcub::Max(), n, s);
}

hipError_t pixlib_reduce_by_key(void *tmp, size_t &bytes, const uint32_t *keys, uint32_t *uniq,
                                const uint32_t *vals, uint32_t *sums, uint32_t *n_runs, uint32_t n,
                                hipStream_t s) {
    return hipcub::DeviceReduce::ReduceByKey(tmp, bytes, keys, uniq, vals, sums, n_runs,
                                             hipcub::Sum(), n, s);
}

hipError_t pixlib_run_lengths(void *tmp, size_t &bytes, const uint32_t *keys, uint32_t *uniq,
                              uint32_t *lens, uint32_t *n_runs, uint32_t n, hipStream_t s) {
    return hipcub::DeviceRunLengthEncode::Encode(tmp, bytes, keys, uniq, lens, n_runs, n, s);
}

hipError_t pixlib_exclusive_sum(void *tmp, size_t &bytes, const uint32_t *in, uint32_t *out,
                                uint32_t n, hipStream_t s) {
    return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, out, n, s);
}

hipError_t pixlib_select_flagged(void *tmp, size_t &bytes, const int32_t *in, const uint8_t *flags,
                                 int32_t *out, uint32_t *n_sel, uint32_t n, hipStream_t s) {
    return hipcub::DeviceSelect::Flagged(tmp, bytes, in, flags, out, n_sel, n, s);
}
