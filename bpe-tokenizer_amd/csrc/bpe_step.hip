// bpe_step.hip — the table-state merge pass of the device loop (k_step_loop<MODE_TABLE>, the
// C3 hot path) in a translation unit of its own, compiled with
// -mllvm -structurizecfg-skip-uniform-regions (bpe-tokenizer_amd/Makefile).  With the flag the
// uniform branches of the ring stay scalar branches instead of lane-mask regions: k_step_loop
// 0.789 -> 0.775 ms at C3 (tools/ab_exp.sh, profiles/r03_ab_skip_uniform.json).  The same flag
// made the maintained-state pass (MODE_INCR) 2 % slower on zipf C3, so only this instantiation
// takes it, with its own scheduling flags and ring depth (Makefile STEP_FLAGS).
//
// The kernel header is included with internal linkage (an anonymous namespace), so its other
// kernels are not defined twice in libbpe.so; the launcher therefore takes the engine's
// structures as untyped pointers (same layout: the same header).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wunused-function"   // (the header's other kernels, unused here)
namespace {
#include "bpe_kernels.hip.h"
}
#pragma clang diagnostic pop

namespace bpe_step {

hipError_t launch_step_loop_table(unsigned grid, hipStream_t s, int32_t *ids, int64_t n_chunks,
                                  int64_t cpr, int R, const void *carry, const void *ctl,
                                  uint32_t *partials, unsigned long long *spill, const void *ct,
                                  void *sums, unsigned long long *replaced) {
    using namespace bpe;
    k_step_loop<MODE_TABLE><<<grid, WG, 0, s>>>(
        ids, n_chunks, cpr, R, static_cast<const RegionCarry *>(carry),
        static_cast<const LoopCtl *>(ctl), partials, spill, *static_cast<const ColdTable *>(ct),
        static_cast<RegionSum *>(sums), replaced);
    return hipGetLastError();
}

// The host path's passes of the table state (findNextMerge / applyMerge one call each, the counts
// after a compaction, core.ts:247-360): k_step<NO_MERGE | MERGE_XY | MERGE_XX, MODE_TABLE>, built
// here with the same flags as the device loop's pass (in the engine's translation unit, with its
// 6-slot ring and default flags, the merge pass timed 0.80-0.82 ms at C3 against 0.74 here).
hipError_t launch_step_table(int merge, unsigned grid, hipStream_t s, int32_t *ids, int64_t n_chunks,
                             int64_t cpr, int R, const void *carry, int32_t ma, int32_t mb,
                             int32_t mc, uint32_t *partials, unsigned long long *spill,
                             const void *ct, const uint32_t *heavy, void *sums,
                             unsigned long long *replaced) {
    using namespace bpe;
    const RegionCarry *rc = static_cast<const RegionCarry *>(carry);
    const ColdTable &t = *static_cast<const ColdTable *>(ct);
    RegionSum *su = static_cast<RegionSum *>(sums);
    if (merge == MERGE_XX)
        k_step<MERGE_XX, MODE_TABLE><<<grid, WG, 0, s>>>(ids, n_chunks, cpr, R, rc, ma, mb, mc,
                                                        partials, spill, t, heavy, su, replaced);
    else if (merge == MERGE_XY)
        k_step<MERGE_XY, MODE_TABLE><<<grid, WG, 0, s>>>(ids, n_chunks, cpr, R, rc, ma, mb, mc,
                                                        partials, spill, t, heavy, su, replaced);
    else
        k_step<NO_MERGE, MODE_TABLE><<<grid, WG, 0, s>>>(ids, n_chunks, cpr, R, rc, ma, mb, mc,
                                                        partials, spill, t, heavy, su, replaced);
    return hipGetLastError();
}

}  // namespace bpe_step
