#!/bin/bash
# Round 3: the maintained-state diagnostics (BPE_DEBUG_GLOBAL), the single-context loop tests of
# the fused selection kernels, the timing probes, the bench line.
set -o pipefail
OUT=gpurun_out/${1:-r03g}
mkdir -p "$OUT"
BPE_DEBUG_GLOBAL=1 timeout -k 10 300 python3 -u -m pytest tests/test_multi_device.py -m gpu -v -x -s \
    --timeout 170 --timeout-method thread -k "maintained" > "$OUT/maint.log" 2>&1
echo "maint rc=$?"; grep -h "bpe debug\|BpeError\|passed\|failed" "$OUT/maint.log" | tail -12
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_incremental.py -m gpu -v --maxfail=3 \
    --timeout 170 --timeout-method thread -k "loop or zipf or cold" > "$OUT/loop.log" 2>&1 \
    || { tail -30 "$OUT/loop.log"; exit 1; }
tail -2 "$OUT/loop.log"
tools/probe_breakdown.sh "${1:-r03g}/probe" 1000 || exit 1
tools/gpu_round3.sh "${1:-r03g}" smoke driver bench
