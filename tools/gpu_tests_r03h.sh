#!/bin/bash
# Round 3: the maintained-state bug on 2 shards (debug checks after every merge), then the timing
# probes (after-PRE corpus from the product build), smoke, driver and bench.
set -o pipefail
OUT=gpurun_out/${1:-r03h}
mkdir -p "$OUT"
BPE_DEBUG_GLOBAL=1 BPE_DEBUG_BATCH=1 timeout -k 10 300 python3 -u -m pytest tests/test_multi_device.py -m gpu -v -x -s \
    --timeout 170 --timeout-method thread -k "maintained and 2-8" > "$OUT/maint1.log" 2>&1
echo "maint1 rc=$?"; grep -h "bpe debug\|BpeError\|passed\|failed" "$OUT/maint1.log" | tail -30
BPE_DEBUG_GLOBAL=1 timeout -k 10 300 python3 -u -m pytest tests/test_multi_device.py -m gpu -v -x -s \
    --timeout 170 --timeout-method thread -k "maintained and 2-8" > "$OUT/maint.log" 2>&1
echo "maint rc=$?"; grep -h "bpe debug\|BpeError\|passed\|failed" "$OUT/maint.log" | tail -30
tools/probe_breakdown.sh "${1:-r03h}/probe" 1000 || exit 1
tools/gpu_round3.sh "${1:-r03h}" smoke driver bench
