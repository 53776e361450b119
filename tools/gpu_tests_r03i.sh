#!/bin/bash
# Round 3: the 2-shard maintained-state bug with the all-reduce detector, then driver + bench.
set -o pipefail
OUT=gpurun_out/${1:-r03i}
mkdir -p "$OUT"
BPE_DEBUG_GLOBAL=1 timeout -k 10 300 python3 -u -m pytest tests/test_multi_device.py -m gpu -v -x -s \
    --timeout 170 --timeout-method thread -k "maintained and 2-8" > "$OUT/maint.log" 2>&1
echo "maint rc=$?"; grep -h "bpe debug\|BpeError\|passed\|failed" "$OUT/maint.log" | tail -40
tools/gpu_round3.sh "${1:-r03i}" driver bench
