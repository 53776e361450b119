#!/bin/bash
# Round 3: the max_length hand-off test on the previous build (expected to fail there), then the
# incremental-mode tests and C3 run on the current one (tools/gpu_pix_r03.sh).
set -o pipefail
OUT=gpurun_out/${1:-r03ml}
mkdir -p "$OUT"
BPE_LIB=gpurun_exp/base.so timeout -k 10 300 python3 -u -m pytest tests/test_incremental.py -m gpu -k max_length \
    -v --timeout 120 --timeout-method thread > "$OUT/base_ml.log" 2>&1
rc=$?
tail -3 "$OUT/base_ml.log"
[ $rc -le 1 ] || exit $rc
tools/gpu_pix_r03.sh "${1:-r03ml}"
