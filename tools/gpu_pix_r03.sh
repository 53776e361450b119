#!/bin/bash
# Round 3: the incremental mode's parity tests, then its C3 run under rocprofv3 (kernel stats).
set -o pipefail
OUT=gpurun_out/${1:-r03p}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_incremental.py tests/test_gpu_parity.py tests/test_scale_configs.py \
    -m gpu -k "pix or incremental" -v --maxfail=3 --timeout 300 --timeout-method thread > "$OUT/pix_tests.log" 2>&1 \
    || { tail -40 "$OUT/pix_tests.log"; exit 1; }
tail -2 "$OUT/pix_tests.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/pix" -o run --output-format csv \
    -- python3 tools/pix_bench.py 1024 7995 > "$OUT/pix.json" 2> "$OUT/pix.err" || { tail -20 "$OUT/pix.err"; exit 1; }
cat "$OUT/pix.json"
python3 tools/trace_gaps.py "$OUT/pix" "$OUT/gaps_pix.json" --from-kernel k_pix_select > /dev/null || exit 1
find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
