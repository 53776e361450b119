#!/bin/bash
# Round 3: full GPU suite, then the incremental mode (C3) and the zipf C3 stream run under
# rocprofv3 (kernel stats).
set -o pipefail
OUT=gpurun_out/${1:-r03q}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --maxfail=5 --timeout 400 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { grep -E 'FAILED|Error|error' "$OUT/pytest_gpu.log" | head -30; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/pix" -o run --output-format csv \
    -- python3 tools/pix_bench.py 1024 7995 > "$OUT/pix.json" 2> "$OUT/pix.err" || { tail -20 "$OUT/pix.err"; exit 1; }
cat "$OUT/pix.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/zipf" -o run --output-format csv \
    -- python3 bench.py --corpus zipf --no-cpu-baseline > "$OUT/zipf.jsonl" 2> "$OUT/zipf.err" || { tail -20 "$OUT/zipf.err"; exit 1; }
head -c 1200 "$OUT/zipf.jsonl"
find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
