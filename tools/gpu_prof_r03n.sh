#!/bin/bash
# Round 3: kernel stats of the incremental mode (C3, full run) and of the zipf C3 stream run.
set -o pipefail
OUT=gpurun_out/${1:-r03n}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/pix" -o run --output-format csv \
    -- python3 tools/pix_bench.py 1024 7995 --no-stream > "$OUT/pix.json" 2> "$OUT/pix.err" || { tail -20 "$OUT/pix.err"; exit 1; }
cat "$OUT/pix.json"
python3 tools/trace_gaps.py "$OUT/pix" "$OUT/gaps_pix.json" --from-kernel k_pix_select > /dev/null || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/zipf" -o run --output-format csv \
    -- python3 bench.py --corpus zipf --no-cpu-baseline > "$OUT/zipf.jsonl" 2> "$OUT/zipf.err" || { tail -20 "$OUT/zipf.err"; exit 1; }
head -c 1500 "$OUT/zipf.jsonl"
find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
