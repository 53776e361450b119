#!/bin/bash
# Round 3: kernel-boundary gaps of the device loop (kernel trace), the incremental mode's index
# build time, the host-copy exchange cost over 8 shards.
set -o pipefail
OUT=gpurun_out/${1:-r03k}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
python3 tools/trace_gaps.py "$OUT/trace" "$OUT/gaps.json" --from-kernel k_step_loop || exit 1
timeout -k 10 300 python3 bench.py --incremental --no-cpu-baseline > "$OUT/bench_inc.jsonl" 2> "$OUT/bench_inc.err" || { tail "$OUT/bench_inc.err"; exit 1; }
tail -1 "$OUT/bench_inc.jsonl"
timeout -k 10 400 python3 -u tools/multi_overhead.py 512 8 300 "$OUT/multi_overhead.json" > "$OUT/multi.log" 2>&1
echo "multi rc=$?"; tail -5 "$OUT/multi.log"
find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
