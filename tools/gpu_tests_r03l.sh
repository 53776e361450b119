#!/bin/bash
# Round 3: grid tickets (k_tie_fused decides in block 0 without a tie; hierarchical last-block
# counters; k_select_maint's gather by the whole last block): parity, C3 and zipf traces.
set -o pipefail
OUT=gpurun_out/${1:-r03l}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_incremental.py -m gpu -v --maxfail=3 \
    --timeout 170 --timeout-method thread -k "loop or zipf or cold or tie" > "$OUT/loop.log" 2>&1 \
    || { tail -30 "$OUT/loop.log"; exit 1; }
tail -1 "$OUT/loop.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 bench.py --steps 1000 --warmup 5 --no-cpu-baseline > "$OUT/c3.jsonl" 2> "$OUT/c3.err" || { tail -20 "$OUT/c3.err"; exit 1; }
python3 tools/trace_gaps.py "$OUT/trace" "$OUT/gaps_c3.json" --from-kernel k_step_loop || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/tracez" -o run --output-format csv \
    -- python3 bench.py --corpus zipf --steps 2000 --warmup 5 --no-cpu-baseline > "$OUT/zipf.jsonl" 2> "$OUT/zipf.err" || { tail -20 "$OUT/zipf.err"; exit 1; }
python3 tools/trace_gaps.py "$OUT/tracez" "$OUT/gaps_zipf.json" --from-kernel k_step_loop || exit 1
python3 -c "import json; [print(k, json.loads(l).get('ms_per_step'), json.loads(l).get('breakdown_ms_per_step')) for k in ('c3','zipf') for l in open('$OUT/'+k+'.jsonl')]"
timeout -k 10 400 python3 -u tools/multi_overhead.py 512 8 300 "$OUT/multi_overhead.json" > "$OUT/multi.log" 2>&1
echo "multi rc=$?"; tail -3 "$OUT/multi.log"
find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
