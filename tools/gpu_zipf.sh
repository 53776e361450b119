#!/bin/bash
# GPU tests, then the zipf bench under rocprofv3 kernel stats.  Usage: tools/gpu_zipf.sh TAG [notest]
set -eo pipefail
TAG=${1:-zp}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ "$2" != notest ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 bench.py --corpus zipf --no-cpu-baseline > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
find "$OUT/trace" -name '*kernel_stats.csv' -exec cp {} "$OUT/kstats.csv" \;
python3 tools/ktrace_buckets.py "$(find "$OUT/trace" -name "*kernel_trace.csv" | head -1)" 1000 6 || true
rm -f "$OUT"/trace/*kernel_trace.csv
python3 tools/kstats.py "$OUT/kstats.csv" "$OUT/bench.jsonl"
