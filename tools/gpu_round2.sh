#!/bin/bash
# One GPU-box pass of round 2: GPU parity tests, smoke, the default bench line, the rocprofv3
# kernel-trace stats of the same bench command, FETCH_SIZE / WRITE_SIZE and two SQ counter passes
# (each its own run, no trace domains), the JS drop-in bench.
# Usage (repo root, on the GPU box): tools/gpu_round2.sh TAG [what...]
#   what ∈ tests smoke bench prof pmc sq js
set -eo pipefail
TAG=${1:-r02}; shift || true
WHAT=${*:-tests smoke bench prof pmc sq js}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
has() { [[ " $WHAT " == *" $1 "* ]]; }
if has tests; then
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --maxfail=5 --timeout 400 \
      --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu.log"
fi
if has smoke; then
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  cat "$OUT/smoke.log"
fi
if has bench; then
  timeout -k 10 600 python3 bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
  cat "$OUT/bench.jsonl"
fi
if has prof; then
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
      -- python3 bench.py > "$OUT/trace.log" 2>&1
  find "$OUT/trace" -name '*kernel_stats.csv' -exec head -12 {} \;
fi
PMC_BENCH="bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-incremental"
if has pmc; then
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
      -- python3 $PMC_BENCH > "$OUT/fetch.log" 2>&1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
      -- python3 $PMC_BENCH > "$OUT/write.log" 2>&1
  python3 tools/pmc_summary.py "$OUT" "$OUT/summary.json" > /dev/null && echo pmc summary written
fi
if has sq; then
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
      -d "$OUT/sq" -o run --output-format csv -- python3 $PMC_BENCH > "$OUT/sq.log" 2>&1
  timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM \
      -d "$OUT/sq2" -o run --output-format csv -- python3 $PMC_BENCH > "$OUT/sq2.log" 2>&1
  python3 tools/sq_loop_summary.py "$OUT" > "$OUT/sq_summary.txt" && cat "$OUT/sq_summary.txt"
fi
if has js; then
  timeout -k 10 300 node tools/bench_js.js 64 1000 5 > "$OUT/bench_js.json" 2> "$OUT/bench_js.err"
  cat "$OUT/bench_js.json"
  timeout -k 10 300 python3 tools/loop_bench.py 64 1000 5 > "$OUT/bench_py64.json"
  cat "$OUT/bench_py64.json"
fi
# keep the merged-back output small (the raw per-dispatch CSVs are tens of MB)
find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
