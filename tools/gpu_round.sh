#!/bin/bash
# One GPU-box pass: gpu parity tests, smoke, the default bench line, rocprofv3 kernel-trace stats
# of the same bench command, and FETCH_SIZE / WRITE_SIZE passes (separate runs, no trace domains).
# Usage (repo root, on the GPU box): tools/gpu_round.sh TAG [what...]   what ∈ tests smoke bench prof pmc
set -eo pipefail
TAG=${1:-r01}; shift || true
WHAT=${*:-tests smoke bench prof pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
has() { [[ " $WHAT " == *" $1 "* ]]; }
if has tests; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
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
BENCH="bench.py"   # the driver's default bench command, profiled as is
if has prof; then
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
      -- python3 $BENCH > "$OUT/trace.log" 2>&1
  find "$OUT/trace" -name '*kernel_stats.csv' -exec cat {} \;
fi
# counters per launch of the same kernel on a shorter run of the same bench (each counted dispatch
# is serialised, so the full 8000-merge run would take minutes per pass)
PMC_BENCH="bench.py --steps 500 --warmup 5 --no-cpu-baseline"
if has pmc; then
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
      -- python3 $PMC_BENCH > "$OUT/fetch.log" 2>&1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
      -- python3 $PMC_BENCH > "$OUT/write.log" 2>&1
  echo pmc done
fi
python3 tools/pmc_summary.py "$OUT" "$OUT/summary.json" > /dev/null && echo summary written
