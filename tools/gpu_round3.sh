#!/bin/bash
# One GPU-box pass of round 3.  Usage (repo root, on the GPU box): tools/gpu_round3.sh TAG [what...]
#   what ∈ tests smoke driver bench prof pmc sq pixab slow
#   driver: the driver's exact bench command (python3 bench.py --gpus 1 --steps 20 --warmup 5)
#   pixab:  the incremental mode's parity tests on the -structurizecfg-skip-uniform-regions build
set -eo pipefail
TAG=${1:-r03}; shift || true
WHAT=${*:-tests smoke driver bench prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
has() { [[ " $WHAT " == *" $1 "* ]]; }
if has tests; then
  timeout -k 10 1100 python3 -u -m pytest tests -m gpu -v --maxfail=5 --timeout 400 ${PYTEST_EXTRA} \
      --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu.log"
fi
if has smoke; then
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  cat "$OUT/smoke.log"
fi
if has driver; then
  t0=$(date +%s.%N)
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver.jsonl" 2> "$OUT/driver.err"
  t1=$(date +%s.%N)
  cat "$OUT/driver.jsonl"; echo "driver wall: $(python3 -c "print('%.1f s' % ($t1 - $t0))")" | tee "$OUT/driver.wall"
fi
if has bench; then
  timeout -k 10 600 python3 bench.py --incremental > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
  cat "$OUT/bench.jsonl"
fi
if has prof; then
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
      -- python3 bench.py --no-cpu-baseline > "$OUT/trace.log" 2>&1
  find "$OUT/trace" -name '*kernel_stats.csv' -exec head -14 {} \;
fi
PMC_BENCH="bench.py --steps 300 --warmup 5 --no-cpu-baseline"
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
if has pixab; then
  BPE_LIB=gpurun_exp/sk.so timeout -k 10 600 python3 -u -m pytest tests/test_incremental.py tests/test_gpu_parity.py \
      -m gpu -k "pix or incremental" -v --timeout 300 --timeout-method thread > "$OUT/pixab.log" 2>&1 \
      || { tail -40 "$OUT/pixab.log"; exit 1; }
  tail -3 "$OUT/pixab.log"
fi
# keep the merged-back output small (the raw per-dispatch CSVs are tens of MB)
find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
