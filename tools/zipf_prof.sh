#!/bin/bash
# rocprofv3 kernel stats + FETCH/WRITE + SQ passes of the skewed-corpus bench (zipf C3).
# GPU box, repo root.  Usage: tools/zipf_prof.sh TAG [steps]
set -eo pipefail
OUT=gpurun_out/$1; STEPS=${2:-7995}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 bench.py --corpus zipf --steps $STEPS --no-cpu-baseline > "$OUT/trace.log" 2>&1
find "$OUT/trace" -name '*kernel_stats.csv' -exec head -16 {} \;
PMC="bench.py --corpus zipf --steps 600 --warmup 2000 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 $PMC > "$OUT/fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 $PMC > "$OUT/write.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    -d "$OUT/sq" -o run --output-format csv -- python3 $PMC > "$OUT/sq.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM \
    -d "$OUT/sq2" -o run --output-format csv -- python3 $PMC > "$OUT/sq2.log" 2>&1
python3 tools/sq_loop_summary.py "$OUT" > "$OUT/sq_summary.txt"
python3 tools/pmc_summary.py "$OUT" "$OUT/summary.json" "k_step_loop<4>" > /dev/null
# keep the merged-back output small (the raw per-dispatch CSVs are tens of MB)
find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
cat "$OUT/sq_summary.txt"
