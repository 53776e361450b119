#!/bin/bash
# Quick per-kernel instruction mix: kernel trace + one SQ counter pass (GPU box, repo root).
# Usage: tools/profile_sq.sh OUTDIR [MiB] [steps]   (BPE_LIB selects an experimental build)
set -euo pipefail
OUT=${1:-gpurun_out/sq}
MIB=${2:-1024}
STEPS=${3:-10}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 "$ROOT/tools/microbench.py" "$MIB" 256 "$STEPS" > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD \
    -d "$OUT/sq" -o run --output-format csv \
    -- python3 "$ROOT/tools/microbench.py" "$MIB" 256 "$STEPS" > "$OUT/sq.log" 2>&1
echo done
