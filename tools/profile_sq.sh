#!/bin/bash
# Per-kernel instruction mix of the streaming pass: kernel trace + SQ / LDS / TA counter passes
# (each its own run, no trace domains), on tools/microbench.py.  GPU box, repo root.
# Usage: tools/profile_sq.sh OUTDIR [MiB] [steps] [pre-merges]   (BPE_LIB selects another build)
set -eo pipefail
OUT=${1:-gpurun_out/sq}
MIB=${2:-1024}
STEPS=${3:-10}
PRE=${4:-0}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
MB="$ROOT/tools/microbench.py $MIB 256 $STEPS $PRE"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 $MB > "$OUT/trace.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD \
    -d "$OUT/sq" -o run --output-format csv -- python3 $MB > "$OUT/sq.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES \
    -d "$OUT/lds" -o run --output-format csv -- python3 $MB > "$OUT/lds.log" 2>&1
echo done
