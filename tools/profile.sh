#!/bin/bash
# rocprofv3 evidence for the streaming kernel (run on the GPU box from the repo root):
#   kernel trace + stats, then PMC passes (each counter group in its own pass, no trace domains).
# Usage: tools/profile.sh OUTDIR [MiB] [steps]
set -euo pipefail
OUT=${1:-gpurun_out/prof}
MIB=${2:-1024}
STEPS=${3:-10}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # $1 = tag, rest = rocprofv3 options
    local tag=$1; shift
    timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$tag" -o run --output-format csv \
        -- python3 "$ROOT/tools/microbench.py" "$MIB" 256 "$STEPS" > "$OUT/$tag.log" 2>&1
}
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
run lds --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
echo profile done
