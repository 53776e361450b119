#!/bin/bash
# device-loop parity tests, then the C3 bench A/B line (2500 merges, twice)
set -o pipefail
OUT=gpurun_out/${1:-r03loop}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_scale_configs.py tests/test_incremental.py -m gpu -v --maxfail=3 \
    --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { grep -E 'FAILED|Error' "$OUT/tests.log" | head; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
bash tools/ab_exp.sh ${1:-r03loop}/ab 2500 bpe-tokenizer_amd/libbpe.so bpe-tokenizer_amd/libbpe.so
