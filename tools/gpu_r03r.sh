#!/bin/bash
# Round 3: full GPU suite on the current build, A/B of the streaming pass against the HEAD build
# (gpurun_exp/base.so), and the zipf selection probe.
set -o pipefail
OUT=gpurun_out/${1:-r03r}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --maxfail=5 --timeout 400 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { grep -E 'FAILED|Error|error' "$OUT/pytest_gpu.log" | head -30; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
bash tools/ab_exp.sh ${1:-r03r}/ab 3000 gpurun_exp/base.so bpe-tokenizer_amd/libbpe.so gpurun_exp/base.so bpe-tokenizer_amd/libbpe.so || exit 1
timeout -k 10 200 python3 tools/zipf_sel.py 1024 2000 2000 > "$OUT/zsel.json" 2>&1 || { cat "$OUT/zsel.json"; exit 1; }
cat "$OUT/zsel.json"
