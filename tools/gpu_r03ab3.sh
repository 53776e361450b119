#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r03ab3}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_sharded_gpu.py tests/test_multi_device.py -m gpu -k "loop or rank or shard or multi or golden or config" -v --maxfail=3 \
    --timeout 300 --timeout-method thread > "$OUT/loop.log" 2>&1 || { tail -30 "$OUT/loop.log"; exit 1; }
tail -1 "$OUT/loop.log"
bash tools/ab_exp.sh ${1:-r03ab3}/ab 3000 gpurun_exp/base.so bpe-tokenizer_amd/libbpe.so gpurun_exp/base.so bpe-tokenizer_amd/libbpe.so || exit 1
bash tools/gpu_zsel.sh ${1:-r03ab3}/zsel
