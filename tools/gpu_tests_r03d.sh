#!/bin/bash
set -eo pipefail
OUT=gpurun_out/${1:-r03d}
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests/test_sharded_gpu.py tests/test_scale_configs.py -m gpu -v --maxfail=3 \
    --timeout 170 --timeout-method thread -k "maintained or config4" > "$OUT/pytest.log" 2>&1 \
    || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
tools/probe_breakdown.sh "${1:-r03d}/probe" 1000
tools/gpu_round3.sh "${1:-r03d}" smoke driver bench prof
