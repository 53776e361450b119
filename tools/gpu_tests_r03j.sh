#!/bin/bash
# Round 3: the sharded paths after the exchange-buffer fix (poisoned buffers).
set -o pipefail
OUT=gpurun_out/${1:-r03j}
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests/test_multi_device.py tests/test_sharded_gpu.py -m gpu -v \
    --maxfail=3 --timeout 170 --timeout-method thread > "$OUT/sharded.log" 2>&1
rc=$?; echo "sharded rc=$rc"; grep -h "PASS\|FAIL\|Error\|passed\|failed" "$OUT/sharded.log" | tail -45
exit $rc
