#!/bin/bash
# Round-3 targeted GPU check: the incremental mode (hand-written index build), the sharded rank
# loop's maintained state, then smoke + the driver's bench command + the full bench + rocprof.
set -eo pipefail
OUT=gpurun_out/${1:-r03c}
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests/test_incremental.py tests/test_gpu_parity.py tests/test_sharded_gpu.py \
    tests/test_scale_configs.py tests/test_multi_device.py -m gpu -v --maxfail=3 --timeout 170 --timeout-method thread \
    -k "pix or incremental or sharded_gpu or config3 or maintained or rank_loop" > "$OUT/pytest.log" 2>&1 \
    || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
tools/gpu_round3.sh "${1:-r03c}" smoke driver bench prof
