#!/bin/bash
# The maintained-state tests first (diagnostics), then the full GPU suite, the timing probes and
# the bench line.
set -eo pipefail
OUT=gpurun_out/${1:-r03f}
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests/test_multi_device.py tests/test_sharded_gpu.py -m gpu -v \
    --timeout 170 --timeout-method thread -k "maintained" > "$OUT/maint.log" 2>&1 || true
tail -6 "$OUT/maint.log"; grep -h "BpeError\|RuntimeError" "$OUT/maint.log" | sort | uniq | head -5 || true
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --maxfail=5 --timeout 170 --timeout-method thread \
    --deselect tests/test_sharded_gpu.py::test_rank_loop_maintained_state_on_zipf_words \
    --deselect tests/test_sharded_gpu.py::test_rank_loop_maintained_state_three_ranks_max_length \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
tools/probe_breakdown.sh "${1:-r03f}/probe" 1000
tools/gpu_round3.sh "${1:-r03f}" smoke driver bench
