#!/bin/bash
# Quick GPU check after a kernel change: GPU parity tests, then microbench at the start of C3 and
# after PRE merges, then (optional) SQ counters.  Usage: tools/gpu_quick.sh TAG [PRE] [sq]
set -eo pipefail
TAG=${1:-q}; PRE=${2:-1000}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 120 python3 tools/microbench.py 1024 256 20 0
timeout -k 10 120 python3 tools/microbench.py 1024 256 20 "$PRE"
if [ "$3" == "sq" ]; then
  tools/profile_sq.sh "$OUT/sq0" 1024 10 0 && tools/profile_sq.sh "$OUT/sqp" 1024 10 "$PRE"
  python3 tools/sq_summary.py "$OUT/sq0" | grep "k_step"
  python3 tools/sq_summary.py "$OUT/sqp" | grep "k_step<1"
fi
