#!/bin/bash
# Round 3: index-build A/B (BPE_LIB builds) under kernel stats, after the incremental-mode tests.
# Usage (GPU box): tools/gpu_fx.sh TAG lib1 lib2 ...
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_incremental.py -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
for lib in "$@"; do
  n=$(basename "$lib" .so)
  BPE_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$n" -o run --output-format csv \
      -- python3 tools/pix_bench.py 1024 2000 --no-stream > "$OUT/$n.json" 2> "$OUT/$n.err" || { tail -20 "$OUT/$n.err"; exit 1; }
  python3 tools/trace_gaps.py "$OUT/$n" "$OUT/gaps_$n.json" > /dev/null || exit 1
  python3 - "$OUT/gaps_$n.json" "$OUT/$n.json" "$n" <<'PY'
import json, sys
g = json.load(open(sys.argv[1]))['kernels']; b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ks = ['k_pix_fill_x', 'k_pix_fill_y', 'k_pix_hot_count', 'k_pix_hot_fill']
print(sys.argv[3], 'build_ms %.2f' % (b.get('pix_build_ms', 0) / max(b.get('pix_builds', 1), 1)),
      ' '.join('%s %.0fus' % (k[6:], g[k]['avg_us']) for k in ks if k in g),
      'incr %.4f ms/merge' % b.get('incremental_ms_per_merge', 0))
PY
  find "$OUT/$n" -name "*kernel_trace.csv" -delete
done
