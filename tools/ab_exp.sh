#!/bin/bash
# A/B of libbpe builds on the bench's device loop (C3, N merges, no CPU baseline).
# Usage (GPU box): tools/ab_exp.sh TAG STEPS lib1 lib2 ...
set -eo pipefail
OUT=gpurun_out/$1; STEPS=$2; shift 2
mkdir -p "$OUT"
for lib in "$@"; do
  BPE_LIB=$lib timeout -k 10 200 python3 bench.py --steps $STEPS --no-cpu-baseline > "$OUT/$(basename $lib).json"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], 'ms/step %.4f k_step %.4f frac %.3f value %.4g' % (d['ms_per_step'], r['kernel_avg_ms'], r['frac'], d['value']))" "$OUT/$(basename $lib).json"
done
