#!/bin/bash
# Skewed-corpus (zipf C3) A/B of libbpe builds: bench line per build.  GPU box, repo root.
# Usage: tools/zipf_ab.sh TAG STEPS lib1 lib2 ...
set -eo pipefail
OUT=gpurun_out/$1; STEPS=$2; shift 2
mkdir -p "$OUT"
for lib in "$@"; do
  BPE_LIB=$lib timeout -k 10 300 python3 bench.py --corpus zipf --steps $STEPS --no-cpu-baseline > "$OUT/zipf_$(basename $lib).json"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; b=d['breakdown_ms_per_step']; print(sys.argv[1], 'ms/step %.4f k_step %.4f value %.4g exact %s' % (d['ms_per_step'], r['kernel_avg_ms'], d['value'], b['exact_passes']))" "$OUT/zipf_$(basename $lib).json"
done
