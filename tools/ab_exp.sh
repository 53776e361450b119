#!/bin/bash
# A/B of libbpe builds (and engine env knobs) on the bench's device loop (C3, N merges, no CPU
# baseline, no incremental-mode line).
# Usage (GPU box): tools/ab_exp.sh TAG STEPS spec1 spec2 ...   with spec = lib[:VAR=value[,VAR=value]]
# (AB_EXTRA: more bench.py flags, e.g. "--corpus zipf"; AB_REPS: runs per spec, interleaved)
set -eo pipefail
OUT=gpurun_out/$1; STEPS=$2; shift 2
mkdir -p "$OUT"
for rep in $(seq 1 ${AB_REPS:-1}); do
for spec in "$@"; do
  lib=${spec%%:*}
  envs=""
  [[ "$spec" == *:* ]] && envs=${spec#*:}
  name=$(basename "$lib" .so)${envs:+_${envs//[=,]/_}}_$rep
  env BPE_LIB=$lib ${envs//,/ } timeout -k 10 300 python3 bench.py --steps $STEPS --no-cpu-baseline $AB_EXTRA > "$OUT/$name.json"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; b=d['breakdown_ms_per_step']; print(sys.argv[2], 'ms/step %.4f k_step %.4f frac %.3f value %.4g compactions %d sha %s' % (d['ms_per_step'], r['kernel_avg_ms'], r['frac'], d['value'], b['compactions'], d['merges_sha256'][:12]))" "$OUT/$name.json" "$name"
done
done
