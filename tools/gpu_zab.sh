#!/bin/bash
# zipf selection/pass A/B: tools/zipf_sel.py on two libraries, twice each
set -o pipefail
OUT=gpurun_out/${1:-zab}; A=$2; B=$3
mkdir -p "$OUT"
for rep in 1 2; do
  for lib in $A $B; do
    n=$(basename $lib .so)
    BPE_LIB=$lib timeout -k 10 200 python3 tools/zipf_sel.py 1024 2000 2000 > "$OUT/$n.$rep.json" 2>&1 || { cat "$OUT/$n.$rep.json"; exit 1; }
    echo "$n $rep $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('ms/merge %.4f hash %d' % (d['ms_per_merge'], d['merges_hash']))" "$OUT/$n.$rep.json")"
  done
done
