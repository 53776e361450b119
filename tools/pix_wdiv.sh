#!/bin/bash
# The incremental mode's heavy-merge threshold (BPE_PIX_WDIV: merges with W > n_live / WDIV go to
# the stream before the index is built) on the skewed corpus: one bench line per divisor.
# Usage (GPU box, repo root): tools/pix_wdiv.sh TAG div1 div2 ...
set -eo pipefail
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for d in "$@"; do
  BPE_PIX_WDIV=$d timeout -k 10 300 python3 bench.py --corpus zipf --no-cpu-baseline > "$OUT/zipf_wdiv$d.json"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); i=d['incremental_mode']; print(sys.argv[2], 'stream ms/step %.4f  incremental ms/step %.4f builds %d on_index %d host %d same %s' % (d['ms_per_step'], i['ms_per_step'], i['index_builds'], i['merges_on_index'], i['handed_to_stream'], i['identical_merges_to_stream']))" "$OUT/zipf_wdiv$d.json" "$d"
done
