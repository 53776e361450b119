#!/bin/bash
# Time breakdown of the streaming pass on C3 from timing-probe builds of libbpe (gpurun_exp/):
# nocount (ring + apply, no counting), noapply (ring + count, no merge detection), none (ring
# and bookkeeping only), against the product build.  tools/microbench.py: plain count pass and
# merge pass, at the start of the run and after PRE merges.
set -eo pipefail
OUT=gpurun_out/${1:-probe}; PRE=${2:-1000}
mkdir -p "$OUT"
for lib in bpe-tokenizer_amd/libbpe.so gpurun_exp/nocount.so gpurun_exp/noapply.so gpurun_exp/none.so; do
  n=$(basename $lib .so)
  BPE_LIB=$lib timeout -k 10 120 python3 tools/microbench.py 1024 256 20 0 > "$OUT/$n.0.json"
  if [ "$n" = libbpe ]; then
    MB_SAVE=/tmp/mb_pre.npz BPE_LIB=$lib timeout -k 10 180 python3 tools/microbench.py 1024 256 20 $PRE > "$OUT/$n.$PRE.json"
  else
    MB_LOAD=/tmp/mb_pre.npz BPE_LIB=$lib timeout -k 10 180 python3 tools/microbench.py 1024 256 20 $PRE > "$OUT/$n.$PRE.json"
  fi
  echo "$n: $(cat $OUT/$n.0.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print("recount %.4f merge %.4f" % (d["recount_ms"], d["merge_pass_ms"]))') | after $PRE: $(cat $OUT/$n.$PRE.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print("recount %.4f merge %.4f" % (d["recount_ms"], d["merge_pass_ms"]))')"
done
