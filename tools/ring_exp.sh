#!/bin/bash
# Ring-depth experiment: the default build and build/libbpe_r*.so on the bench's device loop
# (3000 merges of C3, no CPU baseline), plus the streaming probe.  GPU box, repo root.
set -eo pipefail
OUT=gpurun_out/${1:-ring}
mkdir -p "$OUT"
timeout -k 10 120 tools/probe/stream_probe > "$OUT/probe.txt" 2>&1 && cat "$OUT/probe.txt"
for lib in bpe-tokenizer_amd/libbpe.so build/libbpe_r9.so build/libbpe_r11.so; do
  BPE_LIB=$lib timeout -k 10 200 python3 bench.py --steps 3000 --no-cpu-baseline > "$OUT/$(basename $lib).json"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], 'ms/step %.4f k_step %.4f frac %.3f' % (d['ms_per_step'], r['kernel_avg_ms'], r['frac']))" "$OUT/$(basename $lib).json"
done
