#!/usr/bin/env python3
"""mergeUntil through the C ABI (ctypes) on the same corpus as tools/bench_js.js, for comparison
with the drop-in: MiB of xorshift32 latin1 (seed 12345, 256-char alphabet, 1 MiB samples).
Usage: tools/loop_bench.py [MiB=64] [merges=1000] [warmup=5]"""
import importlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module('bpe-tokenizer_amd')

mib, merges, warmup = (int(a) for a in (sys.argv[1:] + ['64', '1000', '5'][len(sys.argv) - 1:])[:3])
e = pkg.Engine(0)
e.add_latin1(pkg.synth_latin1(mib << 20, seed=12345, A=256), sample_bytes=1 << 20)
e.merge_until(0, 2, warmup)
live = e.corpus_size()[1]
t0 = time.perf_counter()
ms = e.merge_until(0, 2, merges)
dt = time.perf_counter() - t0
scans = 0
for m in ms:
    scans += live
    live -= m[2]
print(json.dumps({'what': 'C ABI bpe_merge_until (ctypes)', 'corpus_mib': mib, 'merges': len(ms),
                  'seconds': dt, 'ms_per_merge': 1e3 * dt / len(ms), 'pair_scans_per_s': scans / dt}))
