#!/usr/bin/env python3
"""Does the merge pass run slower in the first milliseconds of GPU work (clock ramp) than later on
the same corpus?  C3 (1 GiB, 256-char alphabet), merges timed one call each (host clock around a
synchronous merge_until of one merge), after an optional heat phase of plain count passes
(bpe_recount, no merge: the corpus is unchanged).
Usage: tools/warm_probe.py HEAT_MS [N_SINGLE] [N_BATCH]"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

heat_ms = float(sys.argv[1]) if len(sys.argv) > 1 else 0.0
n_single = int(sys.argv[2]) if len(sys.argv) > 2 else 40
n_batch = int(sys.argv[3]) if len(sys.argv) > 3 else 400

import torch  # noqa: E402  (the HIP runtime first, as bench.py)

pkg = importlib.import_module('bpe-tokenizer_amd')
torch.cuda.set_device(0)
data = pkg.synth_latin1(1 << 30, seed=12345, A=256, base=0)
e = pkg.Engine(0)
e.add_latin1(data, sample_bytes=1 << 20)
del data
e.recount()
heat_passes = 0
t0 = time.perf_counter()
while (time.perf_counter() - t0) * 1e3 < heat_ms:
    e.recount()
    heat_passes += 1
torch.cuda.synchronize()
single = []
for _ in range(n_single):
    t = time.perf_counter()
    e.merge_until(0, 2, 1)
    single.append((time.perf_counter() - t) * 1e3)
t = time.perf_counter()
got = e.merge_until(0, 2, n_batch)
batch_ms = (time.perf_counter() - t) * 1e3 / max(1, len(got))
single2 = []
for _ in range(n_single):
    t = time.perf_counter()
    e.merge_until(0, 2, 1)
    single2.append((time.perf_counter() - t) * 1e3)
e.close()
print(json.dumps({'heat_ms': heat_ms, 'heat_passes': heat_passes,
                  'single_ms_first': [round(x, 4) for x in single],
                  'batch_ms_per_merge': batch_ms, 'batch_merges': len(got),
                  'single_ms_after': [round(x, 4) for x in single2]}), flush=True)
