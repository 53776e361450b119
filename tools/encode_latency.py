#!/usr/bin/env python3
"""Latency of ONE text per bpe_encode_batch call (the JS drop-in's encodeToCode shape): for
merge lists of several lengths (mergeUntil on a zipf word corpus) and texts of several lengths,
the wall time per call and the kernel time (HIP events) per call, with the greedy steps taken.
Prints one JSON object.  Usage: tools/encode_latency.py [--reps 50]"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module('bpe-tokenizer_amd')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=50)
    ap.add_argument('--mib', type=int, default=64)
    a = ap.parse_args()
    n = a.mib << 20
    data = pkg.synth_zipf(n + (1 << 20), seed=12345)
    e = pkg.Engine(0)
    cmap, n_tok, _ = e.add_latin1(data[:n], sample_bytes=1 << 20)
    e.set_mode('incremental')
    got = e.merge_until(0, 2, 8000)
    e.close()
    allm = np.asarray([(x, y, n_tok + k) for k, (x, y, _w) in enumerate(got)], np.int32)
    rest = cmap[data[n:]]
    rest = rest[rest >= 0].astype(np.int32)
    rows = []
    for m in (16, 128, 1024, 4096, 8000):
        enc = pkg.Encoder(0, allm[:m])
        for chars in (16, 64, 256, 1024, 4096, 16384):
            t = rest[:chars]
            enc.encode([t])
            enc.reset_stats()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                enc.encode([t])
            dt = (time.perf_counter() - t0) / a.reps
            st = enc.stats()
            rows.append({'merges': m, 'chars': chars, 'call_us': dt * 1e6,
                         'kernel_us': st['kernel_ms'] * 1e3 / a.reps,
                         'steps': st['steps'] / a.reps, 'out_len': st['tokens_out'] // a.reps})
        enc.close()
    print(json.dumps({'what': 'one text per bpe_encode_batch call (zipf-trained merges)', 'rows': rows}))


if __name__ == '__main__':
    main()
