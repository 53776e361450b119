#!/usr/bin/env python3
"""The incremental mode (position index) against the streaming mode on BASELINE config 3:
1 GiB of the C3 stream, mergeUntil({min_weight: 2}) for N merges in each mode on a fresh copy;
prints one JSON line with both timings, the index build time and whether the merge logs and final
corpora are identical.  Usage: tools/pix_bench.py [MiB] [merges] [--no-stream]"""
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module('bpe-tokenizer_amd')


def run(data, mode, merges):
    e = pkg.Engine(0)
    e.add_latin1(data, sample_bytes=1 << 20)
    e.stats_enable(True)
    live0 = e.corpus_size()[1]
    if mode == 'incremental':
        e.set_mode('incremental')
    t0 = time.perf_counter()
    e.merge_until(0, 2, 5)                    # warmup (incremental: one index build + finish)
    t_first = time.perf_counter() - t0
    t0 = time.perf_counter()
    got = e.merge_until(0, 2, merges)
    dt = time.perf_counter() - t0
    scans, live = 0, e.corpus_size()[1] + sum(m[2] for m in got)
    for m in got:
        scans += live
        live -= m[2]
    ids, off = e.read_corpus()
    st = e.stats()
    e.close()
    st['first_call_s'] = t_first
    return got, dt, scans, ids, st


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    merges = int(sys.argv[2]) if len(sys.argv) > 2 else 7995
    data = pkg.synth_latin1(mib << 20, seed=12345, A=256, base=0)
    g1, t1, s1, i1, st1 = run(data, 'incremental', merges)
    out = {'corpus_mib': mib, 'merges': len(g1), 'incremental_s': t1,
           'incremental_ms_per_merge': 1e3 * t1 / max(1, len(g1)),
           'incremental_equiv_pair_scans_per_s': s1 / t1,
           'first_call_5_merges_s': st1['first_call_s'], 'pix_builds': st1['pix_builds'], 'pix_build_ms': st1['pix_build_ms'],
           'pix_host': st1['pix_host'], 'pix_merges': st1['pix_merges']}
    if '--no-stream' not in sys.argv:
        g2, t2, s2, i2, st2 = run(data, 'stream', merges)
        out.update({'stream_s': t2, 'stream_ms_per_merge': 1e3 * t2 / max(1, len(g2)),
                    'stream_pair_scans_per_s': s2 / t2, 'speedup': t2 / t1,
                    'identical_merges': g1 == g2, 'identical_corpus': bool(np.array_equal(i1, i2))})
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
