#!/usr/bin/env python3
"""Kernel-level timing of the engine on the C3 corpus: plain count passes (K1 alone) and merge
passes (fused K4+K1), from the engine's own HIP events, optionally after PRE untimed merges
(the steady state of a long run).  Usage: python tools/microbench.py [MiB] [alphabet] [steps] [PRE]

MB_SAVE=path: after the PRE merges, the corpus is saved there (npz); MB_LOAD=path: the corpus is
loaded from such a file instead of ingested and merged (the timing-probe builds cannot merge
correctly, so their "after PRE" corpus comes from the product build)."""
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
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    A = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    pre = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    e = pkg.Engine(0)
    t0 = time.perf_counter()
    if os.environ.get('MB_LOAD'):
        z = np.load(os.environ['MB_LOAD'])
        ids, off = z['ids'], z['off']
        for i in range(len(off) - 1):
            e.add_sample(ids[off[i]:off[i + 1]])
        nt = int(z['nt'])
        if e.num_tokens() < nt:   # (ids no sample holds any more: one sample registers them)
            e.add_sample(np.array([nt - 1], np.int32))
        del z, ids
        ingest = time.perf_counter() - t0
    else:
        data = pkg.synth_latin1(mib << 20, seed=12345, A=A, base=0 if A == 256 else 0x20)
        cmap, nt, _ = e.add_latin1(data, sample_bytes=1 << 20)
        ingest = time.perf_counter() - t0
        del data
        if pre:
            nt += len(e.merge_until(0, 2, pre))
        if os.environ.get('MB_SAVE'):
            ids, off = e.read_corpus()
            np.savez(os.environ['MB_SAVE'], ids=ids, off=off, nt=nt)
            del ids
    e.stats_enable(True)
    e.recount()
    e.reset_stats()
    for _ in range(5):
        e.recount()
    rc = e.stats()
    e.reset_stats()
    n_tokens = nt
    t0 = time.perf_counter()
    for _ in range(steps):
        m = e.find_next_merge(0, 2)
        if m is None:   # (a timing-probe build that counts nothing)
            break
        e.apply_merge(m[0], m[1], n_tokens)
        n_tokens += 1
    dt = time.perf_counter() - t0
    st = e.stats()
    live = rc['step_live'] / rc['step_launches']
    out = {
        'corpus_mib': mib, 'pre_merges': pre, 'ingest_s': ingest,
        'recount_ms': rc['step_ms'] / max(1, rc['step_timed']),
        'recount_GBps_alg': 4 * live / (rc['step_ms'] / max(1, rc['step_timed']) * 1e-3) / 1e9,
        'merge_pass_ms': st['step_ms'] / max(1, st['step_timed']),
        'merge_pass_GBps_alg': (4 * st['step_live'] / max(1, st['step_launches']) /
                                (st['step_ms'] / max(1, st['step_timed']) * 1e-3) / 1e9
                                if st['step_ms'] else None),
        'select_ms_per_iter': st['select_ms'] / max(1, steps),
        'wall_ms_per_iter': dt * 1e3 / max(1, steps),
        'tie_passes': st['tie_passes'], 'exact_passes': st['exact_passes'], 'compactions': st['compactions'],
    }
    print(json.dumps(out))


if __name__ == '__main__':
    main()
