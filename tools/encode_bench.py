#!/usr/bin/env python3
"""Throughput of the device encoder (bpe_encode_batch, csrc/bpe_encode.hip): encodeToCode
(core.ts:392-409) of a batch of short texts with a trained merge list.

The merges: mergeUntil({min_weight: 2, max_iterations: M}) on MiB of a synthetic corpus (the
incremental mode, identical merges to the streaming one).  The texts: a later, disjoint stretch of
the same stream cut into texts of random length in [min, max] chars.  Prints one JSON line:
kernel time (HIP events around the launches), end-to-end time of the call (host packing, copies,
kernels, unpacking), input tokens/s for both, the greedy steps taken, and two CPU legs:
  - cpu_baseline: the same rank-greedy algorithm on the host's cores (oracle/bpe_cpu_encode.cc,
    bench.encode_cpu_baseline) over every text of the batch, whose outputs must equal the device's;
  - cpu_replay: the reference's own algorithm (oracle_encode: every merge in order over each text,
    core.ts:404-406) on a bounded sample, one thread, also checked against the device.

Usage: tools/encode_bench.py [--corpus uniform|zipf] [--mib 256] [--merges 8000] [--texts 100000]
                             [--min 16] [--max 1024] [--reps 5]
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
pkg = importlib.import_module('bpe-tokenizer_amd')
from bench import encode_cpu_baseline   # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--corpus', default='uniform')
    ap.add_argument('--mib', type=int, default=256)
    ap.add_argument('--merges', type=int, default=8000)
    ap.add_argument('--texts', type=int, default=100000)
    ap.add_argument('--min', type=int, default=16)
    ap.add_argument('--max', type=int, default=1024)
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--cpu-texts', type=int, default=200)
    a = ap.parse_args()

    n = a.mib << 20
    rng = np.random.default_rng(5)
    lens = rng.integers(a.min, a.max + 1, size=a.texts)
    need = int(lens.sum())
    if a.corpus == 'zipf':
        data = pkg.synth_zipf(n + need, seed=12345)
        train, rest = data[:n], data[n:n + need]
    else:
        train = pkg.synth_latin1(n, seed=12345, A=256)
        rest = pkg.synth_latin1(need, seed=12345, A=256, skip=n)
    e = pkg.Engine(0)
    cmap, n_tok, _ = e.add_latin1(train, sample_bytes=1 << 20)
    e.set_mode('incremental')
    t0 = time.perf_counter()
    got = e.merge_until(0, 2, a.merges)
    t_train = time.perf_counter() - t0
    e.close()
    merges = np.asarray([(x, y, n_tok + k) for k, (x, y, _w) in enumerate(got)], np.int32)
    # texts: chars -> ids through the training map (chars unseen in training are dropped)
    ids = cmap[rest]
    ids = ids[ids >= 0].astype(np.int32)
    off = np.zeros(a.texts + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    off = np.minimum(off, ids.size)

    enc = pkg.Encoder(0, merges)
    enc.encode_flat(ids, off)                      # warmup (table upload, code load)
    enc.reset_stats()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        out, oo = enc.encode_flat(ids, off)
    e2e = (time.perf_counter() - t0) / a.reps
    st = enc.stats()
    kern = st['kernel_ms'] / a.reps / 1e3

    # CPU replay on a bounded sample (the reference's algorithm: M rewrites per text)
    import oracle
    k = min(a.cpu_texts, a.texts)
    sample = [ids[off[i]:off[i + 1]] for i in range(k)]
    t0 = time.perf_counter()
    want = oracle.encode(sample, merges)
    t_cpu = time.perf_counter() - t0
    same = all(np.array_equal(w, out[oo[i]:oo[i + 1]]) for i, w in enumerate(want))
    tok_sample = int(off[k] - off[0])
    res = {
        'what': 'encodeToCode of a batch of short texts on the device merge-rank encoder',
        'corpus': a.corpus, 'train_mib': a.mib, 'merges': int(len(merges)), 'train_s': t_train,
        'texts': a.texts, 'text_chars': [a.min, a.max], 'tokens_in': int(off[-1]),
        'tokens_out': int(oo[-1]), 'steps_per_text': st['steps'] / a.reps / a.texts,
        'texts_rank': st['texts_rank'] // a.reps, 'texts_replay': st['texts_replay'] // a.reps,
        'kernel_ms': kern * 1e3, 'e2e_ms': e2e * 1e3,
        'kernel_tokens_per_s': off[-1] / kern, 'e2e_tokens_per_s': off[-1] / e2e,
        'cpu_replay': {'kind': 'port', 'cores': 1, 'texts': k, 'tokens': tok_sample, 's': t_cpu,
                       'tokens_per_s': tok_sample / t_cpu,
                       'what': 'oracle_encode (oracle/bpe_oracle.c): every merge in order, core.ts:404-406'},
        'identical_on_cpu_sample': bool(same),
        'cpu_baseline': encode_cpu_baseline(ids, off, merges, out, oo),
    }
    enc.close()
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
