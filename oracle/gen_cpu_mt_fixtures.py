#!/usr/bin/env python3
"""Long-run fixtures of BASELINE configs 3 and 4 from the multi-threaded CPU restatement
(oracle/bpe_cpu_mt.cc) — TEST INFRASTRUCTURE ONLY.

The restatement is pinned to the reference's own outputs (tests/golden/*.json, every golden case,
and the reference's first three C3 merges in config3_prefix.json: tests/test_oracle_mt.py), so its
long runs stand in for the reference where the reference itself would take days (core.ts streams
1 GiB at ~1e7 pair-scans/s: one C3 merge is ~2 minutes of Node).  Generated here, in the build
container, and committed as data:

  tests/golden/config3_cpu_mt_1000.json — C3: 1 GiB, xorshift32 seed 12345, 256-char alphabet,
      1 MiB samples, mergeUntil({min_weight: 2}) for 1000 merges: the merge list, the live tokens
      after them, and the SHA-256 of the final corpus (int32 ids, little endian, samples back to
      back) with its sample offsets;
  tests/golden/config4_cpu_mt_200.json  — C4: the first 4 GiB of the same stream, 200 merges
      (the merge list and the live tokens after them);
  tests/golden/config3_cpu_mt_8000.json — C3 in full: all 8000 merges of the headline run, the
      final corpus digest, and `merges_sha256` in bench.py's form (sha256 of the (a, b, W) triples
      as int64 LE), so the bench line is checked against it;
  tests/golden/zipf_cpu_mt_2000.json — the skewed variant (bench.py --corpus zipf: 1 GiB of
      Zipf(1.1) words, seed 12345, 1 MiB samples), 2000 merges, the same fields.

Partial progress goes to <name>.partial every 500 merges (merges only).

Usage: python oracle/gen_cpu_mt_fixtures.py [c3] [c4] [c3_8000] [zipf_2000] [--threads T]
"""
import hashlib
import importlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLDEN = os.path.join(ROOT, 'tests', 'golden')
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
from oracle import CpuMT   # noqa: E402

pkg = importlib.import_module('bpe-tokenizer_amd')   # (host-side synth only: no GPU needed)

CONFIGS = {
    'c3': dict(gib=1, merges=1000, name='config3_cpu_mt_1000.json', digest=True),
    'c4': dict(gib=4, merges=200, name='config4_cpu_mt_200.json', digest=False),
    'c3_8000': dict(gib=1, merges=8000, name='config3_cpu_mt_8000.json', digest=True),
    'zipf_2000': dict(gib=1, merges=2000, name='zipf_cpu_mt_2000.json', digest=True,
                      corpus='zipf'),
}
THREADS = 0


def corpus_ids(n, corpus='uniform'):
    data = (pkg.synth_zipf(n, seed=12345) if corpus == 'zipf' else
            pkg.synth_latin1(n, seed=12345, A=256, base=0))
    lut = np.full(256, -1, np.int32)
    uniq, idx = np.unique(data[:1 << 24], return_index=True)
    order = uniq[np.argsort(idx)]
    if len(order) < 256:   # (every char appears in the first 16 MiB of this stream)
        uniq, idx = np.unique(data, return_index=True)
        order = uniq[np.argsort(idx)]
    lut[order] = np.arange(len(order), dtype=np.int32)
    return lut[data], len(order)


def gen(key):
    cfg = CONFIGS[key]
    n = cfg['gib'] << 30
    t0 = time.time()
    corpus = cfg.get('corpus', 'uniform')
    ids, nt = corpus_ids(n, corpus)
    off = np.arange(0, n + 1, 1 << 20, dtype=np.int64)
    threads = THREADS or len(os.sched_getaffinity(0))
    cpu = CpuMT(ids, off, [1] * nt, nt, threads=threads, extra=cfg['merges'] + 64)
    del ids
    merges = []
    while len(merges) < cfg['merges']:
        got = cpu.merge_until(0, 2, min(50, cfg['merges'] - len(merges)))
        if not got:
            break
        merges += got
        print('%s: %d merges, %.0f s' % (key, len(merges), time.time() - t0), flush=True)
        if len(merges) % 500 == 0:
            with open(os.path.join(GOLDEN, cfg['name'] + '.partial'), 'w') as f:
                json.dump({'merges': [list(map(int, m)) for m in merges],
                           'seconds': round(time.time() - t0, 1)}, f)
    if corpus == 'uniform':
        prefix = json.load(open(os.path.join(GOLDEN, 'config3_prefix.json')))
        assert [list(m) for m in merges[:3]] == prefix['merges'], 'CpuMT disagrees with the reference'
    out = {'config': key.upper(), 'corpus': corpus, 'bytes': n, 'seed': 12345,
           'alphabet': 256 if corpus == 'uniform' else None,
           'sample_bytes': 1 << 20, 'char_count': nt, 'min_weight': 2,
           'merges': [list(map(int, m)) for m in merges], 'live_tokens_after': int(cpu.live()),
           # (bench.py's `merges_sha256`: the (a, b, W) triples as int64 LE)
           'merges_sha256': hashlib.sha256(np.asarray(merges, dtype=np.int64).tobytes()).hexdigest(),
           'generator': 'oracle/gen_cpu_mt_fixtures.py: oracle/bpe_cpu_mt.cc on %d threads, '
                        'pinned to tests/golden/config3_prefix.json (the reference run)' % threads,
           'seconds': round(time.time() - t0, 1)}
    if cfg['digest']:
        fin, foff = cpu.read()
        out['sha256_ids_after'] = hashlib.sha256(np.ascontiguousarray(fin, '<i4').tobytes()).hexdigest()
        out['sha256_offsets_after'] = hashlib.sha256(np.ascontiguousarray(foff, '<i8').tobytes()).hexdigest()
    cpu.close()
    with open(os.path.join(GOLDEN, cfg['name']), 'w') as f:
        json.dump(out, f)
    try:
        os.remove(os.path.join(GOLDEN, cfg['name'] + '.partial'))
    except OSError:
        pass
    print('wrote', cfg['name'], out['seconds'], 's', flush=True)


if __name__ == '__main__':
    argv = sys.argv[1:]
    if '--threads' in argv:
        i = argv.index('--threads')
        THREADS = int(argv[i + 1])
        del argv[i:i + 2]
    for k in (argv or ['c3', 'c4']):
        gen(k)
