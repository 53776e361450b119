#!/usr/bin/env python3
"""BASELINE config 5 at its full size on one device: the 16 GiB C5 stream (256-char alphabet,
seed 12345) over 8 shards sharing device 0 (the drop-in's BPE_DEVICES path, exchanged by a device
kernel), taken to the 32k-token vocabulary in the default mode (the streaming rank loop, then the
incremental mode past 18432 ids when the shards' indexes fit beside their corpora, else the
stream on).  Prints a JSON line per chunk of merges (time, ms/merge, mode counters, exchange
bytes), then the checks: tokens conserved (live == n - sum of the replacements), and the final
state's next merge against a recount from scratch of the corpus read back from HBM by the
threaded CPU restatement (oracle/bpe_cpu_mt.cc, test infrastructure: the checker only).  The
first merges of the same stream are pinned against the restatement by
tests/test_scale_configs.py::test_config5_eight_shards_vs_one_context_and_cpu_restatement.
Usage: python tools/c5_full.py [GiB] [shards] [chunk]"""
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))


def main():
    gib = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    shards = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    chunk = int(sys.argv[3]) if len(sys.argv) > 3 else 2048
    pkg = importlib.import_module('bpe-tokenizer_amd')
    n = gib << 30
    t0 = time.perf_counter()
    data = pkg.synth_latin1(n, seed=12345, A=256, base=0)
    e = pkg.Engine(devices=[0] * shards, reduce='host')
    _, nt, _ = e.add_latin1(data, sample_bytes=1 << 20)
    del data
    e.stats_enable(True)
    print(json.dumps({'corpus_gib': gib, 'shards': shards, 'tokens': nt,
                      'setup_s': round(time.perf_counter() - t0, 1)}), flush=True)
    total = 32768 - nt
    merges = []
    prev = (0, 0)
    t_all = time.perf_counter()
    while len(merges) < total:
        k = min(chunk, total - len(merges))
        t1 = time.perf_counter()
        got = e.merge_until(0, 2, k)
        dt = time.perf_counter() - t1
        merges += got
        st = e.stats()
        dx, di = st['xchg_bytes'] - prev[0], st['xchg_iters'] - prev[1]
        prev = (st['xchg_bytes'], st['xchg_iters'])
        print(json.dumps({'merges': len(merges), 'chunk_s': round(dt, 2),
                          'ms_per_merge': round(dt * 1e3 / max(1, len(got)), 4),
                          'last_w': got[-1][2] if got else None, 'pix_merges': st['pix_merges'],
                          'pix_builds': st['pix_builds'], 'pix_fallbacks': st['pix_fallbacks'],
                          'loop_host': st['loop_host'], 'fused_passes': st['fused_passes'],
                          'xchg_bytes_per_iter': round(dx / shards / max(1, di))}), flush=True)
        if len(got) < k:
            break
    run_s = time.perf_counter() - t_all
    live = e.corpus_size()[1]
    conserved = live == n - sum(m[2] for m in merges)
    nxt = e.find_next_merge(0, 2)
    out = {'merges': len(merges), 'run_s': round(run_s, 1),
           'ms_per_merge': round(run_s * 1e3 / max(1, len(merges)), 4),
           'live_tokens': live, 'tokens_conserved': bool(conserved),
           'merges_sha256': pkg_sha(merges), 'next_merge': list(nxt) if nxt else None}
    print(json.dumps(out), flush=True)
    # the recount from scratch on the host (the checker)
    t2 = time.perf_counter()
    ids, off = e.read_corpus()
    e.close()
    from oracle import CpuMT
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    cpu = CpuMT(ids, off, [1] * 32768, 32768, threads=threads)
    del ids
    want = cpu.find_next_merge(0, 2)
    cpu.close()
    out.update({'recount_next_merge': list(want) if want else None,
                'next_merge_matches_recount': (list(want) if want else None) == out['next_merge'],
                'recount_s': round(time.perf_counter() - t2, 1)})
    print(json.dumps(out), flush=True)


def pkg_sha(merges):
    import hashlib
    return hashlib.sha256(np.asarray(merges, dtype=np.int64).tobytes()).hexdigest()


if __name__ == '__main__':
    main()
