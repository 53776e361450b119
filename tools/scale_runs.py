#!/usr/bin/env python3
"""Scale runs of BASELINE configs 4 and 5 on ONE MI355X (the 4- and 8-GPU scaling runs are the
driver's; these show the per-GPU sizes and the 32k vocabulary work on this engine):

  c5shard  — one GPU's shard of C5: 2 GiB of the C5 stream (256-char alphabet, 1 MiB samples),
             mergeUntil({min_weight: 2}) to the 32k-token vocabulary (32768 - 256 merges);
  c4       — the whole C4 corpus (4 GiB, 16 GiB of int32 slots) on one GPU, 1000 merges;
  c5       — the whole C5 corpus (16 GiB, 64 GiB of int32 slots) on one GPU, 200 merges.

Checks: the first merges against the multi-threaded CPU restatement (oracle/bpe_cpu_mt.cc, pinned
to the reference's fixtures) where host memory allows, token conservation (live tokens fall by
exactly the sum of W), and for c5shard the next merge of the FINAL state recomputed from scratch
by the CPU restatement on the corpus read back from HBM.
Usage: tools/scale_runs.py CONFIG OUT.json"""
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
from oracle import CpuMT   # noqa: E402  (checker only)

CONFIGS = {
    'c5shard': dict(gib=2, merges=32768 - 256, cpu_prefix=3, final_check=True),
    'c4': dict(gib=4, merges=1000, cpu_prefix=3, final_check=False),
    'c5': dict(gib=16, merges=200, cpu_prefix=0, final_check=False),
}


def main():
    name, out_path = sys.argv[1], sys.argv[2]
    cfg = CONFIGS[name]
    n = cfg['gib'] << 30
    t0 = time.perf_counter()
    data = pkg.synth_latin1(n, seed=12345, A=256, base=0)
    t_synth = time.perf_counter() - t0
    e = pkg.Engine(0)
    e.stats_enable(True)
    t0 = time.perf_counter()
    cmap, nt, _ = e.add_latin1(data, sample_bytes=1 << 20)
    t_ingest = time.perf_counter() - t0
    live0 = e.corpus_size()[1]
    rep = {'config': name, 'corpus_bytes': n, 'int32_slots_bytes': 4 * (n + n // (1 << 20)),
           'synth_s': t_synth, 'ingest_s': t_ingest, 'char_count': nt}
    want = None
    if cfg['cpu_prefix']:
        ids = cmap[data]
        off = np.arange(0, n + 1, 1 << 20, dtype=np.int64)
        del data
        cpu = CpuMT(ids, off, [1] * nt, nt, threads=16)
        del ids
        t0 = time.perf_counter()
        want = cpu.merge_until(0, 2, cfg['cpu_prefix'])
        rep['cpu_prefix_s'] = time.perf_counter() - t0
        cpu.close()
    else:
        del data
    t0 = time.perf_counter()
    got = e.merge_until(0, 2, cfg['merges'], cap=cfg['merges'] + 8)
    dt = time.perf_counter() - t0
    live1 = e.corpus_size()[1]
    scans, live = 0, live0
    for m in got:
        scans += live
        live -= m[2]
    st = e.stats()
    rep.update({'merges': len(got), 'seconds': dt, 'ms_per_merge': 1e3 * dt / max(1, len(got)),
                'pair_scans_per_s': scans / dt, 'vocab_after': nt + len(got),
                'live_tokens_before': live0, 'live_tokens_after': live1,
                'tokens_conserved': live1 == live0 - sum(m[2] for m in got),
                'first_merges': [list(m) for m in got[:5]], 'last_merges': [list(m) for m in got[-3:]],
                'stats': st})
    if want is not None:
        rep['prefix_matches_cpu_restatement'] = [list(m) for m in got[:len(want)]] == [list(m) for m in want]
    if cfg['final_check']:
        # the final state, recounted from scratch on the host: its next merge must equal the
        # engine's (counts, ties and run parity of the whole merged corpus)
        ids, off = e.read_corpus()
        t0 = time.perf_counter()
        cpu = CpuMT(ids, off, [1] * (nt + len(got)), nt + len(got), threads=16)
        del ids
        cpu_next = cpu.find_next_merge(0, 2)
        rep['final_cpu_recount_s'] = time.perf_counter() - t0
        gpu_next = e.find_next_merge(0, 2)
        rep['final_next_merge'] = {'gpu': list(gpu_next) if gpu_next else None,
                                   'cpu': list(cpu_next) if cpu_next else None}
        rep['final_state_matches_cpu_recount'] = gpu_next == cpu_next
    ok = rep['tokens_conserved'] and rep.get('prefix_matches_cpu_restatement', True) and \
        rep.get('final_state_matches_cpu_recount', True)
    rep['ok'] = bool(ok)
    with open(out_path, 'w') as f:
        json.dump(rep, f, indent=1)
    print(json.dumps({k: rep[k] for k in ('config', 'merges', 'ms_per_merge', 'pair_scans_per_s',
                                          'vocab_after', 'ok')}), flush=True)
    if not ok:
        sys.exit(1)


if __name__ == '__main__':
    main()
